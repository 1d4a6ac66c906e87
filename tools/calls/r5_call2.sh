#!/bin/bash
# round 5, call 2: parity of the changed kernels, then A/B and legs: the A* headline with the
# lane-constant spill offsets (default, fixed: no load for store-only lanes) vs round 4's (lc0), three
# alternating rounds; the DWA split probe; RRT* with split LDS / HBM scans; LPAStar3D; Theta* mq twice
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c2
timeout -k 10 500 python -u -m pytest tests/test_dwa_gpu.py tests/test_rrt_gpu.py tests/test_lpastar3d_gpu.py tests/test_astar2d_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c2/tests.log 2>&1 || { tail -60 gpurun_out/c2/tests.log; exit 1; }
tail -2 gpurun_out/c2/tests.log
for i in 1 2 3; do
  for v in default lc0; do
    lib=$R/python_motion_planning_amd/libpmp_hip.so
    [ "$v" = default ] || lib=$R/python_motion_planning_amd/libpmp_hip_$v.so
    PMP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c2/head_$v.json \
      > gpurun_out/c2/head_${v}_$i.out 2> gpurun_out/c2/head_${v}_$i.err || { tail -20 gpurun_out/c2/head_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c2/head_${v}_$i.out').read().strip().splitlines()[-1]); print('headline $v', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
  done
done
timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c2/dwa_probe.log 2>&1 || { tail -20 gpurun_out/c2/dwa_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c2/dwa_probe.log
leg() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/c2/$n.json "$@" \
    > gpurun_out/c2/$n.out 2> gpurun_out/c2/$n.err || { tail -20 gpurun_out/c2/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c2/$n.json'))['secondary']
for k, v in d.items(): print('$n', k, round(v['value']), v.get('unit'), 'kernel_ms', round(v.get('kernel_ms_per_launch') or 0, 2), 'frac', v.get('roofline', {}).get('frac'))"
}
leg rrt --legs rrt --rrt-steps 3
leg dyn3d --legs dyn3d
for i in 1 2; do for r in 24 32; do leg theta_r${r}_$i --legs graphs --theta-residency $r --lpa-queries 256; done; done
