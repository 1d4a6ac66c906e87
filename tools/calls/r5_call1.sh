#!/bin/bash
# round 5, call 1: the GPU suite (Theta* on the multi-query engine, RRT* coarse tree in LDS, DWA
# k-split, LPA* U past the LDS share, LPAStar3D written-this-query bits, geometry restore), then
# short bench legs for the changed kernels and the MPC tolerance probe
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c1/gpu_tests.log 2>&1 || { tail -60 gpurun_out/c1/gpu_tests.log; exit 1; }
tail -3 gpurun_out/c1/gpu_tests.log
leg() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/c1/$n.json "$@" \
    > gpurun_out/c1/$n.out 2> gpurun_out/c1/$n.err || { tail -20 gpurun_out/c1/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c1/$n.json'))['secondary']
for k, v in d.items(): print('$n', k, round(v['value']), v.get('unit'), 'kernel_ms', v.get('kernel_ms_per_launch'), 'frac', v.get('roofline', {}).get('frac'), 'checked', v.get('timed_launches_checked'))"
}
# the A* headline: lane-constant spill offsets (default) vs the round-4 offsets (lc0) vs the half-block
# layout (blk2), alternating, same box
for i in 1 2; do
  for v in default lc0 blk2; do
    lib=$R/python_motion_planning_amd/libpmp_hip.so
    [ "$v" = default ] || lib=$R/python_motion_planning_amd/libpmp_hip_$v.so
    PMP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c1/head_$v.json \
      > gpurun_out/c1/head_${v}_$i.out 2> gpurun_out/c1/head_${v}_$i.err || { tail -20 gpurun_out/c1/head_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c1/head_${v}_$i.out').read().strip().splitlines()[-1]); print('headline $v', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
  done
done
leg dwa32 --legs dwa --agents 32 --control-steps 50
leg dwa256 --legs dwa --control-steps 50
leg rrt --legs rrt --rrt-steps 3
leg dyn3d --legs dyn3d
for r in 24 32 40; do leg theta_r$r --legs graphs --theta-residency $r; done
leg theta_e0 --legs graphs --theta-engine 0
timeout -k 10 200 python3 tools/mpc_tol.py > gpurun_out/c1/mpc_tol.log 2>&1 || { tail -20 gpurun_out/c1/mpc_tol.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c1/mpc_tol.log
