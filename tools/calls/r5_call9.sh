#!/bin/bash
# round 5, call 9: the half-block spill layout as the default (A* 2D parity on every engine, headline
# vs the round-4 layout), LPAStar3D with unconditional U loads (parity, probe, dyn3d leg)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c9
timeout -k 10 600 python -u -m pytest tests/test_astar2d_gpu.py tests/test_lpastar3d_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c9/tests.log 2>&1 || { tail -40 gpurun_out/c9/tests.log; exit 1; }
tail -1 gpurun_out/c9/tests.log
timeout -k 10 300 python3 tools/lpa3d_probe.py 16 > gpurun_out/c9/lpa3d.log 2>&1 || { tail -20 gpurun_out/c9/lpa3d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c9/lpa3d.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --legs dyn3d --detail-out gpurun_out/c9/dyn3d.json > gpurun_out/c9/dyn3d.out 2>&1 || { tail -20 gpurun_out/c9/dyn3d.out; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/c9/dyn3d.json'))['secondary']
for k, v in d.items(): print(k, round(v['value']), 'kernel_ms', round(v['kernel_ms_per_launch'], 1))"
for i in 1 2; do
  for v in default blk1; do
    lib=$L/libpmp_hip.so
    [ "$v" = default ] || lib=$L/libpmp_hip_$v.so
    PMP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c9/head_$v.json \
      > gpurun_out/c9/head_${v}_$i.out 2> gpurun_out/c9/head_${v}_$i.err || { tail -20 gpurun_out/c9/head_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c9/head_${v}_$i.out').read().strip().splitlines()[-1]); print('headline $v', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
  done
done
