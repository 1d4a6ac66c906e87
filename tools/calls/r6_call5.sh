#!/bin/bash
# round 6, call 5: RRT* grid index -- parity (every RRT test), then the C3 leg, round-5 build vs new
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest tests/test_rrt_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/c5/tests.log 2>&1 || { tail -30 gpurun_out/c5/tests.log; exit 1; }
tail -1 gpurun_out/c5/tests.log
for n in base new; do
  lib=$L/libpmp_hip.so; [ $n = base ] && lib=$L/libpmp_hip_base.so
  PMP_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --legs rrt --steps 2 --warmup 1 --no-cpu-baseline \
    --detail-out gpurun_out/c5/$n.json > gpurun_out/c5/$n.out 2> gpurun_out/c5/$n.err || { tail -20 gpurun_out/c5/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c5/$n.json')); r=d['secondary']['rrt_star']
print('$n', 'rrt', r['value'], 'kernel_ms', r.get('kernel_ms_per_launch'), 'detail', json.dumps(r.get('detail')))"
done
