#!/bin/bash
# round 5, call 12: RRT* with the steer test inside the radius scan's pass (parity, stamps, bench leg)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c12
timeout -k 10 500 python -u -m pytest tests/test_rrt_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c12/tests.log 2>&1 || { tail -40 gpurun_out/c12/tests.log; exit 1; }
tail -1 gpurun_out/c12/tests.log
PMP_HIP_LIB=$L/libpmp_hip_rrtstamps.so timeout -k 10 200 python3 tools/rrt_time.py 4x16384 256x8192 > gpurun_out/c12/rrtstamps.log 2>&1 || { tail -20 gpurun_out/c12/rrtstamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c12/rrtstamps.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --legs rrt --detail-out gpurun_out/c12/rrt.json > gpurun_out/c12/rrt.out 2> gpurun_out/c12/rrt.err || { tail -20 gpurun_out/c12/rrt.err; exit 1; }
python3 -c "
import json; v=json.load(open('gpurun_out/c12/rrt.json'))['secondary']['rrt_star']; print('rrt', round(v['value']), 'kernel_ms', round(v['kernel_ms_per_launch'], 1))"
