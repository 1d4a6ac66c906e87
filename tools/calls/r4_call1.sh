#!/bin/bash
# round 4, call 1: parity (A* 2D, tracking) + A/B of the aligned spill vs unaligned + traffic of both
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py tests/test_track_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c1_tests.log 2>&1 || { tail -30 gpurun_out/r4c1_tests.log; exit 1; }
tail -3 gpurun_out/r4c1_tests.log
bash tools/ab_bench.sh libpmp_hip.so libpmp_hip_shift0.so 2 || exit 1
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip.so bash tools/traffic_probe.sh shift1:1:1:4096:32 || exit 1
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_shift0.so bash tools/traffic_probe.sh shift0:1:1:4096:32 || exit 1
