#!/bin/bash
# round 5, call 20: RRT* at a 128-VGPR cap (amdgpu_waves_per_eu(4), two 512-thread workgroups per CU
# with the LDS share for two) vs the default
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c20
leg() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --legs rrt --detail-out gpurun_out/c20/$n.json "$@" > gpurun_out/c20/$n.out 2> gpurun_out/c20/$n.err || { tail -20 gpurun_out/c20/$n.err; return 1; }
  python3 -c "
import json; v=json.load(open('gpurun_out/c20/$n.json'))['secondary']['rrt_star']; print('$n', round(v['value']), 'kernel_ms', round(v['kernel_ms_per_launch'], 1))"
}
PMP_HIP_LIB=$L/libpmp_hip_rrtw4.so timeout -k 10 400 python -u -m pytest tests/test_rrt_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c20/tests.log 2>&1 || { tail -30 gpurun_out/c20/tests.log; exit 1; }
tail -1 gpurun_out/c20/tests.log
leg def $L/libpmp_hip.so && leg w4_r2 $L/libpmp_hip_rrtw4.so --rrt-resident 2 && leg w4_r2_s4 $L/libpmp_hip_rrtw4.so --rrt-resident 2 --rrt-streams 4
