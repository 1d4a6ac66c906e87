#!/bin/bash
# round 4, call 3: the unified-step mq kernel (parity, A/B, PMC); LPA* / D* Lite with U in LDS (parity, traffic)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_uni.so timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py tests/test_graph_variants_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c3_uni_tests.log 2>&1 || { tail -40 gpurun_out/r4c3_uni_tests.log; exit 1; }
tail -2 gpurun_out/r4c3_uni_tests.log
bash tools/ab_bench.sh libpmp_hip.so libpmp_hip_uni.so 2 || exit 1
bash tools/lpa_traffic.sh || exit 1
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_lpaold.so bash tools/lpa_traffic.sh || exit 1
LIB=libpmp_hip_uni.so bash tools/pmc_headline_issue.sh uni || exit 1
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_pm3.so timeout -k 10 300 python -u -m pytest tests/test_astar3d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4c3_pm3_tests.log 2>&1 || { tail -30 gpurun_out/r4c3_pm3_tests.log; exit 1; }
tail -2 gpurun_out/r4c3_pm3_tests.log
bash tools/ab_leg.sh astar3d astar3d libpmp_hip.so libpmp_hip_pm3.so 2 || exit 1
