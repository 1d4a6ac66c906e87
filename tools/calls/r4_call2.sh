#!/bin/bash
# round 4, call 2: keys-beside-entry A/B + parity of it, PMC issue at the headline geometry
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_keys1.so timeout -k 10 300 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 200 --timeout-method thread -k "small_grids or c2_subset or residency" > gpurun_out/r4c2_keys_tests.log 2>&1 || { tail -30 gpurun_out/r4c2_keys_tests.log; exit 1; }
tail -2 gpurun_out/r4c2_keys_tests.log
bash tools/ab_bench.sh libpmp_hip.so libpmp_hip_keys1.so 2 || exit 1
bash tools/pmc_headline_issue.sh head || exit 1
LIB=libpmp_hip_keys1.so bash tools/pmc_headline_issue.sh keys1 || exit 1
