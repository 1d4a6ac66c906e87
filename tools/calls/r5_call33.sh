#!/bin/bash
# round 5, call 33: DWA LOCAL kernel (256 agents) issue counters; parity of the current build first
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c33
timeout -k 10 400 python3 -u -m pytest tests/test_dwa_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c33/test.log 2>&1 || { tail -30 gpurun_out/c33/test.log; exit 1; }
tail -1 gpurun_out/c33/test.log
timeout -k 10 500 bash tools/pmc_leg_issue.sh dwa dwa_split_kernel dwa256 --agents 256 --control-steps 20 > gpurun_out/c33/pmc.txt 2>&1 || { tail -20 gpurun_out/c33/pmc.txt; exit 1; }
cat gpurun_out/c33/pmc.txt
