#!/bin/bash
# round 5, call 29: DWA phase stamps, LOCAL (256 agents) and k-split (32 agents) after the nibble stencil
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c29
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c29/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c29/dwa_stamps.log; exit 1; }
cat gpurun_out/c29/dwa_stamps.log
