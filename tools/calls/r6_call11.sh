#!/bin/bash
# round 6, call 11: cell-state tile shapes on the headline launch (8x16 default, 16x8, 8x8, 4x32)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c11
timeout -k 10 600 python3 tools/ab_headline.py $L/libpmp_hip.so $L/libpmp_hip_t16x8.so $L/libpmp_hip_t8x8.so $L/libpmp_hip_t4x32.so \
  --rounds 2 --reps 2 --out gpurun_out/c11/ab.json > gpurun_out/c11/ab.log 2>&1 || { tail -20 gpurun_out/c11/ab.log; exit 1; }
tail -4 gpurun_out/c11/ab.log
