#!/bin/bash
# round 6, call 9: residency sweep of the new build on the headline launch, two passes interleaved
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c9
for pass in 1 2; do
for r in 44 48 52 56 60; do
  timeout -k 10 200 python3 tools/ab_headline.py $L/libpmp_hip.so --rounds 1 --reps 2 --residency $r --workers $((r * 256)) \
    > gpurun_out/c9/res${r}_$pass.log 2>&1 || { tail -5 gpurun_out/c9/res${r}_$pass.log; exit 1; }
  echo "pass $pass residency $r: $(tail -1 gpurun_out/c9/res${r}_$pass.log)"
done
done
