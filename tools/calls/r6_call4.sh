#!/bin/bash
# round 6, call 4: interleaved A/B on the headline's own launch (20 batches, 5-batch warmup as the
# driver's --warmup 5): round-5 build vs the tiled-cell-state build
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c4
timeout -k 10 400 python3 tools/ab_headline.py $L/libpmp_hip_base.so $L/libpmp_hip.so --rounds 2 --reps 2 \
  --out gpurun_out/c4/ab.json > gpurun_out/c4/ab.log 2>&1 || { tail -20 gpurun_out/c4/ab.log; exit 1; }
cat gpurun_out/c4/ab.log | grep -v amdgpu.ids
