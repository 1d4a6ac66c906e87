#!/bin/bash
# round 6, call 3: same-process interleaved A/B (tools/ab_headline.py) of the round-5 build vs the
# tiled-cell-state build on the headline launch, then the new build's residency curve
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c3
timeout -k 10 300 python3 tools/ab_headline.py $L/libpmp_hip_base.so $L/libpmp_hip.so $L/libpmp_hip_gtile.so --rounds 4 --reps 2 --batches 5 \
  --out gpurun_out/c3/ab.json > gpurun_out/c3/ab.log 2>&1 || { tail -20 gpurun_out/c3/ab.log; exit 1; }
tail -2 gpurun_out/c3/ab.log
for r in 52 64; do
  timeout -k 10 200 python3 tools/ab_headline.py $L/libpmp_hip.so --rounds 2 --reps 2 --batches 5 --residency $r \
    --workers $((r * 256)) --out gpurun_out/c3/res$r.json > gpurun_out/c3/res$r.log 2>&1 || { tail -20 gpurun_out/c3/res$r.log; exit 1; }
  echo "residency $r: $(tail -1 gpurun_out/c3/res$r.log)"
done
