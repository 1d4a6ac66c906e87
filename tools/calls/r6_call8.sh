#!/bin/bash
# round 6, call 8: the new build's residency curve (56 / 60 / 64 per CU) and priority count, and the
# DPP level shift (PMP_MQ_BPERM=0) against the bpermute one, on the headline launch
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c8
for r in 56 64; do
  timeout -k 10 200 python3 tools/ab_headline.py $L/libpmp_hip.so --rounds 1 --reps 2 --residency $r --workers $((r * 256)) \
    > gpurun_out/c8/res$r.log 2>&1 || { tail -5 gpurun_out/c8/res$r.log; exit 1; }
  echo "residency $r: $(tail -1 gpurun_out/c8/res$r.log)"
done
timeout -k 10 200 python3 tools/ab_headline.py $L/libpmp_hip.so --rounds 1 --reps 2 --prio 0 > gpurun_out/c8/prio0.log 2>&1 || exit 1
echo "prio 0: $(tail -1 gpurun_out/c8/prio0.log)"
timeout -k 10 300 python3 tools/ab_headline.py $L/libpmp_hip.so $L/libpmp_hip_dpp.so --rounds 2 --reps 2 > gpurun_out/c8/dpp.log 2>&1 || exit 1
tail -2 gpurun_out/c8/dpp.log
