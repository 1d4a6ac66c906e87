#!/bin/bash
# round 6, call 42: per-slot G (and Theta*'s Pc) in 4 x 4 tiles on the multi-query engine -- the whole
# GPU suite, the headline A/B against the row-major build (same process), Theta* / Lazy Theta* legs
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c42
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r6c42/gputests.log 2>&1 || { tail -40 gpurun_out/r6c42/gputests.log; exit 1; }
tail -1 gpurun_out/r6c42/gputests.log
timeout -k 10 400 python3 tools/ab_headline.py $L/libpmp_hip.so $L/libpmp_hip_gold.so --rounds 2 --reps 2 > gpurun_out/r6c42/ab.log 2>&1 || { tail -10 gpurun_out/r6c42/ab.log; exit 1; }
tail -4 gpurun_out/r6c42/ab.log
for v in new gold; do
  if [ $v = gold ]; then export PMP_HIP_LIB=$L/libpmp_hip_gold.so; else unset PMP_HIP_LIB; fi
  timeout -k 10 600 python3 bench.py --legs graphs --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c42/d_$v.json \
    > gpurun_out/r6c42/b_$v.out 2> gpurun_out/r6c42/b_$v.err || { tail -20 gpurun_out/r6c42/b_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r6c42/b_$v.out').read().strip().splitlines()[-1])
print('$v', {k: v['value'] for k, v in d['secondary'].items()})"
done
