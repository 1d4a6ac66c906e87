#!/bin/bash
# round 6, call 40: RRT* at 256 threads x 2 per CU: batches per launch x launches in flight
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c40
for r in 1 2; do
  for bs in 8x2 16x2 8x3 16x1 4x3; do
    b=${bs%x*}; s=${bs#*x}
    timeout -k 10 300 python3 bench.py --legs rrt --steps 4 --warmup 1 --no-cpu-baseline --rrt-batches $b --rrt-streams $s \
      > gpurun_out/r6c40/b_${bs}_$r.out 2> gpurun_out/r6c40/b_${bs}_$r.err || { tail -20 gpurun_out/r6c40/b_${bs}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c40/b_${bs}_$r.out').read().strip().splitlines()[-1]); s=d['secondary']['rrt_star']; print('$bs round $r', s['value'])"
  done
done
