#!/bin/bash
# round 6, call 26: Theta* / Lazy Theta* 2D with a warmup of the timed launch's size (12 batches)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c26
for r in 1 2; do
timeout -k 10 600 python3 bench.py --legs graphs --steps 2 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c26/d$r.json \
  > gpurun_out/r6c26/b$r.out 2> gpurun_out/r6c26/b$r.err || { tail -20 gpurun_out/r6c26/b$r.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r6c26/b$r.out').read().strip().splitlines()[-1])
print({k: v['value'] for k, v in d['secondary'].items()})"
done
