#!/bin/bash
# round 4, call 30: D* workers per CU with the batch push (16 = default / 20 / 24), same box
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c30
for i in 1 2; do
for w in 16 20 24 12; do
  timeout -k 10 300 python3 bench.py --legs dstar --no-cpu-baseline --steps 1 --warmup 1 --dstar-workers-per-cu $w > gpurun_out/c30/w${w}_$i.json 2> gpurun_out/c30/w${w}_$i.err || { tail -5 gpurun_out/c30/w${w}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c30/w${w}_$i.json').read().strip().splitlines()[-1]); s=d['secondary']; print('dstar workers $w', s['dstar_256']['value'], s['dstar_512']['value'])"
done
done
