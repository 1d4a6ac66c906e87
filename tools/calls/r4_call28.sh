#!/bin/bash
# round 4, call 28: headline raised-priority count (longest queries at s_setprio 3) at 60 per CU
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c28
for i in 1 2; do
for p in 64 0 256 1024; do
  timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --prio $p > gpurun_out/c28/p${p}_$i.json 2> gpurun_out/c28/p${p}_$i.err || { tail -5 gpurun_out/c28/p${p}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c28/p${p}_$i.json').read().strip().splitlines()[-1]); print('prio $p', round(d['value']), round(d['ms_per_step']))"
done
done
