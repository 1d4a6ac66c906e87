#!/bin/bash
# round 6, call 55: the D* legs' line carries its first pass's PMC traffic (workload:kernel key)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c55
timeout -k 10 300 python3 bench.py --legs dstar --steps 1 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c55/d.json \
  > gpurun_out/r6c55/b.out 2> gpurun_out/r6c55/b.err || { tail -20 gpurun_out/r6c55/b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r6c55/d.json'))
for k in ('dstar_256','dstar_512'):
    v=d['secondary'][k]
    print(k, v['value'], v['roofline'].get('traffic'), v['roofline'].get('traffic_source'))
"
