#!/bin/bash
# round 5, call 36: Theta* legs with and without the DWA leg before them (final-bench Theta* 14.4k vs 18.0k)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c36
leg() {
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --detail-out gpurun_out/c36/$n.json "$@" > gpurun_out/c36/$n.out 2> gpurun_out/c36/$n.err || { tail -20 gpurun_out/c36/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c36/$n.json'))['secondary']
print('$n', {k: round(v['value']) for k, v in d.items()})"
}
leg graphs --legs graphs && leg dwa_graphs --legs dwa,graphs && leg graphs2 --legs graphs
