#!/bin/bash
# round 5, call 15: Theta* legs on fresh contexts vs on the headline's context (--theta-share-ctx)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c15
theta() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --legs graphs --no-cpu-baseline --detail-out gpurun_out/c15/$n.json "$@" \
    > gpurun_out/c15/$n.out 2> gpurun_out/c15/$n.err || { tail -20 gpurun_out/c15/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c15/$n.json'))['secondary']
for k in ('theta_star_2d', 'lazy_theta_star_2d'): print('$n', k, round(d[k]['value']), 'kernel_ms', round(d[k]['kernel_ms_per_launch']))"
}
for i in 1 2 3; do
  theta fresh_$i && theta shared_$i --theta-share-ctx 1 || exit 1
done
