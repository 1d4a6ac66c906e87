#!/bin/bash
# A* 2D headline: batches in flight x workers per launch at a fixed residency (same box):
#   bash tools/sweep_residency.sh -> gpurun_out/resid/*.json, one summary line per run
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/resid
mkdir -p $O
run() {  # name, bench args...
  n=$1; shift
  timeout -k 10 200 python3 $R/bench.py --legs none --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']), round(d['ms_per_step']), round(d['detail']['kernel_ms_per_launch']), flush=True)"
}
K=${K:-20}
run w672_s6_r16_k$K --workers 672 --streams 6 --residency 16 --steps $K
run w725_s6_r17_k$K --workers 725 --streams 6 --residency 17 --steps $K
run w768_s6_r18_k$K --workers 768 --streams 6 --residency 18 --steps $K
run w853_s6_r20_k$K --workers 853 --streams 6 --residency 20 --steps $K
run w658_s7_r18_k$K --workers 658 --streams 7 --residency 18 --steps $K
run w585_s7_r16_k$K --workers 585 --streams 7 --residency 16 --steps $K
run w731_s7_r20_k$K --workers 731 --streams 7 --residency 20 --steps $K
echo sweep-done
