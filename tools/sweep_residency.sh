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
run p64_k$K --steps $K --prio 64
run p16_k$K --steps $K --prio 16
run p32_k$K --steps $K --prio 32
run p128_k$K --steps $K --prio 128
run p0_k$K --steps $K --prio 0
run p64b_k$K --steps $K --prio 64
echo sweep-done
