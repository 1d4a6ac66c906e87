#!/bin/bash
# round 5, call 16: the headline at 56 / 60 / 64 per CU (half-block layout, lane constants)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c16
head1() {  # name args...
  local n=$1; shift
  timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c16/$n.json "$@" \
    > gpurun_out/c16/$n.out 2> gpurun_out/c16/$n.err || { tail -20 gpurun_out/c16/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c16/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
for i in 1 2; do
  head1 r60_$i && head1 r64_$i --residency 64 && head1 r56_$i --residency 56 || exit 1
done
