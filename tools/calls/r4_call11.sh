#!/bin/bash
# round 4, call 11: residency / tier-2 placement sweep of the block spill layout (headline, --legs none)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c11
for spec in 56:1 64:1 48:1 64:0 56:0 60:1; do
  IFS=: read res t2 <<< "$spec"
  timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --residency $res --workers $((256*res)) --t2lds $t2 \
    > gpurun_out/c11/r${res}_t$t2.json 2> gpurun_out/c11/r${res}_t$t2.err || { tail -5 gpurun_out/c11/r${res}_t$t2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c11/r${res}_t$t2.json').read().strip().splitlines()[-1]); print('res $res t2 $t2', round(d['value']), round(d['ms_per_step']))"
done
timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c11/tests.log 2>&1 || { tail -30 gpurun_out/c11/tests.log; exit 1; }
tail -2 gpurun_out/c11/tests.log
# lone-query latency: engine 0 (one query per wave) vs engine 2 (lone: group 0 of a wave with its whole LDS)
for m in c1 c2med; do
  for e in 0 2; do
    MODE=$m ENGINE=$e RESIDENCY=$([ $e = 2 ] && echo 4 || echo 0) REPS=3 timeout -k 10 120 python3 tools/astar2d_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
