#!/bin/bash
# round 4, call 12: residency 56 vs 60 vs 64 per CU on the block spill layout, alternating, same box
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c12
for i in 1 2 3; do
for res in 56 60 64; do
  timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --residency $res --workers $((256*res)) \
    > gpurun_out/c12/r${res}_$i.json 2> gpurun_out/c12/r${res}_$i.err || { tail -5 gpurun_out/c12/r${res}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c12/r${res}_$i.json').read().strip().splitlines()[-1]); print('res $res', round(d['value']), round(d['ms_per_step']), d['kernel_ms_per_launch'] if 'kernel_ms_per_launch' in d else '')"
done
done
# the single-query engine (astar2d_sq.hip): parity, then lone-query latency vs engine 0
timeout -k 10 500 python -u -m pytest tests/test_astar2d_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/c12/tests.log 2>&1 || { tail -40 gpurun_out/c12/tests.log; exit 1; }
tail -3 gpurun_out/c12/tests.log
for m in c1 c2med; do
  for e in 0 3; do
    MODE=$m ENGINE=$e REPS=3 timeout -k 10 120 python3 tools/astar2d_probe.py > gpurun_out/c12/probe_${m}_$e.log 2>&1 || { tail -20 gpurun_out/c12/probe_${m}_$e.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/c12/probe_${m}_$e.log
  done
done
