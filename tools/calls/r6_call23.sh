#!/bin/bash
# round 6, call 23: single-query engine with the 3x3 round pipelined one pop ahead -- A* 2D parity on
# every engine (+ drop-in / graph-variant tests), then the drop-in latency leg against the round-5 engine
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c23
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_astar2d_gpu.py tests/test_graph_variants_gpu.py tests/test_integration_stub.py \
  > gpurun_out/r6c23/pytest.log 2>&1 || { tail -30 gpurun_out/r6c23/pytest.log; exit 1; }
tail -1 gpurun_out/r6c23/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_sqold.so; else unset PMP_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --legs latency --steps 1 --warmup 1 --no-cpu-baseline --detail-out gpurun_out/r6c23/d_$v$r.json \
      > gpurun_out/r6c23/b_$v$r.out 2> gpurun_out/r6c23/b_$v$r.err || { tail -20 gpurun_out/r6c23/b_$v$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c23/b_$v$r.out').read().strip().splitlines()[-1])
print('$v round $r', {k: v for k, v in d['secondary'].items() if 'lat' in k or 'dropin' in k})
"
  done
done
