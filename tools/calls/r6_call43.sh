#!/bin/bash
# round 6, call 43: Theta* / Lazy Theta* with G and Pc in 4 x 4 tiles (A* row-major again) -- graph
# tests, legs and FETCH / WRITE per Theta* dispatch, against the row-major build
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c43
timeout -k 10 600 python -u -m pytest tests/test_graph_variants_gpu.py tests/test_astar2d_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r6c43/gputests.log 2>&1 || { tail -40 gpurun_out/r6c43/gputests.log; exit 1; }
tail -1 gpurun_out/r6c43/gputests.log
cd /tmp && export TMPDIR=/tmp
for v in new gold; do
  if [ $v = gold ]; then export PMP_HIP_LIB=$L/libpmp_hip_gold.so; else unset PMP_HIP_LIB; fi
  timeout -k 10 600 python3 $R/bench.py --legs graphs --steps 2 --warmup 1 --no-cpu-baseline \
    > $R/gpurun_out/r6c43/b_$v.out 2> $R/gpurun_out/r6c43/b_$v.err || { tail -20 $R/gpurun_out/r6c43/b_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/r6c43/b_$v.out').read().strip().splitlines()[-1])
print('$v', {k: v['value'] for k, v in d['secondary'].items() if 'theta' in k})"
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 400 rocprofv3 --pmc $c -d /tmp/p_${v}_$c -o run -- python3 $R/bench.py --legs graphs --steps 1 --warmup 1 --no-cpu-baseline --graph-steps 1 \
      > /tmp/p_${v}_$c.out 2> /tmp/p_${v}_$c.err || { tail -20 /tmp/p_${v}_$c.err; exit 1; }
    for k in ", 1>" ", 2>"; do echo "$v $c theta$k: $(python3 $R/tools/pmc_sum.py /tmp/p_${v}_$c "$k" | tr -s ' ')"; done
  done
done
