#!/bin/bash
# round 6, call 1: A* 2D headline VALU cuts (lane-mask predicates, sqrt_int_rn, mov_dpp, ctz walk) --
# parity on the multi-query engine, then same-box A/B: r5 build / new default / new + position-order spill
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c1
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c1/$n.json "$@" \
    > gpurun_out/c1/$n.out 2> gpurun_out/c1/$n.err || { tail -20 gpurun_out/c1/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c1/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c1/tests.log 2>&1 || { tail -30 gpurun_out/c1/tests.log; exit 1; }
tail -1 gpurun_out/c1/tests.log
PMP_HIP_LIB=$L/libpmp_hip_blk0.so timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 300 --timeout-method thread -k "mq or engine" > gpurun_out/c1/tests_blk0.log 2>&1 || { tail -30 gpurun_out/c1/tests_blk0.log; exit 1; }
tail -1 gpurun_out/c1/tests_blk0.log
for i in 1 2; do
  head1 base_$i $L/libpmp_hip_base.so && head1 new_$i $L/libpmp_hip.so && head1 blk0_$i $L/libpmp_hip_blk0.so || exit 1
done
