#!/bin/bash
# round 6, call 2: tiled (8 x 16) per-slot cell states + lane-mask state on the multi-query and
# single-query engines -- parity (A* 2D, graph variants), then same-box A/B vs the round-5 build
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c2
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c2/$n.json "$@" \
    > gpurun_out/c2/$n.out 2> gpurun_out/c2/$n.err || { tail -20 gpurun_out/c2/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c2/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
timeout -k 10 600 python -u -m pytest tests/test_astar2d_gpu.py tests/test_graph_variants_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c2/tests.log 2>&1 || { tail -30 gpurun_out/c2/tests.log; exit 1; }
tail -1 gpurun_out/c2/tests.log
for i in 1 2; do
  head1 base_$i $L/libpmp_hip_base.so && head1 new_$i $L/libpmp_hip.so || exit 1
done
