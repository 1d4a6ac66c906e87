#!/bin/bash
# round 5, call 19: choice bits from lane masks (PMP_MQ_CBMASK=1, default) vs per-lane selects
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c19
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c19/$n.json "$@" \
    > gpurun_out/c19/$n.out 2> gpurun_out/c19/$n.err || { tail -20 gpurun_out/c19/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c19/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py tests/test_graph_variants_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c19/tests.log 2>&1 || { tail -30 gpurun_out/c19/tests.log; exit 1; }
tail -1 gpurun_out/c19/tests.log
for i in 1 2 3; do
  head1 def_$i $L/libpmp_hip.so && head1 cb0_$i $L/libpmp_hip_cb0.so || exit 1
done
