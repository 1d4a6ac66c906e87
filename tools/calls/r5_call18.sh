#!/bin/bash
# round 5, call 18: path_op's level shift by ds_bpermute (PMP_MQ_BPERM=1) vs the two DPP shifts
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c18
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c18/$n.json "$@" \
    > gpurun_out/c18/$n.out 2> gpurun_out/c18/$n.err || { tail -20 gpurun_out/c18/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c18/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
PMP_HIP_LIB=$L/libpmp_hip_bperm.so timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c18/tests.log 2>&1 || { tail -30 gpurun_out/c18/tests.log; exit 1; }
tail -1 gpurun_out/c18/tests.log
for i in 1 2 3; do
  head1 def_$i $L/libpmp_hip.so && head1 bperm_$i $L/libpmp_hip_bperm.so || exit 1
done
