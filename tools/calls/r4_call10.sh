#!/bin/bash
# round 4, call 10: two-level block spill layout (parity, A/B, traffic); the select-form step (A/B vs base)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c10
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_blk.so timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c10/blk_tests.log 2>&1 || { tail -30 gpurun_out/c10/blk_tests.log; exit 1; }
tail -2 gpurun_out/c10/blk_tests.log
for i in 1 2; do
  for L in libpmp_hip_base.so libpmp_hip.so libpmp_hip_blk.so; do
    n=$(basename $L .so)
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline > gpurun_out/c10/${n}_$i.json 2> gpurun_out/c10/${n}_$i.err || { tail -5 gpurun_out/c10/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/c10/${n}_$i.json').read().strip().splitlines()[-1]); print('$n', round(d['value']), round(d['ms_per_step']))"
  done
done
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip.so bash tools/traffic_probe.sh pos:1:1:14336:56 || exit 1
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_blk.so bash tools/traffic_probe.sh blk:1:1:14336:56 || exit 1
