#!/bin/bash
# round 4, call 7: 3D A* front (A/B, parity), headline residency / priority fine sweep
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c7
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_front4.so timeout -k 10 400 python -u -m pytest tests/test_astar3d_gpu.py tests/test_graph_variants_gpu.py -x -q --timeout 200 --timeout-method thread -k "3d or 3D or csv" > gpurun_out/c7/front4_tests.log 2>&1 || { tail -30 gpurun_out/c7/front4_tests.log; exit 1; }
tail -2 gpurun_out/c7/front4_tests.log
for L in libpmp_hip.so libpmp_hip_front.so libpmp_hip_front4.so; do
  bash tools/ab_leg.sh astar3d astar3d $L $L 1 || exit 1
done
for cfg in "52 13312 64" "60 15360 64" "56 14336 0" "56 14336 256"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --residency $1 --workers $2 --prio $3 > gpurun_out/c7/h_$1_$3.json 2> gpurun_out/c7/h_$1_$3.err || { tail -5 gpurun_out/c7/h_$1_$3.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c7/h_$1_$3.json').read().strip().splitlines()[-1]); print('residency $1 prio $3', round(d['value']), round(d['ms_per_step']))"
done
