#!/bin/bash
# round 6, call 13: push pairs -- multi-query parity (headline schedule, graph variants) then an
# in-process A/B against the same tree built without pairs
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c13
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_astar2d_gpu.py tests/test_graph_variants_gpu.py \
  > gpurun_out/r6c13/pytest.log 2>&1 || { tail -30 gpurun_out/r6c13/pytest.log; exit 1; }
tail -3 gpurun_out/r6c13/pytest.log
timeout -k 10 500 python3 tools/ab_headline.py $L/libpmp_hip.so $L/libpmp_hip_nopair.so --rounds 2 --reps 2 \
  --out gpurun_out/r6c13/ab.json > gpurun_out/r6c13/ab.log 2>&1 || { tail -20 gpurun_out/r6c13/ab.log; exit 1; }
tail -3 gpurun_out/r6c13/ab.log
