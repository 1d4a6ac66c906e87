#!/bin/bash
# round 6, call 28: D* on grids without border walls (the reference's getNeighbor KeyError) -- the D*
# GPU tests, the reference sessions among them
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c28
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_dstar_gpu.py \
  > gpurun_out/r6c28/pytest.log 2>&1 || { tail -30 gpurun_out/r6c28/pytest.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r6c28/pytest.log | tail -12; tail -1 gpurun_out/r6c28/pytest.log
