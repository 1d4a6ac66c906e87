#!/bin/bash
# round 4, call 26: the full-size parity tests (all C2 / C5 / C4 queries, the headline schedule, two
# full C3 trees against the oracle)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c26
timeout -k 10 900 python -u -m pytest tests/test_astar2d_gpu.py tests/test_astar3d_gpu.py tests/test_dwa_gpu.py tests/test_rrt_gpu.py -x -v --timeout 300 --timeout-method thread --durations=8 > gpurun_out/c26/tests.log 2>&1 || { tail -40 gpurun_out/c26/tests.log; exit 1; }
tail -14 gpurun_out/c26/tests.log
