#!/bin/bash
# round 4, call 27: the drop-in overflow fallback test
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c27
timeout -k 10 400 python -u -m pytest tests/test_astar2d_gpu.py -x -v --timeout 300 --timeout-method thread -k "dropin" --durations=4 > gpurun_out/c27/tests.log 2>&1 || { tail -40 gpurun_out/c27/tests.log; exit 1; }
tail -10 gpurun_out/c27/tests.log
