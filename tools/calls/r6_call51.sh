#!/bin/bash
# round 6, call 51: D* tests at the split kernels, then the kernel-trace profile of the driver's bench
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c51
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_dstar_gpu.py \
  > gpurun_out/r6c51/pytest.log 2>&1 || { tail -30 gpurun_out/r6c51/pytest.log; exit 1; }
tail -1 gpurun_out/r6c51/pytest.log
bash tools/calls/r6_prof_kt.sh
