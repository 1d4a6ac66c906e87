#!/bin/bash
# round 6, call 17: the s_memtime rate (the stamps' clock), then the whole GPU suite and smoke() on the
# tree with LPAStar3D's deferred removes
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c17
timeout -k 10 60 ./tools/memtime_rate || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r6c17/gputests.log 2>&1 || { tail -40 gpurun_out/r6c17/gputests.log; exit 1; }
tail -2 gpurun_out/r6c17/gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c17/smoke.log 2>&1 || { tail -20 gpurun_out/r6c17/smoke.log; exit 1; }
tail -2 gpurun_out/r6c17/smoke.log
