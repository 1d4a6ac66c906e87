#!/bin/bash
# round 6, call 58: the whole GPU suite and smoke() on the round's tree, then the driver's bench command
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c58
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r6c58/gputests.log 2>&1 || { tail -40 gpurun_out/r6c58/gputests.log; exit 1; }
tail -2 gpurun_out/r6c58/gputests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6c58/smoke.log 2>&1 || { tail -20 gpurun_out/r6c58/smoke.log; exit 1; }
tail -1 gpurun_out/r6c58/smoke.log | cut -c1-200
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/r6c58/bench_detail.json > gpurun_out/r6c58/bench.out 2> gpurun_out/r6c58/bench.err || { tail -20 gpurun_out/r6c58/bench.err; exit 1; }
tail -1 gpurun_out/r6c58/bench.out | cut -c1-400
