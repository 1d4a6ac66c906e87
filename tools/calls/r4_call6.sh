#!/bin/bash
# round 4, call 6: the whole -m gpu suite and smoke at the head, then the driver's bench command
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/c6/gputest.log 2>&1 || { tail -40 gpurun_out/c6/gputest.log; exit 1; }
tail -3 gpurun_out/c6/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c6/smoke.log 2>&1 || { tail -20 gpurun_out/c6/smoke.log; exit 1; }
tail -2 gpurun_out/c6/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/c6/bench_detail.json > gpurun_out/c6/bench.json 2> gpurun_out/c6/bench.err || { tail -5 gpurun_out/c6/bench.err; exit 1; }
tail -c 1500 gpurun_out/c6/bench.json
