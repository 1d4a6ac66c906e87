#!/bin/bash
# round 4, call 16: the full GPU suite, smoke() and the driver's bench command at the head
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/c16
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/c16/gputest.log 2>&1 || { tail -40 gpurun_out/c16/gputest.log; exit 1; }
tail -2 gpurun_out/c16/gputest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c16/smoke.log 2>&1 || { tail -20 gpurun_out/c16/smoke.log; exit 1; }
tail -1 gpurun_out/c16/smoke.log
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c16/bench.jsonl 2> gpurun_out/c16/bench.err || { tail -20 gpurun_out/c16/bench.err; exit 1; }
tail -c 600 gpurun_out/c16/bench.jsonl
