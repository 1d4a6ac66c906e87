#!/bin/bash
# round 5, final rehearsal of the driver's round-end sequence on the final tree: the GPU suite, smoke(),
# the bench's default command
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputest.log 2>&1 || { tail -40 gpurun_out/final/gputest.log; exit 1; }
tail -1 gpurun_out/final/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out gpurun_out/final/bench_detail.json > gpurun_out/final/bench.jsonl 2> gpurun_out/final/bench.err || { tail -30 gpurun_out/final/bench.err; exit 1; }
tail -1 gpurun_out/final/bench.jsonl | cut -c1-400
