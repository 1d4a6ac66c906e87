#!/bin/bash
# round 5, final tree after the DWA work (repeat): the bench's default command (as the driver runs it)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/final5
timeout -k 10 900 python3 bench.py --detail-out gpurun_out/final5/bench_detail.json > gpurun_out/final5/bench.jsonl 2> gpurun_out/final5/bench.err || { tail -30 gpurun_out/final5/bench.err; exit 1; }
tail -1 gpurun_out/final5/bench.jsonl | cut -c1-300
