#!/bin/bash
# round 5, final tree: the GPU suite and smoke(), then the kernel-trace profile of the default bench
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/final2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final2/gputest.log 2>&1 || { tail -40 gpurun_out/final2/gputest.log; exit 1; }
tail -1 gpurun_out/final2/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1 || { tail -20 gpurun_out/final2/smoke.log; exit 1; }
tail -1 gpurun_out/final2/smoke.log | cut -c1-120
ROUND=r5 PASSES=kt timeout -k 10 800 bash tools/profile_round.sh > gpurun_out/final2/prof.log 2>&1 || { tail -20 gpurun_out/final2/prof.log; tail -20 gpurun_out/bench_prof.err; exit 1; }
tail -1 gpurun_out/final2/prof.log; tail -1 gpurun_out/bench_prof.json | cut -c1-300
