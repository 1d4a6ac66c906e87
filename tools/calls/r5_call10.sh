#!/bin/bash
# round 5, call 10: smoke, then the kernel-trace profile of the default bench command (profiles/r5)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c10
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c10/smoke.log 2>&1 || { tail -20 gpurun_out/c10/smoke.log; exit 1; }
tail -1 gpurun_out/c10/smoke.log
ROUND=r5 PASSES=kt timeout -k 10 900 bash tools/profile_round.sh > gpurun_out/c10/prof.log 2>&1 || { tail -20 gpurun_out/c10/prof.log; tail -20 gpurun_out/bench_prof.err; exit 1; }
tail -3 gpurun_out/c10/prof.log; tail -1 gpurun_out/bench_prof.json | cut -c1-600
