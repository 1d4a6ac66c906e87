#!/bin/bash
# round 6 profiles, pass 1: the driver's bench command under rocprofv3 --kernel-trace --stats
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && ROUND=r6 PASSES=kt bash tools/profile_round.sh > gpurun_out/prof_kt_out.txt 2>&1 || { tail -20 gpurun_out/prof_kt_out.txt; exit 1; }
tail -3 gpurun_out/prof_kt_out.txt; cat gpurun_out/prof_summary.log | head -20; tail -1 gpurun_out/bench_prof.json | cut -c1-600
