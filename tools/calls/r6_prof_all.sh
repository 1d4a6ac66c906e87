#!/bin/bash
# round 6 profiles, the three passes in one call: kernel trace of the driver's bench, FETCH / WRITE,
# SQ issue + MFMA (tools/profile_round.sh PASSES=kt|pmc|issue); the kt pass's files are kept aside
# before the later passes re-summarise
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && mkdir -p gpurun_out/prof_final
ROUND=r6 PASSES=kt bash tools/profile_round.sh > gpurun_out/prof_kt_out.txt 2>&1 || { tail -20 gpurun_out/prof_kt_out.txt; exit 1; }
cp gpurun_out/profiles_r6/kernel_stats*.csv gpurun_out/profiles_r6/astar2d_dispatches.csv gpurun_out/bench_prof.json gpurun_out/prof_final/
cp gpurun_out/prof_kt/detail.json gpurun_out/prof_final/bench_kt_detail_manifest.json
grep "not attributed" gpurun_out/prof_summary.log && exit 1
ROUND=r6 PASSES=pmc bash tools/profile_round.sh > gpurun_out/prof_pmc_out.txt 2>&1 || { tail -20 gpurun_out/prof_pmc_out.txt; exit 1; }
cp gpurun_out/profiles_r6/pmc_traffic.json gpurun_out/prof_final/
ROUND=r6 PASSES=issue bash tools/profile_round.sh > gpurun_out/prof_issue_out.txt 2>&1 || { tail -20 gpurun_out/prof_issue_out.txt; exit 1; }
cp gpurun_out/profiles_r6/pmc_issue.json gpurun_out/profiles_r6/pmc_mfma.json gpurun_out/prof_final/
tail -1 gpurun_out/prof_final/bench_prof.json | cut -c1-200
echo all-profiles-done
