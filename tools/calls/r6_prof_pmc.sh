#!/bin/bash
# round 6 profiles, pass 2: FETCH_SIZE / WRITE_SIZE passes of the short bench (per-workload traffic)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && ROUND=r6 PASSES=pmc bash tools/profile_round.sh > gpurun_out/prof_pmc_out.txt 2>&1 || { tail -20 gpurun_out/prof_pmc_out.txt; exit 1; }
tail -3 gpurun_out/prof_pmc_out.txt; tail -8 gpurun_out/prof_summary.log | cut -c1-1500
