#!/bin/bash
# round 6 profiles, pass 3: the SQ issue pass of the short bench and the MPC leg's MFMA pass
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R && ROUND=r6 PASSES=issue bash tools/profile_round.sh > gpurun_out/prof_issue_out.txt 2>&1 || { tail -20 gpurun_out/prof_issue_out.txt; exit 1; }
tail -3 gpurun_out/prof_issue_out.txt; tail -8 gpurun_out/prof_summary.log | cut -c1-1500
