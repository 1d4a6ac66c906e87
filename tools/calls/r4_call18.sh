#!/bin/bash
# round 4, call 18: the round profile's PMC passes (FETCH_SIZE, WRITE_SIZE, MFMA), then the issue
# breakdowns of the headline kernel and of the single-query engine on the README query
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
ROUND=r4 PASSES=pmc bash tools/profile_round.sh || exit 1
bash tools/pmc_headline_issue.sh head_r4 > gpurun_out/pmc_issue_head_r4.txt 2>&1 || { tail -5 gpurun_out/pmc_issue_head_r4.txt; exit 1; }
cat gpurun_out/pmc_issue_head_r4.txt
MODE=c1 ENGINE=3 KERN=sq W_=1 RES=0 bash tools/pmc_headline_issue.sh sq_c1 > gpurun_out/pmc_issue_sq_c1.txt 2>&1 || { tail -5 gpurun_out/pmc_issue_sq_c1.txt; exit 1; }
cat gpurun_out/pmc_issue_sq_c1.txt
find gpurun_out/pmc_issue_* -name "*.db" -delete
