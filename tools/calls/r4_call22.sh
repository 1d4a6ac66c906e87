#!/bin/bash
# round 4, call 22 (final head): the round profile's PMC passes and the issue breakdowns
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
ROUND=r4 PASSES=pmc bash tools/profile_round.sh || exit 1
bash tools/pmc_headline_issue.sh head_r4 > gpurun_out/pmc_issue_head_r4.txt 2>&1 || { tail -5 gpurun_out/pmc_issue_head_r4.txt; exit 1; }
tail -17 gpurun_out/pmc_issue_head_r4.txt | head -3
MODE=c1 ENGINE=3 KERN=sq W_=1 RES=0 bash tools/pmc_headline_issue.sh sq_c1 > gpurun_out/pmc_issue_sq_c1.txt 2>&1 || { tail -5 gpurun_out/pmc_issue_sq_c1.txt; exit 1; }
find gpurun_out/pmc_issue_* -name "*.db" -delete
echo pmc-done
