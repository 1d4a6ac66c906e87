#!/bin/bash
# round 5, final tree after the DWA rotation table: GPU suite + smoke + kernel-trace profile (final2),
# the PMC passes (final3), the bench's default command (final4), in one call
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/calls/r5_final2.sh || exit 1
bash tools/calls/r5_final3.sh > gpurun_out/final3_out.txt 2>&1 || { tail -20 gpurun_out/final3_out.txt; exit 1; }
tail -2 gpurun_out/final3_out.txt
sed -i 's#gpurun_out/final5#gpurun_out/final6#g' tools/calls/r5_final5.sh
bash tools/calls/r5_final5.sh || exit 1
