# one GPU call: the round's profile (kernel trace of the default bench, FETCH / WRITE / MFMA passes), summarised on the box
cd $GRAFT_REPO_ROOT
ROUND=r3 timeout -k 10 1500 bash tools/profile_round.sh > gpurun_out/r3_profile.log 2>&1
