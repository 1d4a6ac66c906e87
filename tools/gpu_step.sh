# one GPU call: PMC issue breakdown of the C1 single query (engine 0, LDS grid)
cd $GRAFT_REPO_ROOT
ENGINE=0 MODE=c1 TAG=c1 timeout -k 10 500 bash tools/pmc_probe.sh > gpurun_out/r3_pmc_c1.log 2>&1
