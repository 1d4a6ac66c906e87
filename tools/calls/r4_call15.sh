#!/bin/bash
# round 4, call 15: cycle stamps of the single-query engine vs the one-query-per-wave engine (lone queries)
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/c15
cd $R
for m in c1 c2med; do
  for e in 3 0; do
    PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_sqstamps.so MODE=$m ENGINE=$e REPS=2 timeout -k 10 120 python3 tools/astar2d_probe.py > gpurun_out/c15/${m}_$e.log 2>&1 || { tail -20 gpurun_out/c15/${m}_$e.log; exit 1; }
    echo "$m engine $e"; grep stamps gpurun_out/c15/${m}_$e.log | tail -1
  done
  MODE=$m ENGINE=3 REPS=3 timeout -k 10 120 python3 tools/astar2d_probe.py 2>&1 | grep plans | tail -1
done
