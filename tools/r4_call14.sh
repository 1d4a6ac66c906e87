#!/bin/bash
# round 4, call 14: cycle stamps of the single-query engine vs the one-query-per-wave engine (lone queries)
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/c14
for m in c1 c2med; do
  for e in 3 0; do
    PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_sqstamps.so MODE=$m ENGINE=$e REPS=2 timeout -k 10 120 python3 $R/tools/astar2d_probe.py > $R/gpurun_out/c14/${m}_$e.log 2>&1 || { tail -20 $R/gpurun_out/c14/${m}_$e.log; exit 1; }
    echo "$m engine $e"; grep stamps $R/gpurun_out/c14/${m}_$e.log
  done
done
