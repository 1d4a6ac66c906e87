#!/bin/bash
# round 4, call 14: the single-query engine with the trivial-push path -- parity, lone-query kernel
# time, and cycle stamps (pop / 3x3 wait / expansion + pushes) vs the one-query-per-wave engine
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/c14
cd $R
timeout -k 10 500 python -u -m pytest tests/test_astar2d_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c14/tests.log 2>&1 || { tail -40 gpurun_out/c14/tests.log; exit 1; }
tail -2 gpurun_out/c14/tests.log
for m in c1 c2med; do
  for e in 3 0; do
    MODE=$m ENGINE=$e REPS=3 timeout -k 10 120 python3 tools/astar2d_probe.py > gpurun_out/c14/t_${m}_$e.log 2>&1 || { tail -20 gpurun_out/c14/t_${m}_$e.log; exit 1; }
    grep plans gpurun_out/c14/t_${m}_$e.log | tail -1
    PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_sqstamps.so MODE=$m ENGINE=$e REPS=2 timeout -k 10 120 python3 tools/astar2d_probe.py > gpurun_out/c14/${m}_$e.log 2>&1 || { tail -20 gpurun_out/c14/${m}_$e.log; exit 1; }
    echo "$m engine $e"; grep stamps gpurun_out/c14/${m}_$e.log | tail -1
  done
done
