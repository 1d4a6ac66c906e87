#!/bin/bash
# round 6, call 35: RRT* LDS-only barriers where global stores may stay in flight: parity + A/B
# result: new 527.6 / 526.8 ms vs old 515.3 / 514.8 ms (parity green) -- not adopted
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c35
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c35/pytest.log 2>&1 || { tail -30 gpurun_out/r6c35/pytest.log; exit 1; }
tail -1 gpurun_out/r6c35/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrtold.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r: $(timeout -k 10 200 python3 -u tools/rrt_time.py 256x65536 2>&1 | grep 'nq=')"
  done
done
