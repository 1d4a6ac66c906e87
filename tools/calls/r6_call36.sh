#!/bin/bash
# round 6, call 36: RRT* at 256 threads per query, two workgroups per CU (the scans are cheap since the
# integer coarse distances) -- parity on the variant, A/B against the 512-thread kernel
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c36
PMP_HIP_LIB=$L/libpmp_hip_rrt256.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c36/pytest.log 2>&1 || { tail -30 gpurun_out/r6c36/pytest.log; exit 1; }
tail -1 gpurun_out/r6c36/pytest.log
for r in 1 2; do
  for v in 256 512; do
    if [ $v = 256 ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrt256.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r: $(timeout -k 10 200 python3 -u tools/rrt_time.py 512x65536 2>&1 | grep 'nq=')"
  done
done
