#!/bin/bash
# round 6, call 16: LPAStar3D push without the bpermute round, branch-free key compare -- parity, A/B
# against the round-5 form (libpmp_hip_l3old.so), and the removes / pushes / compaction stamps
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c16
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lpastar3d_gpu.py \
  > gpurun_out/r6c16/pytest.log 2>&1 || { tail -30 gpurun_out/r6c16/pytest.log; exit 1; }
tail -1 gpurun_out/r6c16/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_l3old.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r"
    timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 | head -1 || exit 1
  done
done
echo "== stamps2"
PMP_HIP_LIB=$L/libpmp_hip_stamps2.so timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 || exit 1
