#!/bin/bash
# round 6, call 14: LPAStar3D deferred removes -- lpa3d parity, then an A/B against the round-5 form
# (libpmp_hip_l3old.so = -DPMP_L3_DEFER=0), alternating processes
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c14
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lpastar3d_gpu.py \
  > gpurun_out/r6c14/pytest.log 2>&1 || { tail -30 gpurun_out/r6c14/pytest.log; exit 1; }
tail -3 gpurun_out/r6c14/pytest.log
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export PMP_HIP_LIB=$L/libpmp_hip_l3old.so; else unset PMP_HIP_LIB; fi
    echo "== $v round $r"
    timeout -k 10 200 python3 -u tools/lpa3d_probe.py 16 2>&1 | tail -2 || exit 1
  done
done
