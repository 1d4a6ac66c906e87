#!/bin/bash
# round 6, call 27: multi-query LDS share per wave (512-B granules, even caps): the headline-schedule
# parity test on that build, then 56 / 60 / 64 groups per CU against the round's build at 56, alternating
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c27
PMP_HIP_LIB=$L/libpmp_hip_gran512.so timeout -k 10 500 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_astar2d_gpu.py -k "headline_schedule" > gpurun_out/r6c27/pytest.log 2>&1 || { tail -30 gpurun_out/r6c27/pytest.log; exit 1; }
tail -1 gpurun_out/r6c27/pytest.log
for r in 1 2; do
  for cfg in "libpmp_hip.so 56" "libpmp_hip_gran512.so 56" "libpmp_hip_gran512.so 60" "libpmp_hip_gran512.so 64"; do
    set -- $cfg
    timeout -k 10 200 python3 -u tools/ab_headline.py $L/$1 --rounds 1 --reps 2 --residency $2 --workers $((256 * $2)) \
      > gpurun_out/r6c27/ab_$1_$2_$r.log 2>&1 || { tail -20 gpurun_out/r6c27/ab_$1_$2_$r.log; exit 1; }
    echo "$1 @$2 round $r: $(grep median gpurun_out/r6c27/ab_$1_$2_$r.log)"
  done
done
