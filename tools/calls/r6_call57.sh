#!/bin/bash
# round 6, call 57: RRT* with a smaller random window (128) and hit staging (256) for a larger LDS tree
# share -- parity on the variant, bench-leg A/B
# result: def 1,528 / 1,531 vs rrtsm 1,537 / 1,539 plans/s (parity green): +0.5 %, within the box noise -- defaults kept (the profiled kernel)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c57
PMP_HIP_LIB=$L/libpmp_hip_rrtsm.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c57/pytest.log 2>&1 || { tail -30 gpurun_out/r6c57/pytest.log; exit 1; }
tail -1 gpurun_out/r6c57/pytest.log
for r in 1 2; do
  for v in def rrtsm; do
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs rrt --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c57/b_${v}_$r.out 2> gpurun_out/r6c57/b_${v}_$r.err || { tail -20 gpurun_out/r6c57/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c57/b_${v}_$r.out').read().strip().splitlines()[-1]); s=d['secondary']['rrt_star']; print('$v round $r', s['value'])"
  done
done
