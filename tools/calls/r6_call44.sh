#!/bin/bash
# round 6, call 44: RRT* LDS-only barriers at 256 threads x 2 per CU (slower at 512 x 1, call 35) --
# parity on the variant, bench-leg A/B
# result: def 1540 / 1535 vs rrtldsb 1467 / 1486 plans/s (parity green) -- not adopted
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c44
PMP_HIP_LIB=$L/libpmp_hip_rrtldsb.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
  > gpurun_out/r6c44/pytest.log 2>&1 || { tail -30 gpurun_out/r6c44/pytest.log; exit 1; }
tail -1 gpurun_out/r6c44/pytest.log
for r in 1 2; do
  for v in def rrtldsb; do
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs rrt --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c44/b_${v}_$r.out 2> gpurun_out/r6c44/b_${v}_$r.err || { tail -20 gpurun_out/r6c44/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c44/b_${v}_$r.out').read().strip().splitlines()[-1]); s=d['secondary']['rrt_star']; print('$v round $r', s['value'])"
  done
done
