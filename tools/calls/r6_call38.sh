#!/bin/bash
# round 6, call 38: RRT* at 256 threads x 2 per CU: obstacles in dynamic LDS sized to the map (a larger
# LDS tree share), candidate LDS lists of 256 / 128 / 64 -- parity on the default and k64, bench-leg A/B
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c38
for v in def k64; do
  if [ $v = k64 ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrtk64.so; else unset PMP_HIP_LIB; fi
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_rrt_gpu.py \
    > gpurun_out/r6c38/pytest_$v.log 2>&1 || { tail -30 gpurun_out/r6c38/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r6c38/pytest_$v.log)"
done
for r in 1 2; do
  for v in rrt256 def rrtk128 rrtk64; do
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs rrt --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c38/b_${v}_$r.out 2> gpurun_out/r6c38/b_${v}_$r.err || { tail -20 gpurun_out/r6c38/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c38/b_${v}_$r.out').read().strip().splitlines()[-1]); s=d['secondary']['rrt_star']; print('$v round $r', s['value'])"
  done
done
