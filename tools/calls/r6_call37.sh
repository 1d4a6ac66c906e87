#!/bin/bash
# round 6, call 37: RRT* bench leg (8 batches x 2 streams), 256 threads x 2 per CU vs 512 x 1, alternating
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c37
for r in 1 2; do
  for v in 256 512; do
    if [ $v = 256 ]; then export PMP_HIP_LIB=$L/libpmp_hip_rrt256.so; else unset PMP_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --legs rrt --steps 4 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c37/b_${v}_$r.out 2> gpurun_out/r6c37/b_${v}_$r.err || { tail -20 gpurun_out/r6c37/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c37/b_${v}_$r.out').read().strip().splitlines()[-1]); s=d['secondary']['rrt_star']; print('$v round $r', s['value'], s.get('kernel_ms_per_launch'))"
  done
done
