#!/bin/bash
# round 6, call 53: 3D A* (C5) scratch budget 32 GiB (~4,870 workers) vs 48 GiB (the 20-per-CU 5,120)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c53
for r in 1 2; do
  for v in def a3b48; do
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs astar3d --steps 1 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c53/b_${v}_$r.out 2> gpurun_out/r6c53/b_${v}_$r.err || { tail -20 gpurun_out/r6c53/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c53/b_${v}_$r.out').read().strip().splitlines()[-1]); print('$v round $r', d['secondary']['astar3d']['value'])"
  done
done
