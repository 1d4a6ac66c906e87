#!/bin/bash
# round 6, call 56: two-pass D* budget 48 GiB (~3,760 first-pass workers at 512^2) vs 56 GiB (the
# 16-per-CU 4,096), 3 streams, D* legs only
# result (256^2 / 512^2 plans/s): 48 GiB 32,310 / 6,513 and 32,230 / 6,516; 56 GiB 32,350 / 6,538 and 32,520 / 6,478 -- no change, 48 kept
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c56
for r in 1 2; do
  for v in def ds56; do
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs dstar --steps 1 --warmup 1 --no-cpu-baseline \
      > gpurun_out/r6c56/b_${v}_$r.out 2> gpurun_out/r6c56/b_${v}_$r.err || { tail -20 gpurun_out/r6c56/b_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c56/b_${v}_$r.out').read().strip().splitlines()[-1]); print('$v round $r', d['secondary']['dstar_256']['value'], d['secondary']['dstar_512']['value'])"
  done
done
