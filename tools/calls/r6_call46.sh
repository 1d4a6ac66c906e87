#!/bin/bash
# round 6, call 46: D* at 512^2 is capped by its 48 GiB scratch budget (~1,750 workers, ~7 per CU at
# ~29 MB each): budget 96 GiB (~3,500 workers) x 1 / 2 streams vs 48 GiB x 2 / 3 streams, D* legs only
# result (512^2 plans/s): 48 GiB x 3 streams 5,951 / 5,896 (default); x 2 4,614 / 4,601; 96 GiB x 2 5,755 / 6,011; x 1 4,042 / 4,068 -- the budget is not adopted (3 x 96 GiB exceeds the HBM)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/r6c46
for r in 1 2; do
  for vs in def:3 def:2 ds96:2 ds96:1; do
    v=${vs%:*}; s=${vs#*:}
    if [ $v = def ]; then unset PMP_HIP_LIB; else export PMP_HIP_LIB=$L/libpmp_hip_$v.so; fi
    timeout -k 10 300 python3 bench.py --legs dstar --steps 1 --warmup 1 --no-cpu-baseline --dstar-streams $s \
      > gpurun_out/r6c46/b_${v}_${s}_$r.out 2> gpurun_out/r6c46/b_${v}_${s}_$r.err || { tail -20 gpurun_out/r6c46/b_${v}_${s}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r6c46/b_${v}_${s}_$r.out').read().strip().splitlines()[-1]); print('$v streams $s round $r', d['secondary']['dstar_256']['value'], d['secondary']['dstar_512']['value'])"
  done
done
