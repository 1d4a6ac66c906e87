#!/bin/bash
# round 5, call 32: DWA A/B -- paired nibble lookups (PAIR) and paired heading chains (COLPAIR), two rounds
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c32
for rnd in 1 2; do
for L in libpmp_hip.so libpmp_hip_pair0.so libpmp_hip_colpair0.so libpmp_hip_both0.so; do
  for A in 256 32; do
    n=${L%.so}_${A}_$rnd
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 200 python3 bench.py --legs dwa --agents $A --steps 1 --warmup 1 \
      --no-cpu-baseline --control-steps 40 --detail-out gpurun_out/c32/$n.json > gpurun_out/c32/$n.out 2> gpurun_out/c32/$n.err || { tail -20 gpurun_out/c32/$n.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/c32/$n.json'))['secondary']
print('$n', {k: (round(v['value']), round(v['kernel_ms_per_launch']*1e3, 1), v.get('timed_launches_checked')) for k, v in d.items()})"
  done
done
done
