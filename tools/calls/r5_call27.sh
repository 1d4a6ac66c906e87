#!/bin/bash
# round 5, call 27: DWA nibble-map stencil (R <= 1) -- parity, then the control leg per build
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c27
timeout -k 10 400 python3 -u -m pytest tests/test_dwa_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c27/test.log 2>&1 || { tail -30 gpurun_out/c27/test.log; exit 1; }
tail -3 gpurun_out/c27/test.log
for L in libpmp_hip.so libpmp_hip_local0.so libpmp_hip_split3.so libpmp_hip.so; do
  for A in 256 32; do
    n=${L%.so}_$A
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 200 python3 bench.py --legs dwa --agents $A --steps 1 --warmup 1 \
      --no-cpu-baseline --control-steps 40 --detail-out gpurun_out/c27/$n.json > gpurun_out/c27/$n.out 2> gpurun_out/c27/$n.err || { tail -20 gpurun_out/c27/$n.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/c27/$n.json'))['secondary']
print('$n', {k: (round(v['value']), round(v['kernel_ms_per_launch']*1e3, 1), v.get('timed_launches_checked')) for k, v in d.items()})"
  done
done
