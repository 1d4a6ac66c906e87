#!/bin/bash
# round 5, call 30: DWA leaf sums on 8-lane groups + two-run nibble build -- parity, control leg, DWA.plan, stamps
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c30
timeout -k 10 400 python3 -u -m pytest tests/test_dwa_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/c30/test.log 2>&1 || { tail -30 gpurun_out/c30/test.log; exit 1; }
tail -2 gpurun_out/c30/test.log
timeout -k 10 200 python3 tools/dwa_plan_time.py 3 || exit 1
for A in 256 32; do
  n=dwa_$A
  timeout -k 10 200 python3 bench.py --legs dwa --agents $A --steps 1 --warmup 1 \
    --no-cpu-baseline --control-steps 40 --detail-out gpurun_out/c30/$n.json > gpurun_out/c30/$n.out 2> gpurun_out/c30/$n.err || { tail -20 gpurun_out/c30/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c30/$n.json'))['secondary']
print('$n', {k: (round(v['value']), round(v['kernel_ms_per_launch']*1e3, 1), v.get('timed_launches_checked')) for k, v in d.items()})"
done
PMP_HIP_LIB=$R/python_motion_planning_amd/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c30/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c30/dwa_stamps.log; exit 1; }
grep -E "per-phase|LOCAL" gpurun_out/c30/dwa_stamps.log
