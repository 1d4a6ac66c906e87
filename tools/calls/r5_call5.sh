#!/bin/bash
# round 5, call 5: DWA split (one-round lookahead, leaf table beside the tail, coherent loads in place
# of the acquire fence) and RRT* (8-wide LDS scans, LDS share knob, 256-thread variants, phase stamps)
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c5
timeout -k 10 400 python -u -m pytest tests/test_dwa_gpu.py tests/test_rrt_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5/tests.log 2>&1 || { tail -40 gpurun_out/c5/tests.log; exit 1; }
tail -1 gpurun_out/c5/tests.log
PMP_HIP_LIB=$L/libpmp_hip_rrt256.so timeout -k 10 400 python -u -m pytest tests/test_rrt_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5/tests256.log 2>&1 || { tail -40 gpurun_out/c5/tests256.log; exit 1; }
tail -1 gpurun_out/c5/tests256.log
leg() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --detail-out gpurun_out/c5/$n.json "$@" > gpurun_out/c5/$n.out 2> gpurun_out/c5/$n.err || { tail -20 gpurun_out/c5/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c5/$n.json'))['secondary']
for k, v in d.items(): print('$n', k, round(v['value']), 'kernel_ms', round(v.get('kernel_ms_per_launch', 0), 4), 'frac', v.get('roofline', {}).get('frac'))"
}
leg dwa32 $L/libpmp_hip.so --legs dwa --agents 32 --steps 5 --warmup 2 &&
leg dwa32acq $L/libpmp_hip_dwaacq.so --legs dwa --agents 32 --steps 5 --warmup 2 &&
leg dwa256 $L/libpmp_hip.so --legs dwa --steps 5 --warmup 2 || exit 1
PMP_HIP_LIB=$L/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c5/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c5/dwa_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c5/dwa_stamps.log
for v in rrtstamps rrt256stamps; do
  PMP_HIP_LIB=$L/libpmp_hip_$v.so timeout -k 10 200 python3 tools/rrt_time.py 4x16384 256x8192 > gpurun_out/c5/$v.log 2>&1 || { tail -20 gpurun_out/c5/$v.log; exit 1; }
  echo $v; grep -v amdgpu.ids gpurun_out/c5/$v.log
done
leg rrt_r1 $L/libpmp_hip.so --legs rrt &&
leg rrt_r2 $L/libpmp_hip.so --legs rrt --rrt-resident 2 &&
leg rrt256_r1 $L/libpmp_hip_rrt256.so --legs rrt &&
leg rrt256_r2 $L/libpmp_hip_rrt256.so --legs rrt --rrt-resident 2 &&
leg rrt256w3_r3 $L/libpmp_hip_rrt256w3.so --legs rrt --rrt-resident 3 --rrt-streams 4
