#!/bin/bash
# round 5, call 6: LPAStar3D (U peak vs the LDS share, workers per CU, cycle split, the round-4
# kernel beside it), the A* headline's half-block layout at 56 / 64 per CU, Theta* 2D at 32 per CU x3
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c6
timeout -k 10 300 python -u -m pytest tests/test_dwa_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c6/tests.log 2>&1 || { tail -40 gpurun_out/c6/tests.log; exit 1; }
tail -1 gpurun_out/c6/tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --legs dwa --agents 32 --steps 5 --warmup 2 --detail-out gpurun_out/c6/dwa32.json > gpurun_out/c6/dwa32.out 2> gpurun_out/c6/dwa32.err || { tail -20 gpurun_out/c6/dwa32.err; exit 1; }
python3 -c "
import json; v=json.load(open('gpurun_out/c6/dwa32.json'))['secondary']['mpc_sampled_dwa']; print('dwa32', round(v['value']), 'kernel_ms', v['kernel_ms_per_launch'])"
PMP_HIP_LIB=$L/libpmp_hip_dwastamps.so timeout -k 10 200 python3 tools/dwa_split_probe.py > gpurun_out/c6/dwa_stamps.log 2>&1 || { tail -20 gpurun_out/c6/dwa_stamps.log; exit 1; }
grep "per-phase" gpurun_out/c6/dwa_stamps.log
timeout -k 10 300 python3 tools/lpa3d_probe.py 8 12 16 24 > gpurun_out/c6/lpa3d.log 2>&1 || { tail -20 gpurun_out/c6/lpa3d.log; exit 1; }
PMP_HIP_LIB=$L/libpmp_hip_lpastamps.so timeout -k 10 200 python3 tools/lpa3d_probe.py 16 > gpurun_out/c6/lpa3d_stamps.log 2>&1 || { tail -20 gpurun_out/c6/lpa3d_stamps.log; exit 1; }
PMP_HIP_LIB=$L/libpmp_hip_lpar4.so timeout -k 10 200 python3 tools/lpa3d_probe.py 16 > gpurun_out/c6/lpa3d_r4.log 2>&1 || { tail -20 gpurun_out/c6/lpa3d_r4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c6/lpa3d.log gpurun_out/c6/lpa3d_stamps.log gpurun_out/c6/lpa3d_r4.log
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 200 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c6/$n.json "$@" \
    > gpurun_out/c6/$n.out 2> gpurun_out/c6/$n.err || { tail -20 gpurun_out/c6/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c6/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
for i in 1 2; do
  head1 def60_$i $L/libpmp_hip.so &&
  head1 blk2_56_$i $L/libpmp_hip_blk2.so --residency 56 &&
  head1 blk2_60_$i $L/libpmp_hip_blk2.so &&
  head1 blk2_64_$i $L/libpmp_hip_blk2.so --residency 64 || exit 1
done
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --legs graphs --no-cpu-baseline --theta-residency 32 --detail-out gpurun_out/c6/theta_$i.json \
    > gpurun_out/c6/theta_$i.out 2> gpurun_out/c6/theta_$i.err || { tail -20 gpurun_out/c6/theta_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c6/theta_$i.json'))['secondary']
for k in ('theta_star_2d', 'lazy_theta_star_2d'): print('theta r32 run $i', k, round(d[k]['value']), 'kernel_ms', round(d[k]['kernel_ms_per_launch']))"
done
