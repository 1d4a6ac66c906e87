#!/bin/bash
# round 5, call 13: contiguous scratch (hipDeviceMallocContiguous, dev build) vs hipMalloc on the
# headline and the Theta* legs; Theta* residency 28 / 36
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
cd $R; mkdir -p gpurun_out/c13
head1() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --legs none --no-cpu-baseline --detail-out gpurun_out/c13/$n.json "$@" \
    > gpurun_out/c13/$n.out 2> gpurun_out/c13/$n.err || { tail -20 gpurun_out/c13/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/c13/$n.out').read().strip().splitlines()[-1]); print('$n', round(d['value']), 'ms/step', round(d['ms_per_step'], 1))"
}
theta() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --legs graphs --no-cpu-baseline --detail-out gpurun_out/c13/$n.json "$@" \
    > gpurun_out/c13/$n.out 2> gpurun_out/c13/$n.err || { tail -20 gpurun_out/c13/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c13/$n.json'))['secondary']
for k in ('theta_star_2d', 'lazy_theta_star_2d'): print('$n', k, round(d[k]['value']), 'kernel_ms', round(d[k]['kernel_ms_per_launch']))"
}
head1 def_1 $L/libpmp_hip.so && head1 contig_1 $L/libpmp_hip_contig.so && head1 def_2 $L/libpmp_hip.so && head1 contig_2 $L/libpmp_hip_contig.so || exit 1
theta th_def $L/libpmp_hip.so && theta th_contig $L/libpmp_hip_contig.so && theta th_r28 $L/libpmp_hip.so --theta-residency 28 && theta th_r36 $L/libpmp_hip.so --theta-residency 36
