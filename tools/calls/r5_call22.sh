#!/bin/bash
# round 5, call 22: LPAStar3D write attribution (mirror builds: U spill stores, g / rhs stores, bits)
# and the default build's FETCH / WRITE, one counter per pass, over tools/lpa3d_probe.py 16
R=${GRAFT_REPO_ROOT:-/root/repo}
L=$R/python_motion_planning_amd
OUT=$R/gpurun_out/c22
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in default:WRITE_SIZE default:FETCH_SIZE l3mir1:WRITE_SIZE l3mir2:WRITE_SIZE l3mir4:WRITE_SIZE; do
  v=${spec%%:*}; c=${spec#*:}
  lib=$L/libpmp_hip.so
  [ "$v" = default ] || lib=$L/libpmp_hip_$v.so
  PMP_HIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/$v-$c -o run -- python3 $R/tools/lpa3d_probe.py 16 \
    > $OUT/$v-$c.log 2>&1 || { echo "$v $c failed"; tail -5 $OUT/$v-$c.log; exit 1; }
  echo "$v $c $(grep 'plans/s' $OUT/$v-$c.log)"
  python3 $R/tools/pmc_sum.py $OUT/$v-$c lpa3d_kernel
  rm -rf $OUT/$v-$c
done
# Theta* 2D residency beyond 48 per CU (needs 4 waves per SIMD: the 128-VGPR build, which spills)
cd $R
theta() {  # name lib args...
  local n=$1 lib=$2; shift 2
  PMP_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --legs graphs --no-cpu-baseline --detail-out $OUT/$n.json "$@" \
    > $OUT/$n.out 2> $OUT/$n.err || { tail -20 $OUT/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$n.json'))['secondary']
for k in ('theta_star_2d', 'lazy_theta_star_2d'): print('$n', k, round(d[k]['value']), 'kernel_ms', round(d[k]['kernel_ms_per_launch']))"
}
theta r48 $L/libpmp_hip.so --theta-residency 48 && theta tw4_r48 $L/libpmp_hip_tw4.so --theta-residency 48 &&
theta tw4_r56 $L/libpmp_hip_tw4.so --theta-residency 56 && theta tw4_r64 $L/libpmp_hip_tw4.so --theta-residency 64
