#!/bin/bash
# A/B of two builds of libpmp_hip.so on the LQR / MPC tracking legs (same box, alternating):
#   bash tools/ab_track.sh libA.so libB.so [rounds]
R=${GRAFT_REPO_ROOT:-/root/repo}
A=$1; B=$2; N=${3:-2}
mkdir -p $R/gpurun_out/abt
for i in $(seq 1 $N); do
  for L in $A $B; do
    n=$(basename $L .so)
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 300 python3 $R/bench.py --legs lqr,mpc --no-cpu-baseline \
      --steps 1 --warmup 1 > $R/gpurun_out/abt/${n}_$i.json 2> $R/gpurun_out/abt/${n}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/abt/${n}_$i.json').read().strip().splitlines()[-1]); s=d['secondary']; print('$n', round(s['lqr']['value']), round(s['mpc_qp']['value']))"
  done
done
