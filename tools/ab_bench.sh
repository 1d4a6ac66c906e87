#!/bin/bash
# A/B of two builds of libpmp_hip.so on the A* headline (same box, alternating):
#   bash tools/ab_bench.sh libA.so libB.so [rounds]
R=${GRAFT_REPO_ROOT:-/root/repo}
A=$1; B=$2; N=${3:-3}
mkdir -p $R/gpurun_out/ab
for i in $(seq 1 $N); do
  for L in $A $B; do
    n=$(basename $L .so)
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 200 python3 $R/bench.py --legs none --no-cpu-baseline \
      > $R/gpurun_out/ab/${n}_$i.json 2> $R/gpurun_out/ab/${n}_$i.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('$R/gpurun_out/ab/${n}_$i.json').read().strip().splitlines()[-1]); print('$n', round(d['value']), round(d['ms_per_step']))"
  done
done
