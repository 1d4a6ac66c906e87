#!/bin/bash
# A/B of two builds on one secondary leg (headline shortened to one batch), alternating:
#   bash tools/ab_leg.sh <leg> <secondary key> libA.so libB.so [rounds] [extra bench args]
R=${GRAFT_REPO_ROOT:-/root/repo}
LEG=$1; KEY=$2; A=$3; B=$4; N=${5:-2}; shift 5; EXTRA="$@"
mkdir -p $R/gpurun_out/ab
for i in $(seq 1 $N); do
  for L in $A $B; do
    n=$(basename $L .so)
    PMP_HIP_LIB=$R/python_motion_planning_amd/$L timeout -k 10 300 python3 $R/bench.py --legs $LEG --no-cpu-baseline \
      --steps 1 --warmup 1 $EXTRA --detail-out $R/gpurun_out/ab/${LEG}_${n}_$i.detail.json \
      > $R/gpurun_out/ab/${LEG}_${n}_$i.json 2> $R/gpurun_out/ab/${LEG}_${n}_$i.err || { tail -5 $R/gpurun_out/ab/${LEG}_${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$R/gpurun_out/ab/${LEG}_${n}_$i.json').read().strip().splitlines()[-1]); print('$n', '$KEY', d['secondary']['$KEY'])"
  done
done
