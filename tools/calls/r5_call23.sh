#!/bin/bash
# round 5, call 23: LPAStar3D bench schedule sweep (workers per CU, launches in flight, batches per launch)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c23
leg() {  # name args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --legs dyn3d --detail-out gpurun_out/c23/$n.json "$@" > gpurun_out/c23/$n.out 2> gpurun_out/c23/$n.err || { tail -20 gpurun_out/c23/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c23/$n.json'))['secondary']
print('$n', {k: round(v['value']) for k, v in d.items() if k.startswith('lpa')})"
}
leg base && leg w12 --lpa3d-workers-per-cu 12 && leg w20 --lpa3d-workers-per-cu 20 && leg w24 --lpa3d-workers-per-cu 24 &&
leg s6 --dyn3d-streams 6 && leg b12 --dyn3d-batches-per-launch 12 && leg b24 --dyn3d-batches-per-launch 24 --dyn3d-streams 1
