#!/bin/bash
# round 5, call 17: do the legs after the headline run slower in memory the headline just freed?
# (the headline's context freed as usual vs kept until exit)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/c17
leg() {  # name args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --legs astar3d,dstar,dyn3d --detail-out gpurun_out/c17/$n.json "$@" \
    > gpurun_out/c17/$n.out 2> gpurun_out/c17/$n.err || { tail -20 gpurun_out/c17/$n.err; return 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c17/$n.json'))['secondary']
print('$n', {k: round(v['value']) for k, v in d.items()})"
}
for i in 1 2; do
  leg freed_$i && leg kept_$i --keep-headline-ctx 1 || exit 1
done
