#!/bin/bash
# round 6, call 21: RRT* continuous batching sweep -- batches of 256 C3 queries per launch x launches
# in flight (the round-5 schedule first)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R; mkdir -p gpurun_out/r6c21
for cfg in "1 3 4" "4 2 4" "8 1 2" "8 2 4" "16 1 2"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --legs rrt --steps 2 --warmup 1 --no-cpu-baseline --rrt-batches $1 --rrt-streams $2 \
    --rrt-steps $3 --detail-out gpurun_out/r6c21/d_$1_$2_$3.json > gpurun_out/r6c21/b_$1_$2_$3.out 2> gpurun_out/r6c21/b_$1_$2_$3.err \
    || { tail -20 gpurun_out/r6c21/b_$1_$2_$3.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r6c21/d_$1_$2_$3.json'))
def find(o):
    if isinstance(o, dict):
        if o.get('metric', '').startswith('RRT*'): return o
        for v in o.values():
            r = find(v)
            if r: return r
r = find(d); print('batches $1 streams $2 steps $3:', round(r['value'], 1), 'plans/s, kernel ms/launch', round(r['kernel_ms_per_launch'], 1), 'checked', r['timed_launches_checked'])
"
done
