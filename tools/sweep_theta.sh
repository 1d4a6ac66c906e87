#!/bin/bash
# Theta* / Lazy Theta* 2D legs under the headline's residency schedule (same box)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/theta
mkdir -p $O
run() {
  n=$1; shift
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 --legs graphs --graph-steps 12 "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); s=d['secondary']; print('$n', round(s['theta_star_2d']['value']), round(s['lazy_theta_star_2d']['value']), flush=True)"
}
run base_w3072_s3
run w768_s6_r18 --theta-workers 768 --theta-streams 6 --theta-residency 18
run w640_s6_r15 --theta-workers 640 --theta-streams 6 --theta-residency 15
echo sweep-done
