#!/bin/bash
# 3D A* (C5) and D* legs: workers per CU per launch x batches in flight x resident per CU (same box):
#   bash tools/sweep_resident3d.sh -> gpurun_out/res3d/*.json, one summary line per run
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/res3d
mkdir -p $O
run() {  # name, bench args...
  n=$1; shift
  timeout -k 10 240 python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || exit 1
  python3 - $O/$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = d.get("secondary", {})
out = [f"{k}={v['value']:.4g}" for k, v in sec.items() if isinstance(v, dict) and "value" in v and v.get("unit") != "ms"]
print(sys.argv[2], " ".join(out), flush=True)
PY
}
run a3_w16_s6 --legs astar3d --a3-workers-per-cu 16 --a3-streams 6
run a3_w4_s6_r24 --legs astar3d --a3-workers-per-cu 4 --a3-streams 6 --a3-residency 24
run a3_w4_s6_r16 --legs astar3d --a3-workers-per-cu 4 --a3-streams 6 --a3-residency 16
run a3_w3_s8_r24 --legs astar3d --a3-workers-per-cu 3 --a3-streams 8 --a3-residency 24
run a3_w5_s6_r30 --legs astar3d --a3-workers-per-cu 5 --a3-streams 6 --a3-residency 30
run a3_w8_s6_r32 --legs astar3d --a3-workers-per-cu 8 --a3-streams 6 --a3-residency 32
run ds_w16_s3 --legs dstar --dstar-streams 3
run ds_w4_s6_r24 --legs dstar --dstar-workers-per-cu 4 --dstar-streams 6 --dstar-residency 24
run ds_w4_s4_r16 --legs dstar --dstar-workers-per-cu 4 --dstar-streams 4 --dstar-residency 16
run ds_w6_s4_r24 --legs dstar --dstar-workers-per-cu 6 --dstar-streams 4 --dstar-residency 24
run ds_w3_s6_r18 --legs dstar --dstar-workers-per-cu 3 --dstar-streams 6 --dstar-residency 18
echo sweep-done
