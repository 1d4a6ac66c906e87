#!/bin/bash
# Batches-in-flight sweep of the one-wave-per-query secondary legs (same box):
#   bash tools/sweep_inflight.sh   -> gpurun_out/inflight/*.json, one summary line per run
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/inflight
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
for q in 8 16; do
  for s in 4 6 8; do
    run a3_s${s}_q${q} --legs astar3d --a3-steps 24 --a3-streams $s --hw-queues $q
    run dyn_s${s}_q${q} --legs dyn3d --dyn3d-steps 12 --dyn3d-streams $s --hw-queues $q
  done
done
for s in 2 3 4; do run dstar_s$s --legs dstar --dstar-streams $s --hw-queues 8; done
for s in 3 5; do run graphs_s$s --legs graphs --lpa-streams $s --theta-streams $s --hw-queues 8; done
echo sweep-done
