#!/bin/bash
# round 5: A* 2D write-traffic attribution at the bench geometry (20 C2 batches in one launch, 60 per
# CU).  One WRITE_SIZE pass per build: the default and the mirror builds of astar2d_mq.hip
# (PMP_MQ_MIRROR bits 1 / 2 / 4 / 8: tools/build_variant.sh mir<bit>), each store of the mirrored
# category issued twice; blk2 / blk2mir = the half-block spill layout (PMP_MQ_BLOCKS=2), plain / all
# spill stores mirrored.  Per-dispatch WRITE_SIZE of the 20-batch launch -> gpurun_out/attr/summary.txt
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${ATTR_DIR:-attr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# spec = build[:counter,counter...] (default counter WRITE_SIZE); blk2 = the half-block spill layout
for spec in ${SPECS:-default:WRITE_SIZE,FETCH_SIZE mir1 mir2 mir4 mir8 blk2:WRITE_SIZE,FETCH_SIZE blk2mir}; do
  v=${spec%%:*}
  cs=WRITE_SIZE
  [ "$spec" = "$v" ] || cs=${spec#*:}
  lib=$R/python_motion_planning_amd/libpmp_hip.so
  [ "$v" = default ] || lib=$R/python_motion_planning_amd/libpmp_hip_$v.so
  for c in ${cs//,/ }; do
    PMP_HIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $c -d $OUT/$v-$c -o run -- \
      python3 $R/bench.py --legs none --no-cpu-baseline --steps 20 --warmup 5 --detail-out $OUT/$v-$c.detail.json \
      > $OUT/$v-$c.json 2> $OUT/$v-$c.err || { echo "$v $c failed"; tail -5 $OUT/$v-$c.err; exit 1; }
    python3 - $OUT $v $c >> $OUT/summary.txt <<'PY'
import glob, json, sqlite3, sys
out, v, c = sys.argv[1:4]
db = (glob.glob(f"{out}/{v}-{c}/**/*.db", recursive=True) + glob.glob(f"{out}/{v}-{c}/*.db"))[0]
d = sqlite3.connect(db)
cols = [r[1] for r in d.execute("pragma table_info(counters_collection)")]
key = "dispatch_id" if "dispatch_id" in cols else "correlation_id"
rows = list(d.execute(f"select kernel_name, sum(value) from counters_collection where counter_name = ? "
                      f"group by {key} order by {key}", (c,)))
mq = [x for n, x in rows if "mqu_kernel" in n]
line = json.loads(open(f"{out}/{v}-{c}.json").read().strip().splitlines()[-1])
print(v, c, "per-dispatch KiB", [round(x) for x in mq], "plans/s", round(line["value"]))
PY
    rm -rf $OUT/$v-$c
  done
done
cat $OUT/summary.txt
