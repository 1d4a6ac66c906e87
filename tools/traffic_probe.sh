#!/bin/bash
# A* 2D traffic attribution (dev): FETCH_SIZE / WRITE_SIZE passes of one C2 batch (tools/astar2d_probe.py,
# REPS=1) under several engine / residency settings; totals per variant in gpurun_out/traffic_<tag>.txt.
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do   # spec = tag:ENGINE:T2LDS:WORKERS:RESIDENCY
  IFS=: read tag eng t2 w res <<< "$spec"
  for c in FETCH_SIZE WRITE_SIZE; do
    ENGINE=$eng T2LDS=$t2 WORKERS=$w RESIDENCY=$res REPS=1 timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/$tag-$c -o run -- \
      python3 $R/tools/astar2d_probe.py > $OUT/$tag-$c.log 2>&1 || { echo "$tag $c failed"; exit 1; }
  done
  python3 - $OUT $tag >> $OUT/summary.txt <<'PY'
import sqlite3, sys, glob
out, tag = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    db = glob.glob(f"{out}/{tag}-{c}/**/*.db", recursive=True) + glob.glob(f"{out}/{tag}-{c}/*.db")
    d = sqlite3.connect(db[0])
    res[c] = d.execute("select sum(value) from counters_collection where counter_name = ? and kernel_name like '%astar2d%kernel%'", (c,)).fetchone()[0]
log = open(f"{out}/{tag}-FETCH_SIZE.log").read().strip().splitlines()
print(tag, "FETCH_KiB", res["FETCH_SIZE"], "WRITE_KiB", res["WRITE_SIZE"], "|", log[-1] if log else "")
PY
  rm -rf $OUT/$tag-FETCH_SIZE $OUT/$tag-WRITE_SIZE
done
cat $OUT/summary.txt
