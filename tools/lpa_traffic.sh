#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of one LPA* / D* Lite launch (tools/lpa_probe.py): bytes per algorithmic byte
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/lpa_traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lite in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    LITE=$lite timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/$lite-$c -o run -- python3 $R/tools/lpa_probe.py > $OUT/$lite-$c.log 2>&1 || { echo "lite=$lite $c failed"; tail -5 $OUT/$lite-$c.log; exit 1; }
  done
  python3 - $OUT $lite <<'PY'
import glob, re, sqlite3, sys
out, lite = sys.argv[1], sys.argv[2]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    db = glob.glob(f"{out}/{lite}-{c}/**/*.db", recursive=True)
    d = sqlite3.connect(db[0])
    res[c] = d.execute("select sum(value) from counters_collection where counter_name = ? and kernel_name like '%lpa_kernel%'", (c,)).fetchone()[0]
log = open(f"{out}/{lite}-FETCH_SIZE.log").read()
m = re.search(r"alg_bytes (\d+)", log)
alg = float(m.group(1))
line = [l for l in log.splitlines() if "alg_bytes" in l][0]
print(line)
# the warm launch (64 queries) is in the sums too: negligible
print(f"  FETCH {res['FETCH_SIZE'] * 1024 / 1e9:.2f} GB (x2 {2 * res['FETCH_SIZE'] * 1024 / alg:.2f}x alg)  WRITE {res['WRITE_SIZE'] * 1024 / 1e9:.2f} GB  "
      f"traffic_x (fetch doubled + write) {(2 * res['FETCH_SIZE'] + res['WRITE_SIZE']) * 1024 / alg:.2f}  raw {(res['FETCH_SIZE'] + res['WRITE_SIZE']) * 1024 / alg:.2f}")
PY
  rm -rf $OUT/$lite-FETCH_SIZE $OUT/$lite-WRITE_SIZE
done
