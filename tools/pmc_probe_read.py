"""Summarise tools/pmc_probe.sh: per-heap-op PMC counts of the A* 2D kernel (either engine)."""
import glob
import re
import sqlite3
import sys

root = sys.argv[1]
vals = {}
for db in sorted(glob.glob(f"{root}/p*/run_results.db")):
    d = sqlite3.connect(db)
    for name, s in d.execute("select counter_name, sum(value) from counters_collection "
                             "where kernel_name like '%astar2d%kernel%' group by counter_name"):
        vals[name] = s
m = re.search(r"(\S+ engine .*?): ([\d.]+) ms pushes (\d+) pops (\d+) exp (\d+)", open(f"{root}/p1.log").read())
P, Q, E = int(m.group(3)), int(m.group(4)), int(m.group(5))
print(m.group(1), "launch ms", m.group(2), "ops", P + Q, "expansions", E)
for k, v in sorted(vals.items()):
    print(f"  {k:24s} {v:18.0f}  per-op {v / (P + Q):9.2f}")
