"""Summarise tools/pmc_astar2d.sh output: per-heap-op PMC counts of the A* 2D kernel."""
import glob
import re
import sqlite3
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_a2"
for mode in ("longest", "batch"):
    vals = {}
    for db in sorted(glob.glob(f"{root}/{mode}_*/run_results.db")):
        d = sqlite3.connect(db)
        for name, s in d.execute("select counter_name, sum(value) from counters_collection "
                                 "where kernel_name like '%astar2d_kernel%' group by counter_name"):
            vals[name] = s
    if not vals:
        continue
    m = re.search(r"pushes (\d+) pops (\d+) exp (\d+)", open(f"{root}/{mode}_1.log").read())
    P, Q, E = map(int, m.groups())
    print(mode, "ops", P + Q, "expansions", E)
    for k, v in sorted(vals.items()):
        print(f"  {k:24s} {v:18.0f}  per-op {v / (P + Q):9.2f}")
