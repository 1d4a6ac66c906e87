"""Sum rocprofv3 --pmc counters per counter over the dispatches of the kernels whose name contains a
substring: python3 tools/pmc_sum.py <rocprof output dir> <kernel substring> [expansions]"""
import glob
import sqlite3
import sys

out, sub = sys.argv[1], sys.argv[2]
units = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
tot = {}
# (round 6: "**/*.db" with recursive=True already matches the top directory's databases; the round-5
# version also globbed "*.db" and counted those twice -- the 2x of profiles/r5/pmc_mq_issue_r5.txt)
for db in sorted(set(glob.glob(f"{out}/**/*.db", recursive=True))):
    d = sqlite3.connect(db)
    for name, cn, v in d.execute("select kernel_name, counter_name, value from counters_collection"):
        if sub in name:
            tot[cn] = tot.get(cn, 0.0) + v
wc = tot.get("SQ_WAVE_CYCLES", 0.0)
for k in sorted(tot):
    extra = f"  per-wave-cycle {tot[k] / wc:.3f}" if wc else ""
    if units:
        extra += f"  per-unit {tot[k] / units:.1f}"
    print(f"  {k:28s} {tot[k]:18.0f}{extra}")
