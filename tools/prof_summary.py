"""Summarise a round's rocprofv3 databases (tools/profile_round.sh) into profiles/<round>/:
  kernel_stats.csv   -- rocprofv3 --kernel-trace --stats of the default bench command
  pmc_traffic.json   -- per-kernel FETCH_SIZE / WRITE_SIZE per dispatch from the two --pmc passes,
                        with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE counts half the
                        bytes of wide streaming reads: doubled; WRITE_SIZE as is; both in KiB)
usage: python tools/prof_summary.py gpurun_out profiles/r1
"""
import csv
import json
import os
import re
import sqlite3
import sys

KERNELS = {  # short name -> regex on the demangled kernel name
    "lpt_hist": r"lpt_hist\(", "lpt_scan": r"lpt_scan\(", "lpt_scatter": r"lpt_scatter\(",
    "lpt3_hist": r"lpt3_hist\(", "lpt3_scan": r"lpt3_scan\(", "lpt3_scatter": r"lpt3_scatter\(",
    "astar2d_kernel": r"astar2d_kernel<",
    "dwa_kernel": r"dwa_kernel\(",
    "rrt_kernel": r"rrt_kernel<",
    "astar3d_kernel": r"astar3d_kernel[<(]",
    "dstar_kernel": r"dstar_kernel\(",
    "dstar3d_kernel": r"dstar3d_kernel<",
    "lpa_kernel": r"lpa_kernel\(",
    "lpa3d_kernel": r"lpa3d_kernel\(",
    "track_kernel_lqr": r"track_kernel<0>",
    "track_kernel_mpc": r"track_kernel<1>",
    "totp3d_kernel": r"totp3d_kernel\(",
}


# the 2D graph kernel's template <HEUR, GZERO, THETA> (astar2d.hip): one short name per planner, so the
# headline's traffic is never taken from the Theta* launches of the same kernel template
_G2D = re.compile(r"astar2d_kernel<(\d+), (true|false), (\d)>")


def short(name):
    m = _G2D.search(name)
    if m:
        heur, gzero, theta = int(m.group(1)), m.group(2) == "true", int(m.group(3))
        if theta:
            return "theta2d_kernel" if theta == 1 else "lazy_theta2d_kernel"
        if gzero:
            return "gbfs2d_kernel"
        return "dijkstra2d_kernel" if (heur & 3) == 2 else "astar2d_kernel"
    for k, rx in KERNELS.items():
        if re.search(rx, name):
            return k
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    kt = os.path.join(src, "prof_kt", "run_results.db")
    rows = []
    if os.path.exists(kt):
        rows = kernel_stats(kt, dst)
    traffic_and_mfma(src, dst, rows)


def kernel_stats(kt, dst):
    db = sqlite3.connect(kt)
    # one row per (kernel, grid size): a planner launched with different batch sizes (e.g. the small
    # A* batches that build the control legs' global paths) gets separate statistics
    rows = list(db.execute("select name, grid_x, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                           "from kernels group by name, grid_x order by sum(duration) desc"))
    tot = sum(r[3] for r in rows) or 1.0
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_threads", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "percent"])
        for n, g, c, t, a, mn, mx in rows:
            w.writerow([short(n), g, c, f"{t:.0f}", f"{a:.0f}", f"{mn:.0f}", f"{mx:.0f}", f"{100.0 * t / tot:.3f}"])
    # per-dispatch durations of the headline kernel, in launch order (warmups first)
    with open(os.path.join(dst, "astar2d_dispatches.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "grid_threads", "duration_ns"])
        for i, (n, g, d) in enumerate(db.execute("select name, grid_x, duration from kernels where name like "
                                                "'%astar2d_kernel%' order by start")):
            if short(n) == "astar2d_kernel":
                w.writerow([i, g, d])
    return [(n, c, t, a, 100.0 * t / tot) for n, g, c, t, a, mn, mx in rows]


def traffic_and_mfma(src, dst, rows):
    traffic = {}
    for counter, sub in (("FETCH_SIZE", "prof_fetch"), ("WRITE_SIZE", "prof_write")):
        path = os.path.join(src, sub, "run_results.db")
        if not os.path.exists(path):
            continue
        d = sqlite3.connect(path)
        # the largest launch configuration of each kernel (the bench leg's own batch)
        for name, n, mean_kb in d.execute(
                "select kernel_name, count(*), avg(value) from counters_collection c where counter_name = ? "
                "and grid_size = (select max(grid_size) from counters_collection c2 where c2.kernel_name = "
                "c.kernel_name and c2.counter_name = c.counter_name) group by kernel_name", (counter,)):
            k = short(name)
            e = traffic.setdefault(k, {})
            e[f"{counter}_kib_per_dispatch"] = mean_kb
            e["dispatches"] = n
    for k, e in traffic.items():
        fb = e.get("FETCH_SIZE_kib_per_dispatch")
        wb = e.get("WRITE_SIZE_kib_per_dispatch")
        e["read_bytes_per_dispatch"] = None if fb is None else 2.0 * fb * 1024.0
        e["write_bytes_per_dispatch"] = None if wb is None else wb * 1024.0
        e["hbm_bytes_per_dispatch"] = (None if fb is None or wb is None
                                       else e["read_bytes_per_dispatch"] + e["write_bytes_per_dispatch"])
    traffic["_note"] = ("FETCH_SIZE doubled per MI355X_MICROARCH.md (calibrated for 16 B/lane streaming reads; "
                        "the planners' reads are scattered 4-16 B accesses, for which the guide gives no "
                        "calibration) and WRITE_SIZE as is; Infinity-Cache hits are counted by these counters")
    with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    # MFMA utilisation pass (rocprofv3's MfmaUtil expression: SQ_VALU_MFMA_BUSY_CYCLES summed over the
    # chip / (GRBM_GUI_ACTIVE x SIMDs), per dispatch)
    path = os.path.join(src, "prof_mfma", "run_results.db")
    if os.path.exists(path):
        d = sqlite3.connect(path)
        mf = {}
        for name, cn, n, avg in d.execute("select kernel_name, counter_name, count(*), avg(value) from "
                                          "counters_collection group by kernel_name, counter_name"):
            mf.setdefault(short(name), {})[cn] = avg
            mf[short(name)]["dispatches"] = n
        simds = 256 * 4
        for k, e in mf.items():
            if e.get("GRBM_GUI_ACTIVE"):
                e["mfma_util_pct"] = 100.0 * e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (e["GRBM_GUI_ACTIVE"] * simds)
        mf["_note"] = ("per-dispatch averages of the separate --pmc pass; mfma_util_pct = SQ_VALU_MFMA_BUSY_CYCLES / "
                       "(GRBM_GUI_ACTIVE x 1024 SIMDs) x 100 (rocprofv3 MfmaUtil)")
        with open(os.path.join(dst, "pmc_mfma.json"), "w") as f:
            json.dump(mf, f, indent=1, sort_keys=True)
        print("mfma", {k: v.get("mfma_util_pct") for k, v in mf.items() if not k.startswith("_")})
    for n, c, t, a, p in rows[:8]:
        print(f"{short(n):24s} calls {c:5d} avg {a / 1e6:12.3f} ms  {p:6.2f} %")
    print(json.dumps({k: v.get("hbm_bytes_per_dispatch") for k, v in traffic.items() if not k.startswith("_")}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
