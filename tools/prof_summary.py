"""Summarise a round's rocprofv3 databases (tools/profile_round.sh) into profiles/<round>/:
  kernel_stats.csv            -- rocprofv3 --kernel-trace --stats of the default bench command, per kernel
  kernel_stats_workloads.csv  -- the same dispatches keyed per (workload, kernel) through the bench's
                                 launch manifest (bench.py: every C-ABI planner call is logged under
                                 the label of the leg that made it, in launch order)
  pmc_traffic.json            -- FETCH_SIZE / WRITE_SIZE per dispatch from the two --pmc passes, keyed
                                 per workload the same way ("workloads"), with the gfx950 correction of
                                 MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide streaming
                                 reads: doubled; WRITE_SIZE as is; both in KiB)
  pmc_mfma.json               -- MFMA busy cycles of the MPC pass
  pmc_issue.json              -- the SQ issue pass (SQ_INSTS_VALU / SALU / LDS, wave cycles, GRBM_GUI_ACTIVE)
                                 per dispatch, keyed per workload: valu_issue_frac = VALU instructions over
                                 1024 SIMDs x (GRBM_GUI_ACTIVE / 8 XCDs) / 2 (one wave64 VALU instruction per
                                 2 cycles per SIMD, MI355X_MICROARCH.md)
A kernel whose dispatch count in a database differs from its manifest total is not attributed (its
workload entries are left out, so bench.py reports traffic null rather than a mis-keyed number).
usage: python tools/prof_summary.py gpurun_out profiles/r3
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
    "dwa_kernel": r"\bdwa_kernel[<(]",
    "dwa_split_kernel": r"\bdwa_split_kernel[<(]",
    "rrt_kernel": r"\brrt_kernel[<(]",
    "astar3d_kernel": r"\bastar3d_kernel[<(]",
    "dstar_kernel": r"\bdstar_kernel[<(]",
    "dstar_rerun_kernel": r"\bdstar_rerun_kernel[<(]",
    "dstar3d_kernel": r"\bdstar3d_kernel[<(]",
    "lpa_kernel": r"\blpa_kernel[<(]",
    "lpa3d_kernel": r"\blpa3d_kernel[<(]",
    "track_kernel_lqr": r"track_kernel<0>",
    "track_kernel_mpc": r"track_kernel<1>",
    "track_mpc_step": r"\btrack_mpc_step\(",
    "track_mpc_solve": r"\btrack_mpc_solve\(",
    "lqr_control_kernel": r"\blqr_control_kernel[<(]",
    "mpc_control_kernel": r"\bmpc_control_kernel[<(]",
    "totp3d_kernel": r"\btotp3d_kernel[<(]",
}


# the 2D graph kernels' template <HEUR, GZERO, THETA> (astar2d.hip): one short name per planner, so the
# headline's traffic is never taken from the Theta* launches of the same kernel template
_G2D = re.compile(r"astar2d_kernel<(\d+), (true|false), (\d)(?:, (?:true|false))?>")  # 4th: LDS grid state
_MQ = re.compile(r"astar2d_(?:mqu?|sq)_kernel<(\d+), (true|false), (true|false)(?:, (\d))?>")  # multi- / single-query


def short(name):
    m = _G2D.search(name)
    if m:
        heur, gzero, theta = int(m.group(1)), m.group(2) == "true", int(m.group(3))
        if theta:
            return "theta2d_kernel" if theta == 1 else "lazy_theta2d_kernel"
        if gzero:
            return "gbfs2d_kernel"
        return "dijkstra2d_kernel" if (heur & 3) == 2 else "astar2d_kernel"
    m = _MQ.search(name)
    if m:  # the multi-query <HEUR, GZERO, T2LDS> and single-query <HEUR, GZERO, LDSG> engines: the
        # short names of the one-query-per-wave kernel (pmp_graph2d_batch picks among the three)
        heur, gzero, theta = int(m.group(1)), m.group(2) == "true", int(m.group(4) or 0)
        if theta:  # <HEUR | Theta* layout, false, T2LDS, THETA> (round 5)
            return "theta2d_kernel" if theta == 1 else "lazy_theta2d_kernel"
        return "gbfs2d_kernel" if gzero else ("dijkstra2d_kernel" if heur == 2 else "astar2d_kernel")
    for k, rx in KERNELS.items():
        if re.search(rx, name):
            return k
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]


def load_manifest(path):
    """[label, kernel, dispatches] in launch order, from a bench detail file (bench.py --detail-out)."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("launch_manifest")


def attribute(seq, manifest):
    """seq: [(short kernel name, record)] in dispatch order.  Returns ({label: [(kernel, record), ...]},
    {kernel: (seen, expected)} for the kernels that could not be attributed)."""
    by_k = {}
    for k, rec in seq:
        by_k.setdefault(k, []).append(rec)
    want = {}
    for label, k, n in manifest:
        want[k] = want.get(k, 0) + n
    bad = {k: (len(by_k.get(k, [])), n) for k, n in want.items() if len(by_k.get(k, [])) != n}
    pos = {k: 0 for k in want}
    out = {}
    for label, k, n in manifest:
        recs = by_k.get(k, [])[pos[k]: pos[k] + n]
        pos[k] += n
        if k in bad:
            continue
        out.setdefault(label, []).extend((k, r) for r in recs)
    return out, bad


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    kt = os.path.join(src, "prof_kt", "run_results.db")
    if os.path.exists(kt):
        kernel_stats(kt, dst, load_manifest(os.path.join(src, "prof_kt", "detail.json")))
    traffic_and_mfma(src, dst)
    issue(src, dst)


def kernel_stats(kt, dst, manifest):
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
    seq = [(short(n), d) for n, d in db.execute("select name, duration from kernels order by start")]
    with open(os.path.join(dst, "astar2d_dispatches.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["dispatch", "duration_ns"])
        for i, (k, d) in enumerate(x for x in seq if x[0] == "astar2d_kernel"):
            w.writerow([i, d])
    if manifest:
        per, bad = attribute(seq, manifest)
        with open(os.path.join(dst, "kernel_stats_workloads.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["workload", "kernel", "dispatches", "avg_ns", "min_ns", "max_ns"])
            for label, recs in per.items():
                for k in sorted({k for k, _ in recs}):
                    d = [r for kk, r in recs if kk == k]
                    w.writerow([label, k, len(d), f"{sum(d) / len(d):.0f}", f"{min(d):.0f}", f"{max(d):.0f}"])
        if bad:
            print("kernel trace: not attributed (seen, manifest):", bad)
    for n, g, c, t, a, mn, mx in rows[:8]:
        print(f"{short(n):24s} calls {c:5d} avg {a / 1e6:12.3f} ms  {100.0 * t / tot:6.2f} %")


def pmc_dispatches(path, counter):
    """[(short kernel name, value)] per dispatch in dispatch order for one counter of a --pmc pass."""
    d = sqlite3.connect(path)
    cols = [r[1] for r in d.execute("pragma table_info(counters_collection)")]
    order = "dispatch_id" if "dispatch_id" in cols else ("correlation_id" if "correlation_id" in cols else None)
    if order:
        q = (f"select kernel_name, sum(value) from counters_collection where counter_name = ? group by {order} "
             f"order by {order}")
    else:
        q = "select kernel_name, value from counters_collection where counter_name = ? order by rowid"
    return [(short(n), v) for n, v in d.execute(q, (counter,))], cols


def traffic_and_mfma(src, dst):
    kernels, workloads, unattributed = {}, {}, {}
    for counter, sub in (("FETCH_SIZE", "prof_fetch"), ("WRITE_SIZE", "prof_write")):
        path = os.path.join(src, sub, "run_results.db")
        if not os.path.exists(path):
            continue
        seq, cols = pmc_dispatches(path, counter)
        print(sub, "counters_collection columns:", cols)
        for k in {k for k, _ in seq}:
            v = [x for kk, x in seq if kk == k]
            e = kernels.setdefault(k, {})
            e[f"{counter}_kib_per_dispatch"] = sum(v) / len(v)
            e[f"{counter}_dispatches"] = len(v)
        manifest = load_manifest(os.path.join(src, sub, "detail.json"))
        if not manifest:
            continue
        per, bad = attribute(seq, manifest)
        unattributed[counter] = bad
        for label, recs in per.items():
            ks = {k for k, _ in recs}
            # a workload's own kernel: the one the leg is about (the setup A* path batches of the
            # control legs are labelled "setup", not with the leg's name)
            for k in ks:
                v = [x for kk, x in recs if kk == k]
                key = label if len(ks) == 1 else f"{label}:{k}"
                e = workloads.setdefault(key, {"kernel": k})
                e[f"{counter}_kib_per_dispatch"] = sum(v) / len(v)
                e[f"{counter}_dispatches"] = len(v)
    for e in list(kernels.values()) + list(workloads.values()):
        fb = e.get("FETCH_SIZE_kib_per_dispatch")
        wb = e.get("WRITE_SIZE_kib_per_dispatch")
        e["read_bytes_per_dispatch"] = None if fb is None else 2.0 * fb * 1024.0
        e["write_bytes_per_dispatch"] = None if wb is None else wb * 1024.0
        e["hbm_bytes_per_dispatch"] = (None if fb is None or wb is None
                                       else e["read_bytes_per_dispatch"] + e["write_bytes_per_dispatch"])
    out = {"workloads": workloads, "kernels": kernels, "unattributed": unattributed,
           "_note": ("per dispatch, keyed per workload through the bench's launch manifest; FETCH_SIZE doubled per "
                     "MI355X_MICROARCH.md (calibrated for 16 B/lane streaming reads; the planners' reads are "
                     "scattered 4-16 B accesses, for which the guide gives no calibration) and WRITE_SIZE as is; "
                     "Infinity-Cache hits are counted by these counters")}
    if kernels:
        with open(os.path.join(dst, "pmc_traffic.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
        print(json.dumps({k: v.get("hbm_bytes_per_dispatch") for k, v in workloads.items()}))
        if any(unattributed.values()):
            print("pmc: not attributed (seen, manifest):", unattributed)
    # MFMA utilisation pass: SQ_VALU_MFMA_BUSY_CYCLES summed over the chip / (GPU cycles x SIMDs), per
    # dispatch.  rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs (MI355X_MICROARCH.md, "DVFS
    # give-back": effective clock = GRBM_GUI_ACTIVE / 8 / wall time), so the dispatch's cycles are
    # GRBM_GUI_ACTIVE / 8; round 4 divided by the sum and under-reported utilisation 8x.
    path = os.path.join(src, "prof_mfma", "run_results.db")
    if os.path.exists(path):
        d = sqlite3.connect(path)
        mf = {}
        for name, cn, n, avg in d.execute("select kernel_name, counter_name, count(*), avg(value) from "
                                          "counters_collection group by kernel_name, counter_name"):
            mf.setdefault(short(name), {})[cn] = avg
            mf[short(name)]["dispatches"] = n
        mfma_util(mf)
        mf["_note"] = ("per-dispatch averages of the separate --pmc pass; mfma_util_pct = SQ_VALU_MFMA_BUSY_CYCLES / "
                       "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) x 100 (GRBM_GUI_ACTIVE is the sum over the 8 XCDs)")
        with open(os.path.join(dst, "pmc_mfma.json"), "w") as f:
            json.dump(mf, f, indent=1, sort_keys=True)
        print("mfma", {k: v.get("mfma_util_pct") for k, v in mf.items() if not k.startswith("_")})


XCDS, SIMDS = 8, 256 * 4
ISSUE_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY",
                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAVES", "GRBM_GUI_ACTIVE")


def issue(src, dst):
    """The SQ issue pass (tools/profile_round.sh, prof_issue): per dispatch sums of each counter, keyed
    per workload through the launch manifest like the traffic passes."""
    path = os.path.join(src, "prof_issue", "run_results.db")
    if not os.path.exists(path):
        return
    manifest = load_manifest(os.path.join(src, "prof_issue", "detail.json"))
    workloads, unattributed = {}, {}
    for counter in ISSUE_COUNTERS:
        seq, _ = pmc_dispatches(path, counter)
        if not seq or not manifest:
            continue
        per, bad = attribute(seq, manifest)
        if bad:
            unattributed[counter] = bad
        for label, recs in per.items():
            ks = {k for k, _ in recs}
            for k in ks:
                v = [x for kk, x in recs if kk == k]
                key = label if len(ks) == 1 else f"{label}:{k}"
                e = workloads.setdefault(key, {"kernel": k})
                e[f"{counter}_per_dispatch"] = sum(v) / len(v)
                e["dispatches"] = len(v)
    for e in workloads.values():
        valu, grbm = e.get("SQ_INSTS_VALU_per_dispatch"), e.get("GRBM_GUI_ACTIVE_per_dispatch")
        if valu is not None and grbm:
            cycles = grbm / XCDS
            e["gpu_cycles_per_dispatch"] = cycles
            e["valu_issue_frac"] = valu / (SIMDS * cycles / 2.0)
        wc = e.get("SQ_WAVE_CYCLES_per_dispatch")
        if wc:
            for c, name in (("SQ_ACTIVE_INST_ANY", "wave_issue_frac"), ("SQ_WAIT_ANY", "wave_wait_frac"),
                            ("SQ_WAIT_INST_ANY", "wave_issue_stall_frac")):
                if e.get(f"{c}_per_dispatch") is not None:
                    e[name] = e[f"{c}_per_dispatch"] / wc
    out = {"workloads": workloads, "unattributed": unattributed,
           "_note": ("per dispatch sums of the SQ issue pass (one rocprofv3 --pmc run of the short bench, the default "
                     "per-launch batch counts); valu_issue_frac = SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 "
                     "XCDs / 2): one wave64 VALU instruction per 2 cycles per SIMD (f64 and 64-bit-shift instructions "
                     "take longer, so this is a lower bound on the VALU pipe's busy time); wave_*_frac over "
                     "SQ_WAVE_CYCLES (all in quad-cycles, ratios unaffected)")}
    with open(os.path.join(dst, "pmc_issue.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("issue", {k: round(v.get("valu_issue_frac", 0.0), 4) for k, v in workloads.items()})
    if unattributed:
        print("issue: not attributed (seen, manifest):", unattributed)


def mfma_util(mf):
    """mfma_util_pct per kernel entry of a pmc_mfma dict (in place): MFMA busy cycles over the
    dispatch's GPU cycles (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs."""
    for k, e in mf.items():
        if isinstance(e, dict) and e.get("GRBM_GUI_ACTIVE"):
            cycles = e["GRBM_GUI_ACTIVE"] / XCDS
            e["gpu_cycles_per_dispatch"] = cycles
            e["mfma_util_pct"] = 100.0 * e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cycles * SIMDS)
    return mf


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
