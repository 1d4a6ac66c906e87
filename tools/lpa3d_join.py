"""Dev tool: join the LPAStar3D probe's per-query dumps (PMP_PROBE_OUT of a normal build: pushes,
expansions, peak |U|; of a PMP_STAMPS=2 build: cycles) -- cycles per expansion by peak |U|, and how
much of the launch the heaviest queries hold."""
import sys

import numpy as np

a = np.load(sys.argv[1])  # normal build
b = np.load(sys.argv[2])  # stamps2 build
nexp = a["n_expanded"].sum(axis=1).astype(np.float64)
maxn = a["counters"][:, 3]
cyc = b["counters"][:, 3].astype(np.float64)  # whole query
ok = nexp > 0
print(f"queries {len(nexp)}; total expansions {nexp.sum():.3e}; query cycles sum {cyc.sum():.3e}")
for lo, hi in [(0, 200), (200, 400), (400, 600), (600, 800), (800, 2000)]:
    m = ok & (maxn >= lo) & (maxn < hi)
    if m.any():
        print(f"peak |U| [{lo},{hi}): {m.sum():6d} queries, {nexp[m].sum() / nexp.sum():.3f} of expansions, "
              f"{cyc[m].sum() / cyc.sum():.3f} of cycles, {cyc[m].sum() / nexp[m].sum():.0f} cycles/expansion")
o = np.argsort(-cyc)
print("heaviest queries (cycles, ms at 2.38 GHz, expansions, peak |U|):")
for q in o[:8]:
    print(f"  {cyc[q]:.3e} {cyc[q] / 2.382e6:.1f} {nexp[q]:.0f} {maxn[q]}")
