"""Dev probe: the drop-in single-query path on the README grid (C1) -- kernel time by HIP events,
and with PMP_HIP_LIB=.../libpmp_hip_stamps.so the kernel's own cycle split (pop / 3x3 wait / push /
total, s_memtime) so that cycles per expansion and the effective clock can be read off."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from python_motion_planning_amd import _lib, batch, workloads as wl  # noqa: E402

torch.cuda.set_device(0)
occ = wl.readme_grid()
W, H = occ.shape
bits = batch.occ_bits_device(occ, torch)
s, g = np.array([[5, 5]], np.int32), np.array([[45, 25]], np.int32)
stamps = os.environ.get("PMP_HIP_LIB", "").endswith("stamps.so")
for eng in (0, 2):
    L, ctx = _lib.load_library(), _lib.context()
    _lib.check(ctx, L.pmp_astar2d_set_engine(ctx, eng, 0), "engine")
    ts = []
    for rep in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = batch.astar2d_batch((W, H), s, g, path_cap=2048, counters=True, occ_bits=bits, retry_overflow=False)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    c = r["counters"].cpu().numpy()[0]
    ne = int(r["n_expanded"][0])
    t = float(np.median(ts))
    line = f"engine {eng}: {t:.3f} ms median ({min(ts):.3f} min) for {ne} expansions: {t * 1e3 / ne:.2f} us/expansion"
    if stamps:
        line += (f"; cycles pop {c[0]} wait {c[1]} push {c[2]} total {c[3]} -> {c[3] / ne:.0f} cycles/expansion, "
                 f"clock ~{c[3] / (t * 1e-3) / 1e6:.0f} MHz if the kernel is the query")
    else:
        line += f"; pushes {c[0]} pops {c[1]}"
    print(line, flush=True)
    # host overhead of the drop-in
t0 = time.perf_counter()
import python_motion_planning_amd as pmp  # noqa: E402

env = pmp.Grid(W, H)
env.update({(int(x), int(y)) for x, y in np.argwhere(occ)})
pl = pmp.AStar((5, 5), (45, 25), env)
pl.plan()
walls = []
for _ in range(30):
    t0 = time.perf_counter()
    pl.plan()
    walls.append(time.perf_counter() - t0)
print(f"drop-in AStar.plan(): {np.median(walls) * 1e3:.3f} ms median", flush=True)
