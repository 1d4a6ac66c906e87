"""The `nccl` (= RCCL) branch of shard.init with the product kernels: one rank
process initialises an RCCL group on cuda:0, plans one batch through batch.astar2d_sharded /
astar3d_sharded (longest-first deal + one all_gather per record field over RCCL) and compares the
gathered records with the direct single-launch results; barrier and max_over_ranks run over RCCL too.
A one-GPU box cannot hold two RCCL ranks (RCCL refuses two ranks on one device), so world size is 1:
the collectives are real RCCL calls on device buffers, the deal is the identity."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

_CHILD = r"""
import os, numpy as np, torch
from python_motion_planning_amd import batch, shard, workloads as wl
dist = shard.init("nccl", always=True)
assert dist is not None and dist.get_backend() == "nccl" and dist.get_world_size() == 1
occ = wl.random_grid(96, 96, 0.2, seed=11)
cells = wl.largest_component_cells(occ)
rng = np.random.default_rng(12)
s = cells[rng.integers(0, len(cells), 200)].astype(np.int32)
g = cells[rng.integers(0, len(cells), 200)].astype(np.int32)
full = batch.astar2d_sharded(occ, s, g, dist=dist, path_cap=4096)
ref = batch.astar2d_batch(occ.shape, s, g, path_cap=4096, occ_bits=batch.occ_bits_device(occ, torch))
for k in ("cost", "path_len", "n_expanded", "status"):
    a, b = full[k].cpu(), ref[k].cpu()
    assert torch.equal(a, b), k
n = int(full["path_len"].max())
assert torch.equal(full["path"][:, :n].cpu(), ref["path"][:, :n].cpu())
shard.barrier(dist)
(m,) = shard.max_over_ranks(dist, [3.5], "cuda")
assert m == 3.5
occ3 = np.zeros((12, 10, 8), np.uint8); occ3[6, 2:8, 1:7] = 1
s3 = np.array([[1, 1, 1], [2, 8, 6], [10, 4, 3]] * 20, np.int32)
g3 = np.array([[10, 8, 6], [10, 1, 1], [1, 5, 5]] * 20, np.int32)
f3 = batch.astar3d_sharded(occ3, s3, g3, dist=dist, path_cap=512)
r3 = batch.astar3d_batch(occ3, s3, g3, path_cap=512)
for k in ("cost", "path_len", "status"):
    assert torch.equal(f3[k].cpu(), r3[k].cpu()), k
dist.destroy_process_group()
print("RCCL-OK", int((full["status"] == 0).sum()))
"""


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_sharded_entry_points_over_rccl():
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), PYTHONPATH=repo)
    p = subprocess.run([sys.executable, "-c", _CHILD], cwd=repo, env=env, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "RCCL-OK" in p.stdout
