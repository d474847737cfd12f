"""Run only the single-GPU local pipeline on N uniform points (for profiling)."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=float, default=1e8)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--impl", default="rows")
ap.add_argument("--seed", type=int, default=None)
ap.add_argument("--grid", type=int, default=0, help="1: cell-grid kernel (knn_grid.hip) for the pass")
a = ap.parse_args()
n = int(a.points)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
E.KNN_IMPL = a.impl
if a.seed is not None:
    E.SEED_BUCKETS = a.seed
if a.grid:
    E.GRID = "on"
idx = E.build_index(p, grid=bool(a.grid))
cfg = E.KnnConfig(k=a.k)
hint2 = E.radius_hint2(idx.box, n, a.k)
for r in range(a.reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    st = E.KnnStats()
    d2 = E.query(idx, cfg, hint2, stats=st if r == 0 else None)
    torch.cuda.synchronize()
    print(f"[{'grid' if idx.grid is not None else a.impl}] knn {n} pts k={a.k}: {time.perf_counter() - t:.3f} s", st.counters, flush=True)
    c = st.counters
    if c.get("prof_wave"):
        tot = c["prof_wave"]
        print("  cycle profile (% of wave time):", {k[5:]: round(100.0 * v / tot, 1)
                                                    for k, v in c.items() if k.startswith("prof_")}, flush=True)
