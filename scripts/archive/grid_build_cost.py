"""Index build with / without the cell grid, and knn_distances end to end (GRID off / auto)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1]) if len(sys.argv) > 1 else 2e7)
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")


def t(fn, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


E.GRID = "auto"
print(f"n={n} k={k} build no grid {t(lambda: E.build_index(p)) * 1e3:.2f} ms,"
      f" with grid {t(lambda: E.build_index(p, grid=True)) * 1e3:.2f} ms", flush=True)
idx = E.build_index(p, grid=True)
print("grid level", None if idx.grid is None else idx.grid.level, flush=True)
for mode in ("off", "auto"):
    E.GRID = mode
    print(f"knn_distances GRID={mode}: {t(lambda: E.knn_distances(p, k)) * 1e3:.2f} ms", flush=True)
