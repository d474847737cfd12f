"""k-NN kernel time of the cell-grid pass at forced grid levels (uniform points).

    python scripts/grid_level_sweep.py N [k] [level ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
auto = E.grid_level_for(n, n)
levels = [int(x) for x in sys.argv[3:]] or [auto - 1, auto, auto + 1]
E.GRID = "on"
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
cfg = E.KnnConfig(k=k)
ref = None
for lvl in levels:
    if lvl > 10:
        continue
    idx = E.build_index(p, grid=True, grid_level=lvl)
    hint2 = E.radius_hint(idx.box, n, k)
    best = 1e9
    for r in range(3):
        st = E.KnnStats()
        torch.cuda.synchronize()
        t = time.perf_counter()
        d2 = E.query(idx, cfg, hint2, stats=st if r == 0 else None)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
        if r == 0:
            c = st.counters
    if ref is None:
        ref = d2
    same = bool(torch.equal(d2, ref))
    print(f"n={n} k={k} level {lvl}{' (auto)' if lvl == auto else ''}: {best:.4f} s  evals/query "
          f"{c.get('evals', 0) / n:.0f}  equal={same}", flush=True)
    del idx, d2
    torch.cuda.empty_cache()
