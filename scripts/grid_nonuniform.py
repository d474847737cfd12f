"""How does the cell-grid kernel do on non-uniform data at a forced level?

    python scripts/grid_nonuniform.py [n] [levels ...]

Per distribution (LSK_DISTS, default clustered,planar,uniform) and grandchild level: the
index with the dense slot table at that level, the grid forced on (GRID=on) for the
k-NN pass, timed (best of 3 after a warmup) against the production choice (GRID=auto:
the rows kernel for these sets), with the kernel counters and a sampled oracle check.
"""
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import verify as V  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
levels = [int(a) for a in sys.argv[2:]] or [8, 9]
k = int(os.environ.get("LSK_K", "100"))
dev = torch.device("cuda", 0)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = math.inf
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best, out


for name in os.environ.get("LSK_DISTS", "clustered,planar,uniform").split(","):
    pts = datasets.GENERATORS[name](n, seed=5).to(dev)
    E.GRID = "auto"
    t_auto, ref = timed(lambda: E.knn_distances(pts, k))
    print(f"{name} n={n} k={k} production (GRID=auto, build + k-NN): {t_auto * 1e3:.1f} ms "
          f"= {n / t_auto / 1e6:.0f} Mpts/s", flush=True)
    for g in levels:
        E.GRID = "on"
        try:
            idx = E.build_index(pts, grid=True, grid_level=g)
        except Exception as e:  # noqa: BLE001
            print(f"  level {g}: build failed: {e}", flush=True)
            continue
        cfg = E.KnnConfig(k=k)
        hint2 = E.radius_hint(idx.box, idx.n, k)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        t_q, _ = timed(lambda: E.query(idx, cfg, hint2, final_out=out))
        st = E.KnnStats()
        E.query(idx, cfg, hint2, final_out=out, stats=st)
        c = st.counters
        chk = V.sampled_exact(SingleComm(dev), pts, out, 0, n, k, 256)
        bad_ref = int((out != ref).sum())
        print(f"  level {g} (grid): k-NN {t_q * 1e3:.1f} ms; evals/q {c.get('evals', 0) / n:.0f} "
              f"passes/wave {c.get('hist_passes', 0) / max(c.get('waves', 1), 1):.2f} "
              f"fallback {c.get('fallback_queries', 0)} fail {c.get('failed_lanes', 0)}; "
              f"oracle {chk['exact']}/{chk['samples']}; vs production {n - bad_ref}/{n} equal", flush=True)
        del idx
        torch.cuda.empty_cache()
    E.GRID = "auto"
    del pts
    torch.cuda.empty_cache()
