"""Where the time goes on non-uniform data (production path): build vs k-NN, kernel counters.

    python scripts/nonuniform_stats.py [n] [k]

Per distribution (LSK_DISTS): build_index alone, the k-NN pass alone (best of 3 each,
events), and the kernel counters of one k-NN pass (evaluations, passes, failures).
"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dev = torch.device("cuda", 0)


def timed(fn, reps=3):
    fn()
    best, out = math.inf, None
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        out = fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best, out


for name in os.environ.get("LSK_DISTS", "uniform,clustered,planar,mixed_scale,tilted_plane,line").split(","):
    pts = datasets.GENERATORS[name](n, seed=5).to(dev)
    t_b, idx = timed(lambda: E.build_index(pts, grid=True))
    cfg = E.KnnConfig(k=k)
    hint2 = E.radius_hint(idx.box, idx.n, k)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    t_q, _ = timed(lambda: E.query(idx, cfg, hint2, final_out=out))
    st = E.KnnStats()
    E.query(idx, cfg, hint2, final_out=out, stats=st)
    c = st.counters
    w = max(c.get("waves", 1), 1)
    dec = idx.grid.decision() if idx.grid is not None else None
    print(f"{name} n={n} k={k}: build {t_b:.2f} ms, k-NN {t_q:.2f} ms ({n / (t_b + t_q) / 1e3:.0f} Mpts/s); "
          f"grid {dec}; kernels {st.kernels if hasattr(st, 'kernels') else ''}", flush=True)
    print("   counters:", {kk: (round(v / n, 2) if kk in ("evals", "hist_evals", "collect_evals") else v)
                          for kk, v in sorted(c.items())}, f"passes/wave {c.get('hist_passes', 0) / w:.2f}",
          flush=True)
    del pts, idx
    torch.cuda.empty_cache()
