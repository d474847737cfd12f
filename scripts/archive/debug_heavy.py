"""Diagnostics for unique points next to many equidistant copies (test_knn_heavy_duplicates)."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

for copies, k in [(60_000, 100), (20_000, 100), (5_000, 100), (60_000, 16), (2_000, 300)]:
    g = torch.Generator().manual_seed(11)
    base = torch.rand((3, 3), generator=g)
    heavy = base.repeat_interleave(copies, dim=0)
    uniq = torch.rand((512, 3), generator=g)
    n = heavy.shape[0] + 512
    p = torch.cat([heavy, uniq])[torch.randperm(n, generator=g)].contiguous()
    stats = E.KnnStats()
    got = E.knn_distances(p.to("cuda"), k, stats=stats).cpu()
    is_u = torch.isin(p[:, 0], uniq[:, 0])
    ref = K.finalize_distances(K.kth_cpu(p, p[is_u], k, math.inf))
    gu = got[is_u]
    bad = gu != ref
    print(f"copies={copies} k={k}: heavy nonzero {int((got[~is_u] != 0).sum())}, "
          f"unique mismatches {int(bad.sum())}/{int(is_u.sum())}", flush=True)
    if bad.any():
        i = bad.nonzero()[:5, 0]
        print("  got", gu[i].tolist(), "ref", ref[i].tolist(), flush=True)
        print("  stats", {a: b for a, b in stats.counters.items() if b and not a.startswith("prof")},
              flush=True)
