"""Throughput and sampled exactness of the single-GPU k-th-NN path on non-uniform data.

    python scripts/dist_robustness.py [n] [k ...]

For each distribution of tests/datasets.py (uniform, clustered, duplicates, planar,
mixed_scale) at n points: times knn_distances (index build + kernel, 2 runs, the second
reported), then checks 4096 random queries against a float64 brute force over all n
points (relative error <= 1e-6; the bitwise oracle comparison lives in the GPU tests at
smaller n). Prints one line per (distribution, k) and a JSON summary line.
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402


def sampled_check(pts, got, k, nq=4096, seed=7):
    g = torch.Generator().manual_seed(seed)
    qi = torch.randint(0, pts.shape[0], (nq,), generator=g).to(pts.device)
    q = pts[qi].double()
    kk = min(k, pts.shape[0])
    refs = []
    for qs in range(0, nq, 64):
        qq = q[qs:qs + 64]
        best = None
        for s in range(0, pts.shape[0], 1 << 20):
            c = pts[s:s + (1 << 20)].double()
            d2 = ((qq[:, None, :] - c[None, :, :]) ** 2).sum(-1)
            part = torch.topk(d2, min(kk, d2.shape[1]), dim=1, largest=False).values
            best = part if best is None else torch.topk(torch.cat([best, part], 1), kk, dim=1,
                                                        largest=False).values
        refs.append(best[:, kk - 1].sqrt())
    ref = torch.cat(refs)
    g_ = got[qi].double()
    err = torch.where(ref > 0, (g_ - ref).abs() / ref.clamp_min(1e-300), g_.abs())
    return float(err.max())


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
    ks = [int(a) for a in sys.argv[2:]] or [100, 16]
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    rows = []
    names = os.environ.get("LSK_DISTS", "uniform,clustered,duplicates,planar,mixed_scale").split(",")
    for name in names:
        pts = datasets.GENERATORS[name](n).to(dev)
        for k in ks:
            for _ in range(2):
                _sync(dev)
                t0 = time.perf_counter()
                got = E.knn_distances(pts, k)
                _sync(dev)
                dt = time.perf_counter() - t0
            err = sampled_check(pts, got, k)
            row = {"dist": name, "n": n, "k": k, "s": round(dt, 4),
                   "Mpts_s": round(n / dt / 1e6, 1), "max_rel_err": err,
                   "finite": bool(torch.isfinite(got).all())}
            rows.append(row)
            print(row, flush=True)
        del pts
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
