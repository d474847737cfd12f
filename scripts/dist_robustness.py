"""Throughput and sampled exactness of the single-GPU k-th-NN path on non-uniform data.

    python scripts/dist_robustness.py [n] [k ...]

For each distribution of tests/datasets.py (uniform, clustered, duplicates, planar,
mixed_scale) at n points: times knn_distances (index build + kernel; one warmup run,
then the best of LSK_REPS-1 runs), then checks 1024 sampled outputs for exactness by brute force over all n points
(utils/verify.py: the claimed float must be exactly sqrtf of the k-th smallest canonical
d2; the bitwise oracle comparison lives in the GPU tests at smaller n). Prints one line per (distribution, k) and a JSON summary line.
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
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import verify as V  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


REPS = int(os.environ.get("LSK_REPS", "4"))


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
    ks = [int(a) for a in sys.argv[2:]] or [100, 16]
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    rows = []
    names = os.environ.get("LSK_DISTS", "uniform,clustered,duplicates,planar,mixed_scale").split(",")
    for name in names:
        pts = datasets.GENERATORS[name](n).to(dev)
        for k in ks:
            dt = float("inf")
            for _ in range(REPS):  # best of REPS after one warmup run
                _sync(dev)
                t0 = time.perf_counter()
                got = E.knn_distances(pts, k)
                _sync(dev)
                dt = min(dt, time.perf_counter() - t0) if _ else dt
            chk = V.sampled_exact(SingleComm(dev), pts, got, 0, n, k, 1024)
            row = {"dist": name, "n": n, "k": k, "s": round(dt, 4),
                   "Mpts_s": round(n / dt / 1e6, 1), "exact": f"{chk['exact']}/{chk['samples']}",
                   "finite": bool(torch.isfinite(got).all())}
            rows.append(row)
            print(row, flush=True)
        del pts
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    print(json.dumps(rows))


if __name__ == "__main__":
    main()
