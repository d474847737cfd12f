"""Which queries does the 16-bit k-NN kernel hand to the exact backstop? (debugging)

    python scripts/fail_probe.py [n] [k] [dist ...]

Runs knn_distances once per distribution with the failure list kept (ops/kernels.py
FailWord.flist) and prints the failed queries' count, positions (distinct, bounding box)
and the k-th distances of a few of them (brute force on the device).
"""
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

CAUGHT = []
_orig = K.knn_gpu


def _wrap(qpts, *a, **kw):
    fw = _orig(qpts, *a, **kw)
    CAUGHT.append((qpts, fw))
    return fw


K.knn_gpu = _wrap
E.K.knn_gpu = _wrap


def main():
    n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    names = sys.argv[3:] or ["mixed_scale", "clustered"]
    dev = torch.device("cuda", 0)
    for name in names:
        pts = datasets.GENERATORS[name](n).to(dev)
        E.knn_distances(pts, k)  # warmup
        CAUGHT.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        E.knn_distances(pts, k)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        for qpts, fw in CAUGHT:
            if fw.count is None:
                continue
            c = int(fw.count.item())
            print(f"{name} k={k}: {dt * 1e3:.2f} ms, launch over {qpts.shape[0]} queries: {c} failed (cap {fw.cap})")
            if c == 0 or fw.flist is None:
                continue
            ids = fw.flist[:min(c, fw.cap)].long()
            q = qpts[:, :3][ids] if qpts.dim() == 2 else qpts.view(-1, 3)[ids]
            u = torch.unique(q, dim=0)
            print(f"  distinct positions {u.shape[0]}; box lo {q.min(0).values.tolist()} hi {q.max(0).values.tolist()}")
            print(f"  ids min {int(ids.min())} max {int(ids.max())}; first 8 positions {q[:8].tolist()}")
            for i in range(min(8, u.shape[0])):
                d2 = ((pts - u[i]) ** 2).sum(1)
                v, _ = torch.topk(d2, k, largest=False)
                nz = int((d2 == 0).sum())
                print(f"  q {u[i].tolist()}: copies {nz}, k-th d2 {float(v[-1]):.6g}, "
                      f"within 2x k-th radius {int((d2 <= 4 * v[-1]).sum())}")
        del pts
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
