"""MFMA vs VALU screening A/B (scripts/micro/screen_ab.hip) on the production data layout.

    python scripts/mfma_screen_ab.py [--points 1e8] [--steps 64] [--k 100]

Points are curve-sorted by the engine's index build; every point is a query whose
threshold is its true k-th squared distance times --scale (2.8 ~ the pass-1 range top,
1.0 ~ the collect band). Prints per mode the time, (query, candidate) pairs per second and
the kept fraction, plus the MFMA screen's violation count (must be 0), as one JSON line.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_cuda_largescaleknn_amd import _native  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402


def run(pts, thr, steps, mode, out, viol):
    lib = _native.hip()
    K.check(lib.lsk_hip_screen_ab(pts.data_ptr(), pts.shape[0], thr.data_ptr(), steps, mode, out.data_ptr(),
                                  viol.data_ptr(), K._stream(pts)), "screen_ab")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=float, default=1e8)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--scale", type=float, nargs="+", default=[2.8, 1.0])
    a = ap.parse_args()
    n = int(a.points) // 64 * 64
    g = torch.Generator(device="cuda").manual_seed(7)
    p = torch.rand((n, 3), device="cuda", generator=g)
    idx = E.build_index(p)
    sp = idx.pts[:n].contiguous()
    d = E.knn_distances(sp, a.k)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    viol = torch.zeros(1, dtype=torch.int32, device="cuda")
    res = {"n": n, "steps": a.steps, "k": a.k, "modes": {}}
    for sc in a.scale:
        thr = (d.double() ** 2 * sc).float().contiguous()
        row = {}
        for mode, name in ((0, "valu"), (1, "mfma")):
            run(sp, thr, a.steps, mode, out, viol)  # warm
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(sp, thr, a.steps, mode, out, viol)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) / 1e3)
            kept = int(out.long().sum())
            pairs = n * 16 * a.steps
            row[name] = {"s": round(min(ts), 4), "Gpairs_s": round(pairs / min(ts) / 1e9, 1),
                         "kept_frac": round(kept / pairs, 4)}
        viol.zero_()
        run(sp, thr, a.steps, 2, out, viol)
        torch.cuda.synchronize()
        row["mfma_violations"] = int(viol.item())
        row["mfma_over_valu_time"] = round(row["mfma"]["s"] / row["valu"]["s"], 3)
        res["modes"][f"thr_x{sc}"] = row
        print(sc, row, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
