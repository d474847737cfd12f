"""Data tools (SURVEY §7.1 lsknn_gen / lsknn_split / lsknn_check):

    python -m mpi_cuda_largescaleknn_amd.apps.tools gen   out.float3 -n N [--dist uniform|clustered] [--seed S]
    python -m mpi_cuda_largescaleknn_amd.apps.tools split in.float3 -p P -o prefix [--spatial]
           -> prefix_%06d.float3 + prefix.list (contiguous blocks, or spatial x-slabs)
    python -m mpi_cuda_largescaleknn_amd.apps.tools check in.float3 dist.float -k K [-r R] [--samples S]
           -> exact CPU oracle on sampled points, bitwise compare (replaces the reference's
              disabled '#if 0' RES dump, unorderedDataVariant.cu:215-227)
    python -m mpi_cuda_largescaleknn_amd.apps.tools cat prefix P out.float  (concatenate per-rank outputs)
    python -m mpi_cuda_largescaleknn_amd.apps.tools cmp a.float b.float
"""
from __future__ import annotations

import argparse
import math
import sys

import torch

from ..models.knn_engine import cut2_of
from ..ops import kernels as K
from ..utils import io


def gen(a) -> int:
    g = torch.Generator().manual_seed(a.seed)
    n = int(a.n)
    chunk = 1 << 24
    out = torch.empty((n, 3), dtype=torch.float32)
    if a.dist == "uniform":
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            out[s:s + m] = torch.rand((m, 3), generator=g)
    else:
        centers = torch.rand((max(1, a.clusters), 3), generator=g)
        for s in range(0, n, chunk):
            m = min(chunk, n - s)
            w = torch.randint(0, centers.shape[0], (m,), generator=g)
            out[s:s + m] = centers[w] + a.sigma * torch.randn((m, 3), generator=g)
    io.write_points(a.out, out)
    print(f"wrote {n} points to {a.out}")
    return 0


def split(a) -> int:
    pts = io.read_points(a.inp)
    n = pts.shape[0]
    names = []
    if a.spatial:
        order = torch.argsort(pts[:, 0], stable=True)
    for r in range(a.p):
        b, e = n * r // a.p, n * (r + 1) // a.p
        part = pts[order[b:e]] if a.spatial else pts[b:e]
        name = f"{a.out}_{r:06d}.float3"
        io.write_points(name, part)
        names.append(name)
    with open(a.out + ".list", "w") as f:
        f.write("\n".join(names) + "\n")
    if a.spatial:
        torch.save(order.to(torch.int64), a.out + ".order.pt")
    print(f"wrote {a.p} files and {a.out}.list")
    return 0


def check(a) -> int:
    pts = io.read_points(a.inp)
    dist = io.read_floats(a.dist_file)
    n = pts.shape[0]
    if dist.shape[0] != n:
        print(f"size mismatch: {dist.shape[0]} distances for {n} points")
        return 1
    g = torch.Generator().manual_seed(0)
    idx = torch.randint(0, n, (min(a.samples, n),), generator=g) if a.samples < n else torch.arange(n)
    ref = K.finalize_distances(K.kth_cpu(pts, pts[idx], a.k, cut2_of(a.r), "kdtree"))
    got = dist[idx]
    bad = int((got != ref).sum())
    print(f"checked {idx.numel()} sampled points: {bad} mismatches")
    for i in (got != ref).nonzero().flatten()[:10].tolist():
        print(f"RES {int(idx[i]):012d} = {got[i].item()!r} (oracle {ref[i].item()!r})")
    return 0 if bad == 0 else 1


def cat(a) -> int:
    parts = [io.read_floats(f"{a.prefix}_{r:06d}.float") for r in range(a.p)]
    out = torch.cat(parts)
    if a.order:
        order = torch.load(a.order, weights_only=True)
        full = torch.empty_like(out)
        full[order] = out
        out = full
    io.write_floats(a.out, out)
    print(f"wrote {out.shape[0]} distances to {a.out}")
    return 0


def cmp(a) -> int:
    x, y = io.read_floats(a.a), io.read_floats(a.b)
    if x.shape != y.shape:
        print(f"different sizes {x.shape[0]} vs {y.shape[0]}")
        return 1
    same = (x == y) | (torch.isnan(x) & torch.isnan(y))
    nbad = int((~same).sum())
    print("identical" if nbad == 0 else f"{nbad} differing values")
    return 0 if nbad == 0 else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="lsknn-tools")
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("gen")
    p.add_argument("out")
    p.add_argument("-n", type=float, required=True)
    p.add_argument("--dist", choices=["uniform", "clustered"], default="uniform")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--clusters", type=int, default=100)
    p.add_argument("--sigma", type=float, default=0.01)
    p = sub.add_parser("split")
    p.add_argument("inp")
    p.add_argument("-p", type=int, required=True)
    p.add_argument("-o", dest="out", required=True)
    p.add_argument("--spatial", action="store_true")
    p = sub.add_parser("check")
    p.add_argument("inp")
    p.add_argument("dist_file")
    p.add_argument("-k", type=int, required=True)
    p.add_argument("-r", type=float, default=math.inf)
    p.add_argument("--samples", type=int, default=10000)
    p = sub.add_parser("cat")
    p.add_argument("prefix")
    p.add_argument("p", type=int)
    p.add_argument("out")
    p.add_argument("--order", default=None, help="order file written by split --spatial")
    p = sub.add_parser("cmp")
    p.add_argument("a")
    p.add_argument("b")
    a = ap.parse_args(argv)
    return {"gen": gen, "split": split, "check": check, "cat": cat, "cmp": cmp}[a.cmd](a)


if __name__ == "__main__":
    sys.exit(main())
