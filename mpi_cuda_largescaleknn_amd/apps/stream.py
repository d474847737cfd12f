"""hipKNN_stream — k-th-NN distances of a stream of independent float3 files.

    hipKNN_stream <a.float3> [<b.float3> ...] -o <prefix> -k <k> [-r <maxRadius>]
                  [--device auto|cuda|cpu] [-v]

Every input file is its own point set (unorderedData semantics: rank r of P reads the
block [floor(N*r/P), floor(N*(r+1)/P)) of each file) and gets its own output
<prefix>_<i:06d>.float with N float32 distances in input order — the same bytes as
running hipKNN_unorderedData on that file alone. The sets go through
parallel/stream.py's SetStream: set i+1's upload overlaps set i's k-NN (and, on several
ranks, set i's result download overlaps set i+1). Launch like the other apps (one
process per GPU: torchrun, mpirun, or a single process).
"""
from __future__ import annotations

import argparse
import math
import sys

import torch

from ..models.knn_engine import KnnConfig
from ..parallel import launch as L
from ..parallel import pipelines as PL
from ..parallel.stream import SetStream
from ..utils import io
from . import common


def parse(argv: list[str]) -> argparse.Namespace:
    ap = argparse.ArgumentParser(prog="hipKNN_stream")
    ap.add_argument("inputs", nargs="+", help="float3 files, one point set each")
    ap.add_argument("-o", dest="prefix", required=True, help="output prefix: <prefix>_<i:06d>.float")
    ap.add_argument("-k", type=int, required=True)
    ap.add_argument("-r", dest="max_radius", type=float, default=math.inf)
    ap.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto")
    ap.add_argument("-v", dest="verbose", action="store_true")
    a = ap.parse_args(argv)
    if a.k < 1:
        ap.error("-k must be at least 1")
    return a


def main(argv: list[str] | None = None) -> int:
    a = parse(list(sys.argv[1:] if argv is None else argv))
    launch = L.init(a.device, 0, a.verbose)
    return common.guarded(launch, lambda: _run(a, launch))


def _run(a, launch) -> int:
    gpu = launch.device.type == "cuda"
    ins, begins, totals = [], [], []
    for f in a.inputs:
        pts, begin, total = io.read_portion(f, launch.rank, launch.size, pin_memory=gpu)
        ins.append(pts)
        begins.append(begin)
        totals.append(total)
    print(f"#{launch.rank}/{launch.size}: got {len(ins)} point sets "
          f"({sum(int(p.shape[0]) for p in ins)} points) to work on", flush=True)
    cfg = KnnConfig(k=a.k, max_radius=a.max_radius)
    outs = [torch.empty(p.shape[0], dtype=torch.float32, pin_memory=gpu) for p in ins]
    t0 = common.now(launch)
    SetStream(launch.comm, cfg, direct_out=gpu and PL.direct_host_out_pays(cfg.k)).run(ins, outs, totals)
    t1 = common.now(launch)
    print("done all queries...", flush=True)
    for i, (res, begin, total) in enumerate(zip(outs, begins, totals)):
        name = f"{a.prefix}_{i:06d}.float"
        if launch.rank == 0:
            io.write_floats(name, res[:0], 0, truncate=True, total_records=total)
        launch.comm.barrier()
        io.write_floats(name, res, begin, truncate=False)
    launch.comm.barrier()
    if a.verbose and launch.rank == 0:
        n = sum(totals)
        print(f"stream of {len(ins)} sets: {t1 - t0:.3f}s  {n / max(t1 - t0, 1e-9) / 1e6:.1f} Mpts/s", flush=True)
    L.finalize(launch)
    return 0


if __name__ == "__main__":
    sys.exit(main())
