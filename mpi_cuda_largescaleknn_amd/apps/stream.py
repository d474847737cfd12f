"""hipKNN_stream — k-th-NN distances of a stream of independent float3 files.

    hipKNN_stream <a.float3> [<b.float3> ...] -o <prefix> -k <k> [-r <maxRadius>]
                  [--device auto|cuda|cpu] [-v]

Every input file is its own point set (unorderedData semantics: rank r of P reads the
block [floor(N*r/P), floor(N*(r+1)/P)) of each file) and gets its own output
<prefix>_<i:06d>.float with N float32 distances in input order — the same bytes as
running hipKNN_unorderedData on that file alone. The sets go through
parallel/stream.py's SetStream: set i+1's upload overlaps set i's k-NN (and set i's
result download overlaps set i+1). Files are read when the stream reaches them and each
output block is written as soon as its set is done, so only ~3 sets hold pinned host
memory at any time. Launch like the other apps (one process per GPU: torchrun, mpirun, or
a single process).
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


class _LazySets:
    """Input blocks / output buffers of the stream, read or allocated on first access and
    released by `drop` (SetStream's on_done): only the ~3 sets in flight hold pinned host
    memory, however long the stream."""

    def __init__(self, files, launch, gpu):
        self.files, self.launch, self.gpu = files, launch, gpu
        self.pts: dict = {}
        self.out: dict = {}
        self.meta: dict = {}

    def __len__(self):
        return len(self.files)

    def load(self, i):
        if i not in self.pts:
            pts, begin, total = io.read_portion(self.files[i], self.launch.rank, self.launch.size,
                                                pin_memory=self.gpu)
            self.pts[i] = pts
            self.meta[i] = (begin, total)
        return self.pts[i]

    def output(self, i):
        if i not in self.out:
            self.out[i] = torch.empty(self.load(i).shape[0], dtype=torch.float32, pin_memory=self.gpu)
        return self.out[i]

    def drop(self, i):
        self.pts.pop(i, None)
        self.out.pop(i, None)


class _View:
    def __init__(self, n, get):
        self.n, self.get = n, get

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return self.get(i)


def _run(a, launch) -> int:
    gpu = launch.device.type == "cuda"
    sets = _LazySets(a.inputs, launch, gpu)
    # global sizes from the file sizes (no data read): rank 0 creates every output file at
    # its final length up front, so each rank can write its block as soon as a set is done
    totals = [io.portion(f, 0, 1)[2] for f in a.inputs]
    print(f"#{launch.rank}/{launch.size}: got {len(a.inputs)} point sets to work on", flush=True)
    names = [f"{a.prefix}_{i:06d}.float" for i in range(len(a.inputs))]
    if launch.rank == 0:
        for name, total in zip(names, totals):
            io.write_floats(name, torch.empty(0, dtype=torch.float32), 0, truncate=True, total_records=total)
    launch.comm.barrier()
    cfg = KnnConfig(k=a.k, max_radius=a.max_radius)

    def on_done(i):
        # set i is complete in host memory: write this rank's block (pwrite at its record
        # offset, the reference's serialized append in parallel) and release the buffers
        begin, _ = sets.meta[i]
        io.write_floats(names[i], sets.out[i], begin, truncate=False)
        sets.drop(i)

    t0 = common.now(launch)
    SetStream(launch.comm, cfg, direct_out=gpu and PL.direct_host_out_pays(cfg.k)).run(
        _View(len(sets), sets.load), _View(len(sets), sets.output), totals, on_done=on_done)
    t1 = common.now(launch)
    print("done all queries...", flush=True)
    launch.comm.barrier()
    if a.verbose and launch.rank == 0:
        n = sum(totals)
        print(f"stream of {len(sets)} sets: {t1 - t0:.3f}s  {n / max(t1 - t0, 1e-9) / 1e6:.1f} Mpts/s", flush=True)
    L.finalize(launch)
    return 0


if __name__ == "__main__":
    sys.exit(main())
