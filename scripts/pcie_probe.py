#!/usr/bin/env python3
"""Fixed-cost probe of the 1-GPU bench step (everything but the k-NN kernel):
H2D of the points, D2H of the results, the result scatter (to device memory and
straight into pinned host memory), keys and sort.

    python scripts/pcie_probe.py [--points 1e9]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402


def timed(name, fn, reps=2):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    print(f"{name:40s} {best * 1e3:9.2f} ms", flush=True)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=float, default=1e9)
    a = ap.parse_args()
    n = int(a.points)
    dev = torch.device("cuda", 0)
    host = torch.empty((n, 3), dtype=torch.float32, pin_memory=True)
    host_out = torch.empty(n, dtype=torch.float32, pin_memory=True)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    dpts = torch.rand((n, 3), generator=g, device=dev)
    host.copy_(dpts)
    torch.cuda.synchronize()
    gb = n * 12 / 1e9
    t = timed("H2D points (one copy)", lambda: dpts.copy_(host, non_blocking=True))
    print(f"   {gb / t:.1f} GB/s")

    streams = [torch.cuda.Stream() for _ in range(4)]

    def h2d4():
        cur = torch.cuda.current_stream()
        ch = (n + 3) // 4
        for i, s in enumerate(streams):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                dpts[i * ch:(i + 1) * ch].copy_(host[i * ch:(i + 1) * ch], non_blocking=True)
        for s in streams:
            cur.wait_stream(s)
    t = timed("H2D points (4 streams)", h2d4)
    print(f"   {gb / t:.1f} GB/s")

    d2 = torch.rand(n, generator=g, device=dev)
    out = torch.empty(n, dtype=torch.float32, device=dev)
    t = timed("D2H results", lambda: host_out.copy_(out, non_blocking=True))
    print(f"   {n * 4 / 1e9 / t:.1f} GB/s")

    box = K.bounds(dpts)
    keys = [None]

    def mk():
        keys[0] = K.morton(dpts, box)
    timed("keys (hilbert + iota)", mk)
    kk, iota = keys[0]
    srt = [None]

    def so():
        srt[0] = K.sort_pairs(kk, iota, 30)
    timed("sort_pairs 30-bit", so)
    perm = srt[0][1]
    del kk, iota, srt
    timed("gather3", lambda: K.gather3(dpts, perm, pad=K.PAD_POINTS))
    timed("scatter1 finalize -> device", lambda: K.scatter1(d2, perm, out, finalize=True))
    timed("scatter1 finalize -> pinned host", lambda: K.scatter1(d2, perm, host_out, finalize=True))
    ref = torch.empty(n, dtype=torch.float32, device=dev)
    K.scatter1(d2, perm, ref, finalize=True)
    torch.cuda.synchronize()
    print("host scatter equal:", bool(torch.equal(host_out.to(dev), ref)))


if __name__ == "__main__":
    main()
