#!/usr/bin/env python3
"""Headline benchmark: Mpoints/s of k-th-NN distance (k=100) on 1B uniform float3.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points P] [--k K] [--variant V]

Launched by the driver as ``torch.distributed.run --nproc-per-node N bench.py --gpus N``
for N > 1 (one rank per GPU, RCCL over xGMI). Each rank owns the reference's
block partition [floor(P*r/N), floor(P*(r+1)/N)) of one global synthetic uniform-random
point set held in pinned host memory. One timed step = the BASELINE.md clock: host
points -> H2D -> (unordered variant) spatial redistribution + bucket-tree k-NN + halo
exchange + result return -> distances back in host memory. W untimed warmup steps, then
K steps bracketed by barrier + device sync; the max over ranks is reported.
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mpi_cuda_largescaleknn_amd.models.knn_engine import KnnConfig  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import refalgo as RA  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm, TorchComm  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import numa, trace  # noqa: E402

METRIC = "Mpoints/sec kNN-distance (k=100) on 1B float3 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no numbers


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--points", type=float, default=1e9)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--variant", choices=["unordered", "prepartitioned"], default="unordered")
    ap.add_argument("--mode", choices=["halo", "ring", "peer"], default="halo",
                    help="halo = MI355X pipeline; ring/peer = reference algorithm (ref-algo baseline)")
    ap.add_argument("--phases", action="store_true", help="print per-phase times (adds syncs)")
    ap.add_argument("--stats", action="store_true", help="collect k-NN kernel counters")
    ap.add_argument("--direct-out", type=int, default=-1,
                    help="1 = on one rank the k-NN kernel writes the distances straight into the "
                         "pinned host buffer over PCIe while it runs (no device-to-host copy after "
                         "it); 0 = device buffer + copy; -1 (default) = 1 when k >= 48 (where the "
                         "PCIe writes hide under the kernel, pipelines.direct_host_out_pays)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1 = capture the whole single-rank step (H2D, index build, k-NN, results "
                         "to host) in one HIP graph after the warmup and replay it per step; "
                         "0 = eager launches; -1 (default) = 1 on one GPU rank without --phases/--stats")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = rehearsal of the launch/timing contract (gloo, CPU oracle); "
                         "never a measurement")
    return ap.parse_args()


def make_points(n_total: int, rank: int, size: int, device, variant: str) -> torch.Tensor:
    """This rank's slice of the global synthetic set, in pinned host memory."""
    b = n_total * rank // size
    e = n_total * (rank + 1) // size
    n = e - b
    g = torch.Generator(device=device)
    g.manual_seed(1234 + rank)
    host = torch.empty((n, 3), dtype=torch.float32, pin_memory=device.type == "cuda")
    chunk = 1 << 26
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        d = torch.rand((m, 3), generator=g, device=device, dtype=torch.float32)
        if variant == "prepartitioned":
            # spatially tiled files: rank r owns the slab [r/size, (r+1)/size) in x
            d[:, 0] = (d[:, 0] + rank) / size
        host[s:s + m].copy_(d)
    _sync(device)
    return host


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device == "cuda":
        # one rank per GPU (ranks beyond the device count wrap: rehearsals with
        # LSKNN_DIST_BACKEND=gloo only, RCCL refuses two ranks on one GPU)
        dev_id = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev_id)
        device = torch.device("cuda", dev_id)
        # host side (pinned input/output buffers) on the GPU's NUMA node
        bound = numa.bind_to_device(device)
        if bound and args.phases:
            print(f"rank {rank}: bound to {bound}", file=sys.stderr)
    else:
        device = torch.device("cpu")
    if world > 1:
        if device.type == "cuda" and os.environ.get("LSKNN_DIST_BACKEND", "nccl") == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
        comm = TorchComm(device)
    else:
        comm = SingleComm(device)
    n_total = int(args.points)
    cfg = KnnConfig(k=args.k, collect_stats=args.stats)

    host_pts = make_points(n_total, rank, world, device, args.variant)
    host_out = torch.empty(host_pts.shape[0], dtype=torch.float32, pin_memory=device.type == "cuda")

    info_last = None
    direct = (PL.direct_host_out_pays(args.k) if args.direct_out < 0 else bool(args.direct_out)) \
        and world == 1 and device.type == "cuda"

    def step():
        with trace.range("lsknn:step"):
            _step()
            _sync(device)

    def _step():
        nonlocal info_last
        info = PL.RunInfo(PL.PhaseTimer(args.phases, device))
        pts = host_pts.to(device, non_blocking=True)
        if args.mode == "ring":
            out = RA.ring_knn(pts, comm, cfg, info)
        elif args.mode == "peer":
            out = RA.peer_knn(pts, comm, cfg, info)
        elif args.variant == "unordered":
            out = PL.unordered_knn(pts, comm, cfg, info, n_total=n_total,
                                   out=host_out if direct else None)
        else:
            out = PL.prepartitioned_knn(pts, comm, cfg, info, out=host_out if direct else None)
        if out.data_ptr() != host_out.data_ptr():
            host_out.copy_(out, non_blocking=True)
        info_last = info

    use_graph = (args.graph == 1 or (args.graph < 0 and not (args.phases or args.stats))) \
        and world == 1 and device.type == "cuda" and args.mode == "halo"
    graph = None
    if use_graph:
        # warm up on a side stream (allocator + library state), then capture one whole
        # step — every launch and both host copies — into a graph replayed per step: the
        # single-rank pipeline has no host round trip (device-side radius hint), so the
        # replay does the same work as an eager step minus the per-launch CPU overhead
        side = torch.cuda.Stream(device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            for _ in range(max(1, args.warmup)):
                _step()
        torch.cuda.current_stream(device).wait_stream(side)
        _sync(device)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            _step()
        _sync(device)

        def step():  # noqa: F811 — graph replay replaces the eager step
            with trace.range("lsknn:step"):
                graph.replay()
                _sync(device)
    else:
        for _ in range(args.warmup):
            step()
    comm.barrier()
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    comm.barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    comm.allreduce_(t, "max")
    elapsed = float(t.item())

    ms = elapsed / args.steps * 1e3
    value = n_total * args.steps / elapsed / 1e6
    # sanity: distances must be finite and positive for uniform data with k <= n
    finite = bool(torch.isfinite(host_out).all()) if host_out.numel() else True
    if rank == 0:
        if args.phases or args.stats:
            print(json.dumps({"phases_s": info_last.timer.times, "counts": info_last.counts,
                              "knn_stats": info_last.stats.counters}), file=sys.stderr)
        rec = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "fp32",
            "data": "synthetic uniform-random float3 in [0,1)^3 (pinned host memory), no file I/O",
            "config": {
                "model": f"{args.variant}Data k-th-NN distance, k={args.k}",
                "global_batch": n_total,
                "seq_len": None,
                "parallelism": (f"ref-algo {args.mode} x{world}" if args.mode != "halo" else
                                f"spatial-redistribute+halo x{world}" if args.variant == "unordered"
                                else f"halo x{world}"),
                "k": args.k,
                "hip_graph": graph is not None,
                "all_finite": finite,
            },
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
