#!/usr/bin/env python3
"""Headline benchmark: Mpoints/s of k-th-NN distance (k=100) on 1B uniform float3.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--points P] [--k K] [--variant V]

Launched by the driver as ``torch.distributed.run --nproc-per-node N bench.py --gpus N``
for N > 1 (one rank per GPU, RCCL over xGMI; bootstrap through parallel/launch.init:
NUMA binding, collective timeout, watchdog, abort broadcast). Each rank owns the
reference's block partition [floor(P*r/N), floor(P*(r+1)/N)) of ONE global synthetic
uniform-random point set held in pinned host memory: the set is generated in chunks of
2^24 points seeded by the chunk's global index, so it is the same for every N and the
outputs at N = 1/2/4/8 are comparable bit for bit. One timed step = the BASELINE.md
clock: host points -> H2D -> (unordered variant) spatial redistribution + bucket-tree
k-NN + halo exchange + result return -> distances back in host memory. W untimed warmup
steps, then K steps bracketed by barrier + device sync; the max over ranks is reported.

Pipelined (--pipeline; default for the unordered halo pipeline on GPUs from 1e7
points): a stream of point sets — two different synthetic sets alternate step by step, and while
step i runs its k-NN on the compute stream, step i+1's points are copied host -> device
(PCIe H2D does not compete with the VALU-bound k-NN). Every step still uploads, builds, queries and
returns its whole set; the first set's upload is inside the timed region, and both sets'
last outputs are verified. ms_per_step is then the per-set time of the stream.

After the timed region (untimed): a brute-force check of 256 sampled outputs per verified
set against all points (utils/verify.py, `sampled_exact`); the SINGLE-SET LATENCY — one
set from pinned host memory through H2D, index build, k-NN and results back in host
memory, nothing overlapped with another set (the BASELINE.md clock for one problem; best
of two runs, max over ranks; `single_set_ms` / `single_set_mpts`); and one instrumented
step of the timed path (per-phase times with device syncs, max over ranks; halo sizes;
per-rank k-NN ms; pipelined: from device-resident points). Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# hardware queues per process: the HIP runtime reads this when torch loads it, so before
# `import torch`. The benchmark's configuration raises it to at least LSKNN_HW_QUEUES
# (default 8; the measured best, mpi_cuda_largescaleknn_amd/__init__.py) even over a lower
# value in the environment (the GPU box exports HIP's default, 4); the JSON records it.
def _int_env(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, "") or default)
    except ValueError:
        return default


HW_QUEUES = min(max(_int_env("GPU_MAX_HW_QUEUES", 4), _int_env("LSKNN_HW_QUEUES", 8)), 32)
os.environ["GPU_MAX_HW_QUEUES"] = str(HW_QUEUES)

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.models.knn_engine import KnnConfig  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import refalgo as RA  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import faults as FA  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import launch as LA  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.stream import SetStream  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import trace, verify  # noqa: E402

HEADLINE_METRIC = "Mpoints/sec kNN-distance (k=100) on 1B float3 at 1/2/4/8 MI355X"
GEN_CHUNK = 1 << 24  # points per seeded generation chunk (global index -> seed)
DATASET_STRIDE = 1_000_003  # seed offset of the second point set of the pipelined bench
PIPELINE_MIN_POINTS = 10**7  # --pipeline -1: stream of sets from this many points on
# "knn_local+halo_exchange": the overlapped form (pipelines.knn_with_halo) — the local k-NN
# and the halo publish/filter/exchange on a side stream end at one mark
PHASES = ["bounds", "partition", "alltoallv_points", "build", "knn_local", "knn_local+halo_exchange",
          "halo_publish", "halo_filter", "halo_alltoallv", "halo_tree", "halo_requery", "return"]
COUNTS = ["sent_points", "owned_points", "halo_sent", "halo_recv", "requery_groups"]


def metric_name(n_total: int, k: int) -> str:
    """The BASELINE.json metric for the headline config; the label follows --points/--k."""
    if n_total == 10**9 and k == 100:
        return HEADLINE_METRIC
    pts = f"{n_total / 1e9:g}B" if n_total >= 10**9 else f"{n_total / 1e6:g}M"
    return f"Mpoints/sec kNN-distance (k={k}) on {pts} float3 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no numbers
BENCH_TIMEOUT_S = 150  # progress timeout of every rank (LSKNN_TIMEOUT overrides)


def comm_info(comm) -> dict:
    """Which communicator moved the data and which RCCL library it runs."""
    inner = getattr(comm, "inner", comm)
    backend = getattr(inner, "backend", "single") if comm.distributed else "single"
    out = {"backend": backend, "rccl_version": None}
    if backend == "rccl":
        v = int(getattr(inner, "version", 0) or 0)  # NCCL_VERSION_CODE: major*10000+minor*100+patch
        out["rccl_version"] = f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v else None
        out["rccl_library"] = "ROCm librccl (native communicator, parallel/rccl.py)"
    elif backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            out["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001 - reporting only
            pass
        out["rccl_library"] = "torch.distributed ProcessGroupNCCL (torch's bundled librccl)"
    return out


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
                         "it); 0 = device buffer + one copy; -1 (default) = a lone set: the copy "
                         "when the cell grid is built (its kernel outruns the PCIe writes), the "
                         "direct writes for the bucket-tree kernel when k >= 48 "
                         "(pipelines.query_into); the stream of sets: 0 (the copy runs on a side "
                         "stream under the next set)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1 = capture the whole single-rank step (H2D, index build, k-NN, results "
                         "to host) in one HIP graph after the warmup and replay it per step; "
                         "0 = eager launches; -1 (default) = 1 on one GPU rank without --phases/--stats")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu = rehearsal of the launch/timing contract (gloo, CPU oracle); "
                         "never a measurement")
    ap.add_argument("--force-dist", action="store_true",
                    help="multi-rank pipeline and RCCL collectives even on one rank")
    ap.add_argument("--pipeline", type=int, default=-1,
                    help="1 = a stream of point sets: two different synthetic sets alternate step "
                         "by step, and the host-to-device copy of step i+1's points runs on a copy "
                         "stream under step i's k-NN (every step still uploads, builds, queries and "
                         "returns its whole set; the first upload is inside the timed region); "
                         "0 = one set, each step uploads then computes (on several ranks the upload "
                         "is streamed under the redistribution); -1 (default) = 1 for the unordered "
                         "halo pipeline on GPUs from 1e7 points")
    ap.add_argument("--verify", type=int, default=256,
                    help="sampled outputs checked by brute force after the timed region (0 = off)")
    return ap.parse_args()


def block_range(n_total: int, rank: int, size: int) -> tuple[int, int]:
    """The reference's readFilePortion partition (unorderedDataVariant.cu:42-63)."""
    return n_total * rank // size, n_total * (rank + 1) // size


def make_points(n_total: int, rank: int, size: int, device, variant: str, dataset: int = 0) -> torch.Tensor:
    """This rank's block of the global synthetic set number `dataset`, in pinned host
    memory. Chunk c of the global set (GEN_CHUNK points) always comes from seed
    1234 + c + DATASET_STRIDE * dataset, so the global set does not depend on the rank
    count (per device type)."""
    b, e = block_range(n_total, rank, size)
    host = torch.empty((e - b, 3), dtype=torch.float32, pin_memory=device.type == "cuda")
    if e > b:
        for c in range(b // GEN_CHUNK, (e - 1) // GEN_CHUNK + 1):
            c0 = c * GEN_CHUNK
            g = torch.Generator(device=device)
            g.manual_seed(1234 + c + DATASET_STRIDE * dataset)
            d = torch.rand((min(GEN_CHUNK, n_total - c0), 3), generator=g, device=device,
                           dtype=torch.float32)
            lo, hi = max(b, c0), min(e, c0 + GEN_CHUNK)
            part = d[lo - c0:hi - c0]
            if variant == "prepartitioned":
                # spatially tiled files: rank r owns the slab [r/size, (r+1)/size) in x
                part[:, 0] = (part[:, 0] + rank) / size
            host[lo - b:hi - b].copy_(part)
    _sync(device)
    return host


def _sync(device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def self_launch(args) -> int | None:
    """--gpus N without a launcher: start N local ranks of this script (the torchrun
    contract: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*; the reference's `mpirun -n P`,
    README.md:31,39) before anything touches the GPU, and return the first non-zero exit
    code (rank 0 prints the JSON line). Under a launcher its world size must equal --gpus.
    Returns None when this process is a rank and should run the benchmark."""
    if not LA.launcher_env():
        if args.gpus > 1:
            return LA.spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]])
        return None
    _, size, _ = LA.rank_info()
    if size != args.gpus:
        sys.stderr.write(f"bench.py: the launcher started {size} ranks but --gpus is {args.gpus}\n")
        return 2
    return None


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    # a hung collective ends the job (watchdog + collective timeout) long before the
    # driver's 600 s limit, and the watchdog names the rank and the collective it stalled
    # in ("#r/P: watchdog: timeout in alltoallv: ...") inside the tail the driver keeps; one
    # rank per GPU (ranks beyond the device count wrap: rehearsals with
    # LSKNN_DIST_BACKEND=gloo only, RCCL refuses two ranks on one GPU); pinned buffers on
    # the GPU's NUMA node
    os.environ.setdefault("LSKNN_TIMEOUT", str(BENCH_TIMEOUT_S))
    launch = LA.init(device_pref=args.device, force_distributed=args.force_dist or None,
                     verbose=args.phases)
    world, rank, device, comm = launch.size, launch.rank, launch.device, launch.comm
    if args.device == "cuda" and device.type != "cuda":
        raise RuntimeError("bench.py: no GPU available (use --device cpu for a rehearsal)")
    n_total = int(args.points)
    cfg = KnnConfig(k=args.k, collect_stats=args.stats)
    if args.mode != "halo":
        # the reference's heaps (N/P*k*8 B per rank) must fit before any point is made
        b0, e0 = block_range(n_total, rank, world)
        cap = (torch.cuda.get_device_properties(device).total_memory if device.type == "cuda"
               else int(float(os.environ.get("LSKNN_REF_CAPACITY_GB", "288")) * 1e9))
        try:
            RA.check_ref_fits(e0 - b0, args.k, cap, world)
        except ValueError as e:
            sys.stderr.write(f"bench.py: {e}\n")
            LA.finalize(launch)
            sys.exit(3)

    # pipelined stream of point sets (see --pipeline): two different synthetic sets alternate
    # (auto: from 1e7 points; below that one HIP-graph replay per set is cheaper than the
    # eager launches of the stream: 1e6 k=8 711 vs 702 Mpts/s, profiles/archive/r2_s3_table)
    pipelined = (args.pipeline == 1 or (args.pipeline < 0 and n_total >= PIPELINE_MIN_POINTS)) \
        and device.type == "cuda" and args.mode == "halo"
    with FA.HEARTBEAT.host_phase("make_points"):
        host_sets = [make_points(n_total, rank, world, device, args.variant, d) for d in range(2 if pipelined else 1)]
    host_outs = [torch.empty(h.shape[0], dtype=torch.float32, pin_memory=device.type == "cuda") for h in host_sets]
    host_pts, host_out = host_sets[0], host_outs[0]

    info_last = None
    graph_kernels: list = []
    # one GPU rank: the pinned output is passed down and pipelines.query_into picks direct
    # PCIe writes or device buffer + copy (--direct-out forces one)
    single_gpu = not comm.distributed and device.type == "cuda"
    direct = None if args.direct_out < 0 else bool(args.direct_out)

    def step():
        with trace.range("lsknn:step"):
            _step()
            _sync(device)

    def _step(phases: bool = args.phases, pts_in=None, out_h=None):
        nonlocal info_last
        out_h = host_out if out_h is None else out_h
        info = PL.RunInfo(PL.PhaseTimer(phases, device))
        if pts_in is not None:
            pts = pts_in  # pipelined: this step's points already on the device
        elif args.variant == "unordered" and args.mode == "halo":
            # the pipeline moves the host points itself: on several ranks in chunks
            # overlapped with the all-to-all (pipelines.redistribute_stream), on one in a
            # single copy (a chunked upload keyed as it lands measured no gain: one set
            # 1193.8 ms with 64M-point chunks against 1191-1194 ms; profiles/r5_stream/)
            pts = host_pts
        else:
            pts = host_pts.to(device, non_blocking=True)
        if args.mode == "ring":
            out = RA.ring_knn(pts, comm, cfg, info)
        elif args.mode == "peer":
            out = RA.peer_knn(pts, comm, cfg, info)
        elif args.variant == "unordered":
            # one rank: host_out through pipelines.query_into (device buffer + copy for the
            # grid kernel); several ranks: the grouped result return copies each group's
            # rows into it under the exchange
            out = PL.unordered_knn(pts, comm, cfg, info, n_total=n_total,
                                   out=out_h if device.type == "cuda" else None, direct=direct)
        else:
            out = PL.prepartitioned_knn(pts, comm, cfg, info, out=out_h if single_gpu else None,
                                        direct=direct)
        if out.data_ptr() != out_h.data_ptr():
            out_h.copy_(out, non_blocking=True)
        info_last = info

    use_graph = (args.graph == 1 or (args.graph < 0 and not (args.phases or args.stats))) \
        and not comm.distributed and device.type == "cuda" and args.mode == "halo" and not pipelined
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
        # over-full key cells seen by the eager warmup: capture the (fixed-size) refinement
        E.REFINE_CAPTURE = E.LAST_REFINED
        E.prepare_capture(device)  # failure-word peaks over every replay
        graph = torch.cuda.CUDAGraph()
        E.reset_kernels_used()
        with torch.cuda.graph(graph):
            _step()
        _sync(device)
        # the replays run exactly the captured launches: report the capture's kernels
        # (the reset before the timed steps would otherwise leave the list empty)
        graph_kernels = E.kernels_used()

        def step():  # noqa: F811 — graph replay replaces the eager step
            with trace.range("lsknn:step"):
                graph.replay()
                _sync(device)
    elif pipelined:
        # stream of sets (parallel/stream.py): set i+1's upload under set i's build and
        # k-NN; several ranks: set i's results to host under set i+1
        # the stream keeps results in device memory and copies them to host on a side
        # stream: the kernel's direct PCIe writes contend with the next set's upload (1B,
        # k=100: 1319 vs 1373 ms per set); prePartitioned sets take the same stream (one
        # rank: the same single-rank pipeline; several: no redistribution)
        runner = SetStream(comm, cfg, direct_out=bool(args.direct_out) if args.direct_out >= 0 else False,
                           variant=args.variant)

        def run_steps(n):
            with trace.range("lsknn:steps"):
                runner.run([host_sets[i % 2] for i in range(n)], [host_outs[i % 2] for i in range(n)],
                           n_totals=[n_total] * n)

        run_steps(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
    comm.barrier()
    _sync(device)
    E.reset_kernels_used()  # report the kernels of the timed steps only
    E.deferred_heavy_cells(clear=True)
    ncoll0 = comm.collectives()
    calls0 = dict(getattr(comm, "calls", {}))
    t0 = time.perf_counter()
    if pipelined:
        run_steps(args.steps)
    else:
        for _ in range(args.steps):
            step()
    comm.barrier()
    _sync(device)
    elapsed = time.perf_counter() - t0
    # collective launches of the timed steps (the closing barrier excluded)
    coll_per_step = (comm.collectives() - ncoll0 - (1 if comm.distributed else 0)) / max(1, args.steps)
    calls = {op: round((c - calls0.get(op, 0)) / max(1, args.steps), 2)
             for op, c in getattr(comm, "calls", {}).items() if op != "*" and c != calls0.get(op, 0)}
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    comm.allreduce_(t, "max")
    elapsed = float(t.item())
    kernels_timed = E.kernels_used()  # (gate reads: after the clock)
    if graph is not None:
        kernels_timed = sorted(set(kernels_timed) | set(graph_kernels))

    ms = elapsed / args.steps * 1e3
    value = n_total * args.steps / elapsed / 1e6
    heavy_unrefined = E.deferred_heavy_cells(clear=True)
    if graph is not None:
        E.verify_captured_failures(clear=True)  # raises if any replay overflowed a failure list
        heavy_unrefined = E.captured_heavy_cells(clear=True) or heavy_unrefined
    # the sets the timed steps wrote last (pipelined: both sets when K >= 2)
    written = sorted({(args.steps - 1 - j) % len(host_sets) for j in range(min(args.steps, len(host_sets)))})
    finite_t = torch.tensor([sum(0 if host_outs[d].numel() == 0 or bool(torch.isfinite(host_outs[d]).all()) else 1
                                 for d in written)], dtype=torch.int64, device=device)
    comm.allreduce_(finite_t, "sum")
    finite = int(finite_t.item()) == 0

    # ---- untimed: sampled brute-force check of the timed result, then one instrumented step
    check = None
    if args.verify > 0:
        # (prePartitioned: rank r's file is the block [b, e) of global ids too — the check
        # counts every sampled id's distances over all ranks' points)
        b, _ = block_range(n_total, rank, world)
        for d in written:
            FA.HEARTBEAT.beat("sampled_exact")
            c = verify.sampled_exact(comm, host_sets[d], host_outs[d], b, n_total, args.k, args.verify)
            check = c if check is None else {"samples": check["samples"] + c["samples"],
                                             "exact": check["exact"] + c["exact"],
                                             "mismatch_ids": check["mismatch_ids"] + c["mismatch_ids"]}
    # single-set latency: one set from pinned host memory to distances in host memory
    # (the default non-streamed path of this variant), best of two, max over ranks
    single_s = None
    if args.mode == "halo" and device.type == "cuda":
        best = math.inf
        for _ in range(2):
            comm.barrier()
            _sync(device)
            t1 = time.perf_counter()
            _step(phases=False)
            _sync(device)
            best = min(best, time.perf_counter() - t1)
        tt = torch.tensor([best], dtype=torch.float64, device=device)
        comm.allreduce_(tt, "max")
        single_s = float(tt.item())
    # the instrumented step takes the timed path: pipelined steps start from points already
    # on the device (their upload ran under the previous step), so this one does too
    pts_dev = host_pts.to(device) if pipelined else None
    _sync(device)
    detail = instrumented_detail(comm, lambda: (_step(phases=True, pts_in=pts_dev), _sync(device)),
                                 lambda: info_last)
    del pts_dev
    if rank == 0:
        if args.phases or args.stats:
            print(json.dumps({"phases_s": info_last.timer.times, "counts": info_last.plain_counts(),
                              "knn_stats": info_last.stats.counters}), file=sys.stderr)
        rec = {
            "metric": metric_name(n_total, args.k),
            "value": round(value, 3),
            "unit": "Mpoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "single_set_ms": round(single_s * 1e3, 3) if single_s else None,
            "single_set_mpts": round(n_total / single_s / 1e6, 3) if single_s else None,
            "dtype": "fp32",
            "data": "synthetic uniform-random float3 in [0,1)^3 (pinned host memory), no file I/O"
                    + ("; two different point sets alternate step by step" if pipelined else ""),
            "config": {
                "model": f"{args.variant}Data k-th-NN distance, k={args.k}",
                "global_batch": n_total,
                "seq_len": None,
                "parallelism": (f"ref-algo {args.mode} x{world}" if args.mode != "halo" else
                                f"spatial-redistribute+halo x{world}" if args.variant == "unordered"
                                else f"halo x{world}"),
                "k": args.k,
                "comm": comm_info(comm)["backend"],
                "comm_info": comm_info(comm),
                "ranks": world,
                "collectives_per_step": round(coll_per_step, 2),
                "hip_graph": graph is not None,
                "hw_queues": HW_QUEUES,
                "pipelined": pipelined,
                "heavy_cells_unrefined": heavy_unrefined,
                "knn_kernels": kernels_timed,
                "all_finite": finite,
                "sampled_exact": (f"{check['exact']}/{check['samples']}" if check else None),
            },
            "detail": dict(detail, sampled_exact=check, comm_calls_per_step=calls),
        }
        print(json.dumps(rec), flush=True)
    LA.finalize(launch)


def instrumented_detail(comm, run_step, last_info) -> dict:
    """One extra untimed step with device-synchronised phase marks; returns the max over
    ranks of every phase time, per-rank k-NN and step ms, and the summed exchange sizes."""
    t0 = time.perf_counter()
    run_step()
    step_s = time.perf_counter() - t0
    info = last_info()
    vec = [info.timer.times.get(p, 0.0) for p in PHASES] + [step_s] + \
        [float(info.plain_counts().get(c, 0)) for c in COUNTS]
    allv = comm.allgather(torch.tensor(vec, dtype=torch.float64, device=comm.device)).cpu()
    np_ = len(PHASES)
    phases_max = {p: round(float(allv[:, i].max()) * 1e3, 3) for i, p in enumerate(PHASES)
                  if float(allv[:, i].max()) > 0}
    counts_sum = {c: int(allv[:, np_ + 1 + i].sum()) for i, c in enumerate(COUNTS)}
    return {
        "phase_ms_max_over_ranks": phases_max,
        "instrumented_step_ms_per_rank": [round(float(x) * 1e3, 3) for x in allv[:, np_]],
        "knn_local_ms_per_rank": [round(float(max(a, b)) * 1e3, 3) for a, b in
                                  zip(allv[:, PHASES.index("knn_local")],
                                      allv[:, PHASES.index("knn_local+halo_exchange")])],
        "halo_requery_ms_per_rank": [round(float(x) * 1e3, 3) for x in allv[:, PHASES.index("halo_requery")]],
        "redistributed_bytes": counts_sum["sent_points"] * 12,
        "halo_bytes": counts_sum["halo_sent"] * 12,
        "requery_groups": counts_sum["requery_groups"],
        "owned_points_per_rank": [int(x) for x in allv[:, np_ + 1 + COUNTS.index("owned_points")]],
    }


if __name__ == "__main__":
    main()
