"""hipKNN_unorderedData — k-th-NN distance of every point of one float3 file.

    hipKNN_unorderedData <in.float3> -o <out.float> -k <k> [-r <maxRadius>] [-g <gpusPerNode>]
                         [--mode auto|halo|ring] [--device auto|cuda|cpu] [--stats s.json] [-v]
                         [--bootstrap auto|env|mpi|spawn --nproc N] [--device-map 0,1,..]

Same grammar, input and output bytes as cudaMpiKNN_unorderedData
(unorderedDataVariant.cu:105-239): rank r of P reads the block
[floor(N*r/P), floor(N*(r+1)/P)) of the file, the output file holds N float32
distances in input order. `--mode ring` runs the reference's ring-rotation schedule
(ref-algo baseline); the default is the MI355X pipeline (spatial redistribution +
halo exchange). Output is written with parallel pwrite at offset begin*4 — the same
bytes as the reference's serialized rank-ordered append (U:229-237).
"""
from __future__ import annotations

import sys

import torch

from ..parallel import launch as L
from ..parallel import pipelines as PL
from ..parallel import refalgo as RA
from ..utils import cli, io
from . import common


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv if argv is None else argv)
    args = cli.parse_or_exit(cli.UNORDERED, argv)
    if args.mode == "peer":
        common.fail("Error: --mode peer applies to hipKNN_prePartitionedData")
    if args.bootstrap == "spawn":
        return L.spawn_local(args.nproc, "mpi_cuda_largescaleknn_amd.apps.unordered", common.without_spawn(argv[1:]))
    launch = L.init(args.device, args.gpu_affinity, args.verbose, bootstrap=args.bootstrap,
                    device_map=args.device_map)
    return common.guarded(launch, lambda: _run(args, launch))


def _run(args, launch) -> int:
    pts, begin, total = io.read_portion(args.input, launch.rank, launch.size,
                                        pin_memory=launch.device.type == "cuda")
    print(f"#{launch.rank}/{launch.size}: got {pts.shape[0]} points to work on", flush=True)
    cfg = common.config(args)
    info = common.make_info(launch, bool(args.stats) or args.verbose)
    t0 = common.now(launch)
    # several GPU ranks (halo mode): the host points stream to the device inside the
    # redistribution; otherwise one copy up front
    streamed = args.mode != "ring" and launch.comm.distributed and launch.device.type == "cuda"
    dpts = pts if streamed else pts.to(launch.device, non_blocking=True)
    if args.mode == "ring":
        out = RA.ring_knn(dpts, launch.comm, cfg, info)
    else:
        # one GPU rank, large k: the k-NN kernel writes the distances straight into
        # pinned host memory (PL.direct_host_out_pays)
        host_out = (torch.empty(pts.shape[0], dtype=torch.float32, pin_memory=True)
                    if launch.device.type == "cuda" and not launch.comm.distributed
                    and PL.direct_host_out_pays(cfg.k) else None)
        out = PL.unordered_knn(dpts, launch.comm, cfg, info, n_total=total, out=host_out)
    res = out.cpu()
    if launch.device.type == "cuda":
        torch.cuda.synchronize(launch.device)
    t1 = common.now(launch)
    print("done all queries...", flush=True)
    # rank 0 creates/truncates and sizes the file, then every rank writes its block
    if launch.rank == 0:
        io.write_floats(args.output, res[:0], 0, truncate=True, total_records=total)
    launch.comm.barrier()
    io.write_floats(args.output, res, begin, truncate=False)
    launch.comm.barrier()
    common.write_stats(launch, args, info, {"points": int(pts.shape[0]), "begin": begin}, t1 - t0)
    if args.verbose and launch.rank == 0:
        print(f"knn time {t1 - t0:.3f}s  {total / max(t1 - t0, 1e-9) / 1e6:.1f} Mpts/s", flush=True)
    L.finalize(launch)
    return 0


if __name__ == "__main__":
    sys.exit(main())
