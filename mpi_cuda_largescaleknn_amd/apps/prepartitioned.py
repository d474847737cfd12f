"""hipKNN_prePartitionedData — one (spatially coherent) input file per rank.

    hipKNN_prePartitionedData <fileList.txt> -o <prefix> -k <k> [-r <maxRadius>] [-g <gpusPerNode>]
                              [--mode auto|halo|peer] [--device auto|cuda|cpu] [--stats s.json] [-v]
                              [--balance auto|on|off] [--bootstrap auto|env|mpi|spawn --nproc N]
                              [--device-map 0,1,..]

Same grammar and files as cudaMpiKNN_prePartitionedData
(prePartitionedDataVariant.cu:176-389): line r of the list is rank r's float3 file,
the rank count must equal the number of files, and rank r writes
``<prefix>_%06d.float`` with its distances in its file's order. `--mode peer` runs the
reference's bounds-culled whole-shard pull schedule (ref-algo baseline); the default is
the MI355X halo exchange.
"""
from __future__ import annotations

import sys

import torch

from ..parallel import launch as L
from ..parallel import pipelines as PL
from ..parallel import refalgo as RA
from ..ops import kernels as K
from ..utils import cli, io
from . import common


def output_name(prefix: str, rank: int) -> str:
    return f"{prefix}_{rank:06d}.float"


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv if argv is None else argv)
    args = cli.parse_or_exit(cli.PREPARTITIONED, argv)
    if args.mode == "ring":
        common.fail("Error: --mode ring applies to hipKNN_unorderedData")
    names = io.read_file_list(args.input)
    if args.bootstrap == "spawn":
        return L.spawn_local(args.nproc, "mpi_cuda_largescaleknn_amd.apps.prepartitioned", common.without_spawn(argv[1:]))
    launch = L.init(args.device, args.gpu_affinity, args.verbose, bootstrap=args.bootstrap,
                    device_map=args.device_map)
    return common.guarded(launch, lambda: _run(args, launch, names))


def _run(args, launch, names) -> int:
    if launch.size != len(names):
        raise RuntimeError("number of input files does not match MPI size")
    pts = io.read_points(names[launch.rank], pin_memory=launch.device.type == "cuda")
    box = K.bounds(pts)[0:6].tolist() if pts.shape[0] else [float("inf")] * 3 + [float("-inf")] * 3
    print(f"#{launch.rank}/{launch.size}: got {pts.shape[0]} points to work on, bounds is "
          f"({box[0]:g},{box[1]:g},{box[2]:g})-({box[3]:g},{box[4]:g},{box[5]:g})", flush=True)
    cfg = common.config(args)
    info = common.make_info(launch, bool(args.stats) or args.verbose)
    t0 = common.now(launch)
    dpts = pts.to(launch.device, non_blocking=True)
    if args.mode == "peer":
        out = RA.peer_knn(dpts, launch.comm, cfg, info,
                          log=(lambda m: print(m, flush=True)))
    else:
        # one GPU rank, large k: the k-NN kernel writes the distances straight into
        # pinned host memory (PL.direct_host_out_pays)
        host_out = (torch.empty(pts.shape[0], dtype=torch.float32, pin_memory=True)
                    if launch.device.type == "cuda" and not launch.comm.distributed
                    and PL.direct_host_out_pays(cfg.k) else None)
        out = PL.prepartitioned_knn(dpts, launch.comm, cfg, info, out=host_out, balance=args.balance)
    res = out.cpu()
    if launch.device.type == "cuda":
        torch.cuda.synchronize(launch.device)
    t1 = common.now(launch)
    print("done all queries...", flush=True)
    io.write_floats(output_name(args.output, launch.rank), res, 0, truncate=True)
    common.write_stats(launch, args, info, {"points": int(pts.shape[0])}, t1 - t0)
    L.finalize(launch)
    return 0


if __name__ == "__main__":
    sys.exit(main())
