"""Inspect published halo boxes of each loopback rank (debug helper)."""
import sys

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import run_loopback  # noqa: E402

n = int(float(sys.argv[1]))
P = int(sys.argv[2])
DEV = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
cfg = E.KnnConfig(k=100)


def fn(comm):
    b, e = n * comm.rank // comm.size, n * (comm.rank + 1) // comm.size
    info = PL.RunInfo(PL.PhaseTimer(False, DEV))
    box = PL.global_box(p[b:e], comm)
    owned, *_ = PL.redistribute(p[b:e], comm, box, info)
    idx = E.build_index(owned, box)
    hint2 = E.radius_hint2(box, n, 100)
    d2 = E.query(idx, cfg, hint2)
    K.tree_set_radii(idx.nodes, idx.n, d2)
    L = min(cfg.publish_levels, idx.depth)
    leaves = idx.nodes[(1 << L):(2 << L)]
    ext = (leaves[:, 4:7] - leaves[:, 0:3]).amax(1)
    ok = torch.isfinite(ext)
    ext = ext[ok]
    r = leaves[ok, 3].sqrt()
    lo, hi = owned.min(0).values.tolist(), owned.max(0).values.tolist()
    q = torch.quantile(ext.float(), torch.tensor([0.5, 0.99, 0.999, 1.0], device=DEV)).tolist()
    return (comm.rank, [round(x, 3) for x in lo], [round(x, 3) for x in hi], [round(x, 4) for x in q],
            int((ext > 0.1).sum()), round(float(r.median()), 4), round(float(r.max()), 4))


for rec in run_loopback(P, fn, DEV):
    print(rec, flush=True)
