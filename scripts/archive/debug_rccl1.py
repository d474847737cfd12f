"""Diagnose the forced 1-rank RCCL path: raw all_to_all_single at growing sizes, then
the unordered pipeline at growing n with a sampled exactness check."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import TorchComm  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import verify as V  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29555")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
comm = TorchComm(dev, force=True)
for n in (10**3, 10**5, 10**6, 10**7, 10**8):
    x = torch.rand((n, 3), device=dev)
    r, _ = comm.alltoallv(x, [n])
    torch.cuda.synchronize()
    print("alltoallv", n, "equal", bool(torch.equal(r, x)), flush=True)
for n in (10**5, 10**6, 10**7, 3 * 10**7):
    p = torch.rand((n, 3), device=dev)
    cfg = E.KnnConfig(k=100)
    info = PL.RunInfo(PL.PhaseTimer(True, dev))
    t = time.perf_counter()
    out = PL.unordered_knn(p, comm, cfg, info)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    chk = V.sampled_exact(comm, p, out, 0, n, 100, 64)
    print("unordered", n, f"{dt:.3f}s", {k: round(v * 1e3, 1) for k, v in info.timer.times.items()},
          info.counts, chk["exact"], "/", chk["samples"], flush=True)
dist.destroy_process_group()
