"""P loopback ranks on one GPU running the unordered pipeline (phase times and halo
counts per rank; ranks share the device, so times include the other ranks' work)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import run_loopback  # noqa: E402

n = int(float(sys.argv[1]))
P = int(sys.argv[2])
DEV = torch.device("cuda", 0)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
# kernel counters only on request: the stats build of the pass costs ~17 % (208 vs
# 177 ms per 125M-point rank, profiles/archive/r1_v20)
cfg = E.KnnConfig(k=100, collect_stats="--stats" in sys.argv)


def fn(comm):
    b, e = n * comm.rank // comm.size, n * (comm.rank + 1) // comm.size
    # --nomarks: no device-wide syncs at phase marks (they serialise the ranks' streams;
    # used for the kernel-trace timeline of the overlapped halo exchange)
    info = PL.RunInfo(PL.PhaseTimer("--nomarks" not in sys.argv, DEV))
    out = PL.unordered_knn(p[b:e], comm, cfg, info, n_total=n)
    return out, info


for rep in range(2):
    t = time.perf_counter()
    res = run_loopback(P, fn, DEV)
    torch.cuda.synchronize()
    print(f"loopback x{P} {n}: {time.perf_counter() - t:.3f}s", flush=True)
for r, (_, info) in enumerate(res):
    print(r, {k: round(v, 4) for k, v in info.timer.times.items()}, info.counts, flush=True)
    if cfg.collect_stats:
        print("   stats", {k: v for k, v in info.stats.counters.items() if v}, flush=True)
single = E.knn_distances(p, 100)
print("equal to single:", torch.equal(torch.cat([o for o, _ in res]), single))
