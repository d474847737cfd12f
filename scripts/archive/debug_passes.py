"""Per-lane pass-count histogram of the rows kernel (qstatus >> 16) (debug helper)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1]))
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
idx = E.build_index(p)
cfg = E.KnnConfig(k=100)
qs = torch.zeros(n, dtype=torch.int32, device="cuda")
st = E.KnnStats()
torch.cuda.synchronize()
t = time.perf_counter()
E.query(idx, cfg, E.radius_hint2(idx.box, n, 100), stats=st, qstatus=qs)
torch.cuda.synchronize()
print(f"time {time.perf_counter() - t:.3f}s", flush=True)
passes = (qs >> 16).cpu()
print("passes histogram:", torch.bincount(passes).tolist()[:20])
bits = qs.cpu() & 0xffff
for b, name in [(1, "ovf"), (2, "udf"), (4, "ref"), (16, "coll"), (32, "band1"), (64, "cut"), (256, "limit")]:
    print(name, int(((bits & b) != 0).sum()))

hi = (qs >> 16).cpu().to(torch.int64)
order = torch.argsort(hi, descending=True)
print("slowest lanes (cycles>>16 or passes):", hi[order[:10]].tolist(), "median", int(hi.median()))
sel = order[:5]
print("their flags:", bits[sel].tolist(), "groups:", (sel // 64).tolist())
d2 = None
