"""Debug helper: compare GPU k-NN against the CPU oracle and dump status bits of mismatches."""
import math
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from datasets import GENERATORS  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

for dist in ["uniform", "clustered", "duplicates", "planar", "mixed_scale"]:
    for k in [1, 8, 16, 100]:
        p = GENERATORS[dist](30000, seed=k)
        idx = E.build_index(p.cuda())
        cfg = E.KnnConfig(k=k)
        st = torch.zeros(idx.n, dtype=torch.int32, device="cuda")
        stats = E.KnnStats()
        hint2 = E.radius_hint2(idx.box, idx.n, k)
        d2 = E.query(idx, cfg, hint2, stats=stats, qstatus=st).cpu()
        ps = idx.pts[: idx.n].cpu()
        ref = K.kth_cpu(ps, ps, k, math.inf)
        bad = (d2 != ref).nonzero().flatten()
        print(dist, k, "mismatches", bad.numel(), stats.counters, flush=True)
        for i in bad[:8].tolist():
            s = int(st[i])
            print("   q", i, "got", d2[i].item(), "ref", ref[i].item(), "status", hex(s & 0xffff), "passes", s >> 16)

# input-order pipeline check: isolate scatter vs sqrt
p = GENERATORS["uniform"](30000, seed=8)
k = 8
ref_d2 = K.kth_cpu(p, p, k, math.inf)
idx = E.build_index(p.cuda())
d2 = E.query(idx, E.KnnConfig(k=k), E.radius_hint2(idx.box, idx.n, k))
out = torch.empty(idx.n, device="cuda")
K.scatter1(d2, idx.perm, out, finalize=False)
o = out.cpu()
print("scatter no-finalize mismatches", int((o != ref_d2).sum()))
fin_gpu = K.finalize_distances(ref_d2.cuda()).cpu()
fin_cpu = K.finalize_distances(ref_d2)
bad = (fin_gpu != fin_cpu).nonzero().flatten()
print("sqrt mismatches", bad.numel())
for i in bad[:5].tolist():
    print("  d2", ref_d2[i].item(), ref_d2[i].view(torch.int32).item(), "gpu", fin_gpu[i].item(), "cpu", fin_cpu[i].item())
import numpy as np
print("numpy sqrt agrees with torch cpu:", bool(np.array_equal(np.sqrt(ref_d2.numpy()), fin_cpu.numpy())))
