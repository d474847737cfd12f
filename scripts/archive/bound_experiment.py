"""How much of the k-NN kernel time is spent because the first pass does not know the
answer? Re-run the kernel seeded with (scaled) exact k-th values as upper bounds."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=float, default=1e8)
ap.add_argument("--k", type=int, default=100)
a = ap.parse_args()
n = int(a.points)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
idx = E.build_index(p)
cfg = E.KnnConfig(k=a.k)
hint2 = E.radius_hint2(idx.box, n, a.k)


def run(init, tag):
    torch.cuda.synchronize()
    t = time.perf_counter()
    st = E.KnnStats()
    d2 = E.query(idx, cfg, hint2, stats=st, init_d2=init)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    c = st.counters
    rows = c["waves"] * 4
    print(f"{tag:>14}: {dt:.3f} s  quarters/row pass1 {c['leaves'] / rows:.1f}  collect {c['collect_steps'] / rows:.1f}"
          f"  nodes/wave {c['nodes'] / c['waves']:.1f}  passes/wave {c['hist_passes'] / c['waves']:.2f}", flush=True)
    return d2


ref = run(None, "no bound")
ref = run(None, "no bound")
for s in (1.0, 1.1, 1.25, 1.5, 2.0, 3.0):
    d = run(ref * s, f"exact*{s}")
    assert torch.equal(d, ref)
