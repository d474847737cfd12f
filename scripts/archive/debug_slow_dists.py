"""Kernel counters + phase split for the slow non-uniform cases (duplicates, mixed_scale)."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
for name in sys.argv[2:] or ["duplicates", "mixed_scale"]:
    p = datasets.GENERATORS[name](n).to("cuda")
    for k in (100, 16):
        torch.cuda.synchronize()
        t = time.perf_counter()
        idx = E.build_index(p)
        torch.cuda.synchronize()
        tb = time.perf_counter() - t
        st = E.KnnStats()
        hint = E.radius_hint(idx.box, n, k)
        t = time.perf_counter()
        E.query(idx, E.KnnConfig(k=k), hint, stats=st)
        torch.cuda.synchronize()
        tq = time.perf_counter() - t
        c = {a: b for a, b in st.counters.items() if b and not a.startswith("prof")}
        print(f"{name} n={n} k={k}: build {tb:.3f}s query {tq:.3f}s", c, flush=True)
