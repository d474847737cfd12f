"""mixed_scale k-th-NN probe: kernel counters and wall time per k (kernel trace via
rocprofv3 around it). python scripts/mixed_probe.py [n] [k ...]"""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
ks = [int(a) for a in sys.argv[2:]] or [100, 16]
p = datasets.GENERATORS["mixed_scale"](n).cuda()
for k in ks:
    for rep in range(2):
        st = E.KnnStats()
        torch.cuda.synchronize()
        t = time.perf_counter()
        E.knn_distances(p, k, stats=st)
        torch.cuda.synchronize()
        c = {kk: v for kk, v in st.counters.items() if v}
        print(f"k={k} rep {rep}: {time.perf_counter() - t:.4f} s", c, flush=True)
