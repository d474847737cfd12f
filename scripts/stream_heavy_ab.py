"""Stream of non-uniform sets: over-full key cells refined (learned from the previous set)
vs always deferred. python scripts/stream_heavy_ab.py [n] [sets] [dist]

Times SetStream over `sets` alternating sets of `dist` (tests/datasets.py) and reports ms
per set (steady state), whether a build refined, and the exactness of sampled outputs."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import datasets  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.stream import SetStream  # noqa: E402
from mpi_cuda_largescaleknn_amd.utils import verify as V  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 20_000_000
nsets = int(sys.argv[2]) if len(sys.argv) > 2 else 6
dist = sys.argv[3] if len(sys.argv) > 3 else "mixed_scale"
dev = torch.device("cuda", 0)
hosts = [datasets.GENERATORS[dist](n, seed=s).pin_memory() for s in (11, 12)]
print(f"{dist}: 2 sets of {n} points ready", flush=True)
outs = [torch.empty(n, dtype=torch.float32).pin_memory() for _ in range(2)]
orig = E.refine_heavy_cells
MODES = os.environ.get("LSK_MODES", "learned,deferred").split(",")


def deferred_only(*a, **kw):  # the round-4 behaviour: every stream build defers
    E._HEAVY_PENDING.clear()
    E._HEAVY_KNOWN[0] = False
    return orig(*a, **kw)


for mode in MODES:
    E.refine_heavy_cells = orig if mode == "learned" else deferred_only
    E.deferred_heavy_cells(clear=True)
    E.LAST_REFINED = False
    runner = SetStream(SingleComm(dev), E.KnnConfig(k=100))
    stamps = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.run([hosts[i % 2] for i in range(nsets)], [outs[i % 2] for i in range(nsets)],
               on_done=lambda i: (stamps.append(time.perf_counter()),
                                  print(f"  {mode} set {i} done at {(stamps[-1] - t0) * 1e3:.0f} ms", flush=True)))
    torch.cuda.synchronize()
    per = (stamps[-1] - stamps[1]) / max(len(stamps) - 2, 1) * 1e3
    chk = V.sampled_exact(SingleComm(dev), hosts[(nsets - 1) % 2], outs[(nsets - 1) % 2], 0, n, 100, 256)
    print(f"{dist} {mode}: {per:.1f} ms per set (steady), total {(time.perf_counter() - t0) * 1e3:.0f} ms, "
          f"refined {E.LAST_REFINED}, unrefined reported {E.deferred_heavy_cells(clear=True)}, "
          f"exact {chk['exact']}/{chk['samples']}", flush=True)
E.refine_heavy_cells = orig
