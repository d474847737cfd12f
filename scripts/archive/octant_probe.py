"""Why is the local k-NN pass of one rank of an 8-rank run slower per point than the
single-rank run? Times the k-NN kernel on 125M uniform points for: the whole cube,
an octant with keys on the global cube (what the pipeline does), an octant on its own
bounds, and a whole cube plus a thin outside shell ignored."""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
k = 100
g = torch.Generator(device="cuda").manual_seed(3)
cfg = E.KnnConfig(k=k)


def timed(label, pts, box, n_total):
    idx = E.build_index(pts, box)
    hint2 = E.radius_hint2(box if box is not None else idx.box, n_total, k)
    st = E.KnnStats()
    for r in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        E.query(idx, cfg, hint2, stats=st if r == 0 else None)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
    c = st.counters
    print(f"{label:34s} {dt:.4f} s  steps/wave {c['recorded_leaves'] / c['waves']:.1f} "
          f"csteps/wave {c['collect_steps'] / c['waves']:.1f} nodes/wave {c['nodes'] / c['waves']:.1f} "
          f"passes/wave {c['hist_passes'] / c['waves']:.3f} ovf {c['overflow_lanes']} udf {c['underflow_lanes']}",
          flush=True)
    del idx


p = torch.rand((n, 3), generator=g, device="cuda")
timed("cube, own bounds", p, None, n)
gbox = K.bounds(torch.tensor([[0.0, 0.0, 0.0], [1.0, 1.0, 1.0]], device="cuda"))
timed("cube, global box", p, gbox, n)
p.mul_(0.5)
timed("octant, global-cube keys", p, gbox, 8 * n)
timed("octant, own bounds", p, None, 8 * n)
