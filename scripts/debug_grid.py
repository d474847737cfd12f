"""Debug the grid k-NN pass on small synthetic sets: per-lane status vs the CPU oracle."""
import math
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from datasets import GENERATORS, uniform  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402


def run(name, p, k, ms=None):
    E.GRID = "on"
    if ms is not None:
        E.GRID_MS = ms
    idx = E.build_index(p.cuda(), grid=True)
    n = idx.n
    cfg = E.KnnConfig(k=k)
    qs = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = E.KnnStats()
    d2 = E.query(idx, cfg, E.radius_hint(idx.box, n, k), stats=st, qstatus=qs)
    ref = K.kth_cpu(idx.pts[:n].cpu(), idx.pts[:n].cpu(), k, math.inf)
    got = d2.cpu()
    qs = qs.cpu()
    bad = got != ref
    fail = (qs & 4096) != 0
    print(f"{name}: n={n} k={k} level={idx.grid.level} bad={int(bad.sum())} failed={int(fail.sum())} "
          f"bad&~failed={int((bad & ~fail).sum())} passes/wave={st.counters['hist_passes'] / st.counters['waves']:.2f}"
          f" ovf={st.counters['overflow_lanes']} limit_waves={st.counters['pass_limit_waves']}", flush=True)
    if int(bad.sum()):
        i = int(bad.nonzero()[0])
        w = i // 64
        print("  first bad", i, "got", float(got[i]), "ref", float(ref[i]), "qs", hex(int(qs[i])),
              "pt", idx.pts[i].tolist(), "wave lanes qs:", [hex(int(x)) for x in qs[w * 64:w * 64 + 8]])
        wb = idx.pts[w * 64:w * 64 + 64].cpu()
        print("  wave box", wb.min(0).values.tolist(), wb.max(0).values.tolist(), "box", idx.box.cpu().tolist())
    E.GRID_MS = 6.0


k = int(sys.argv[1]) if len(sys.argv) > 1 else 8
run("mixed_scale", GENERATORS["mixed_scale"](30000, seed=k + 7), k)
run("uniform*1000", uniform(15000, seed=3) * 1000.0, k)
run("uniform coarse", uniform(30000, seed=3), k, ms=200)
run("uniform", uniform(30000, seed=3), k)
