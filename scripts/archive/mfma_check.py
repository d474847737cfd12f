"""knn_mfma.hip against knn_grid.hip on one index: bitwise outputs, kernel time, counters.

python scripts/mfma_check.py --points 1e6 1e7 --k 8 16 100 [--oracle 2048] [--reps 3]
Every size: uniform points in [0,1)^3; the grid forced on (GRID=on); the same index and
hint for both kernels; outputs compared bit for bit (sorted order), optionally a sample
against the C++ CPU oracle."""
import argparse
import math
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=float, nargs="+", default=[1e6])
ap.add_argument("--k", type=int, nargs="+", default=[100])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--oracle", type=int, default=0, help="check this many sampled queries against the CPU oracle")
ap.add_argument("--dist", default="uniform")
ap.add_argument("--only", default="", help="mfma or sgpr: time one kernel only")
a = ap.parse_args()
E.GRID = "on"


def run(idx, k, kern, reps):
    K.GRID_KERNEL = kern
    cfg = E.KnnConfig(k=k)
    hint2 = E.radius_hint2(idx.box, idx.n, k)
    times = []
    out = None
    st = None
    for r in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s = E.KnnStats() if r == 0 else None
        d2 = E.query(idx, cfg, hint2, stats=s)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        if r == 0:
            out, st = d2.clone(), s
    return out, sorted(times)[len(times) // 2], st


for npts in a.points:
    n = int(npts)
    g = torch.Generator(device="cuda").manual_seed(n % 1000003)
    if a.dist == "uniform":
        p = torch.rand((n, 3), generator=g, device="cuda")
    else:
        sys.path.insert(0, "tests")
        from datasets import GENERATORS  # noqa: E402
        p = GENERATORS[a.dist](n, seed=5).to("cuda")
    idx = E.build_index(p, grid=True)
    for k in a.k:
        res = {}
        for kern in (["mfma", "sgpr"] if not a.only else [a.only]):
            out, t, st = run(idx, k, kern, a.reps)
            res[kern] = out
            c = st.counters
            print(f"n={n} k={k} {kern}: {t * 1e3:.2f} ms  evals/q={c.get('evals', 0) / max(n, 1):.0f} "
                  f"passes={c.get('hist_passes', 0) / max(c.get('waves', 1), 1):.3f} ovf={c.get('overflow_lanes', 0)} "
                  f"low={c.get('underflow_lanes', 0)} high={c.get('refine_lanes', 0)} "
                  f"fail={c.get('failed_lanes', 0)} fallback={c.get('fallback_queries', 0)}", flush=True)
            if c.get("prof_proc_collect"):  # LSK_MF_PROFILE build: cycles per wave by phase
                w = max(c.get("waves", 1), 1)
                ph = {"setup": c["prof_proc_hist"], "stream": c["prof_proc_collect"], "exact": c["prof_walk_hist"],
                      "select": c["prof_walk_collect"]}
                print("  cycles/wave:", {k: round(v / w) for k, v in ph.items()},
                      f"tiles/wave={c['prof_inner_nodes'] / w:.1f} append rounds/tile="
                      f"{c['prof_quarters'] / max(c['prof_inner_nodes'], 1):.2f}", flush=True)
        if len(res) == 2:
            m, s = res["mfma"], res["sgpr"]
            bad = (m.view(torch.int32) != s.view(torch.int32))
            nb = int(bad.sum())
            print(f"  mfma vs sgpr: {nb} differing outputs of {n}", flush=True)
            if nb:
                i = torch.nonzero(bad)[:5].view(-1).tolist()
                print("   e.g.", [(j, float(m[j]), float(s[j])) for j in i], flush=True)
        if a.oracle:
            pts = idx.pts[:n].cpu()
            sel = torch.randperm(n)[: a.oracle]
            ref = K.kth_cpu(pts, pts[sel], k, math.inf)
            got = res[list(res)[0]][sel].cpu()
            nb = int((got.view(torch.int32) != ref.view(torch.int32)).sum())
            print(f"  oracle sample: {nb} of {len(sel)} differ", flush=True)
