"""A/B of the local k-NN pass: cell-grid candidates (knn_grid.hip) vs the bucket-tree walk
(knn_rows.hip) on the same index; outputs compared bit for bit."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=float, default=1e8)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--dist", default="uniform")
ap.add_argument("--levels", default="", help="comma list of sub-cell levels to try (default: auto)")
a = ap.parse_args()
n = int(a.points)
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
if a.dist == "clustered":
    c = torch.rand((20, 3), generator=g, device="cuda")
    w = torch.randint(0, 20, (n,), generator=g, device="cuda")
    p = (c[w] + 0.01 * torch.randn((n, 3), generator=g, device="cuda")).contiguous()
torch.cuda.synchronize()
t = time.perf_counter()
E.GRID = "on"
idx = E.build_index(p, grid=True)
torch.cuda.synchronize()
print(f"build (tree + grid, finest level {idx.grid.level + 2}): {time.perf_counter() - t:.3f} s", flush=True)
cfg = E.KnnConfig(k=a.k)
hint2 = E.radius_hint2(idx.box, n, a.k)
grids = {"grid": idx.grid}
if a.levels:
    from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402
    skeys, _ = K.morton(idx.pts[:n], idx.box, with_iota=False)  # keys of the sorted points
    for g in [int(x) for x in a.levels.split(",")]:  # finest level (cells at g - 2)
        grids[f"grid-L{g}"] = E.GridIndex(K.grid_build(idx.pts, skeys, n, idx.box, g - 2), g - 2, idx.box)
res = {}
for impl in list(grids) + ["rows"]:
    idx.grid = grids.get(impl)
    for r in range(a.reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = E.KnnStats()
        d2 = E.query(idx, cfg, hint2, stats=st if r == 0 else None)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        c = st.counters
        extra = ""
        if r == 0 and c.get("waves"):
            extra = (f" evals/query {c['evals'] / max(1, c['waves']):.0f} (per lane)"
                     f" passes/wave {c['hist_passes'] / c['waves']:.2f} failed {c.get('failed_lanes', 0)}"
                     f" ovf {c.get('overflow_lanes', 0)} udf {c.get('underflow_lanes', 0)}"
                     f" refine {c.get('refine_lanes', 0)} cells/wave {c['leaves'] / c['waves']:.1f}"
                     f" segs/wave {c['nodes'] / c['waves']:.1f}")
        if r == 0 and c.get("prof_wave"):
            tot = c["prof_wave"]
            extra += "\n    cycle profile (% of wave time): " + str(
                {nm: round(100.0 * c.get("prof_" + nm, 0) / tot, 1)
                 for nm in ("proc_hist", "proc_collect", "walk_hist", "walk_collect")})
            if impl != "rows":
                extra += f" evals/query hist {c['recorded_leaves'] / c['waves']:.0f} collect {c['collect_steps'] / c['waves']:.0f}"
        print(f"[{impl}] knn {n} pts k={a.k} ({a.dist}): {dt:.4f} s{extra}", flush=True)
    res[impl] = d2.clone()
same = all(torch.equal(res[g].view(torch.int32), res["rows"].view(torch.int32)) for g in grids)
print("grid == rows bitwise:", same, flush=True)
if not same:
    bad = (res["grid"] != res["rows"]).nonzero().view(-1)
    print("mismatches:", bad.numel(), bad[:10].tolist(), res["grid"][bad[:5]].tolist(), res["rows"][bad[:5]].tolist())
    sys.exit(1)
