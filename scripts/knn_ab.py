"""The grid k-NN pass alone on one index, for library A/B (LSKNN_HIP_LIB=<variant .so>):
kernel time (median of --reps), kernel counters and a SHA-256 of the output bits, so two
libraries' logs can be compared for bit-identical results.

    python scripts/knn_ab.py --points 1e8 --k 100 [--reps 5] [--dist uniform] [--oracle 512]
"""
import argparse
import hashlib
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd import _native  # noqa: E402
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--points", type=float, nargs="+", default=[1e6])
ap.add_argument("--k", type=int, nargs="+", default=[100])
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dist", default="uniform")
ap.add_argument("--grid", default="on", help="knn_engine.GRID: on / auto / off")
ap.add_argument("--oracle", type=int, default=0, help="check this many sampled queries against the CPU oracle")
a = ap.parse_args()
E.GRID = a.grid
print("library:", _native.hip()._name, flush=True)

for npts in a.points:
    n = int(npts)
    g = torch.Generator(device="cuda").manual_seed(n % 1000003)
    if a.dist == "uniform":
        p = torch.rand((n, 3), generator=g, device="cuda")
    else:
        sys.path.insert(0, "tests")
        from datasets import GENERATORS  # noqa: E402
        p = GENERATORS[a.dist](n, seed=5).to("cuda")
    idx = E.build_index(p, grid=a.grid != "off")
    for k in a.k:
        cfg = E.KnnConfig(k=k)
        hint2 = E.radius_hint2(idx.box, idx.n, k)
        times, out, st = [], None, None
        for r in range(a.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            s = E.KnnStats() if r == 0 else None
            d2 = E.query(idx, cfg, hint2, stats=s)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t)
            if r == 0:
                out, st = d2.clone(), s
        t = sorted(times)[len(times) // 2]
        c = st.counters
        w = max(c.get("waves", 1), 1)
        h = hashlib.sha256(out.view(torch.int32).cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"n={n} k={k} {a.dist}: {t * 1e3:.2f} ms (min {min(times) * 1e3:.2f})  evals/q={c.get('evals', 0) / w:.0f} "
              f"cells/w={c.get('leaves', 0) / w:.1f} segs/w={c.get('nodes', 0) / w:.1f} "
              f"hist adds/w={c.get('collect_nodes', 0) / w:.0f} passes={c.get('hist_passes', 0) / w:.3f} ovf={c.get('overflow_lanes', 0)} "
              f"low={c.get('underflow_lanes', 0)} refine={c.get('refine_lanes', 0)} "
              f"fail={c.get('failed_lanes', 0)} fallback={c.get('fallback_queries', 0)} sha={h}", flush=True)
        if c.get("prof_rows_entry"):  # LSK_ROWQ_STATS build
            print(f"  row streams: steps/w {c['prof_rows_entry'] / w:.1f}  real candidates per row "
                  f"{c['prof_rows_in'] / w / 4:.0f} of {16 * c['prof_rows_entry'] / w:.0f} slots  "
                  f"refills/w {c.get('list_invalid_waves', 0) / w:.1f}", flush=True)
        if c.get("prof_wave"):
            tot = c["prof_wave"]
            names = ["proc_hist", "proc_collect", "walk_hist", "walk_collect", "quarters", "inner_nodes", "select"]
            print("  cycle profile (% of wave):", {x: round(100 * c.get("prof_" + x, 0) / tot, 1) for x in names},
                  f"hist evals/q {c.get('recorded_leaves', 0) / w:.0f} collect evals/q {c.get('collect_steps', 0) / w:.0f}",
                  flush=True)
        if a.oracle:
            sel = torch.randperm(n, generator=torch.Generator().manual_seed(7))[:a.oracle]
            ref = K.kth_cpu(idx.pts[:n].cpu(), idx.pts[:n].cpu()[sel], k, float("inf"))
            got = out.cpu()[sel]
            bad = int((ref.view(torch.int32) != got.view(torch.int32)).sum())
            print(f"  oracle: {a.oracle - bad}/{a.oracle} exact", flush=True)
