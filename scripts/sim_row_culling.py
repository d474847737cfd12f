"""Candidates per query of the cell-grid kernel's wave-level culling (64-query box) vs
per-ROW culling (four 16-query boxes, each with its own radius), at grandchild-cell
granularity, from exact k-th distances (scipy cKDTree) on sampled waves:

    python scripts/sim_row_culling.py N GRANDCHILD_LEVEL WAVES     # e.g. 1e7 7 150

"current": wave box + the wave's largest band top (knn_grid.hip today, ~batch rounding);
"rows/cell-sync": rows stepping 16 candidates in lockstep, synchronised per level-lc cell;
"rows ideal": rows streaming across cells (max over rows of their candidate totals).
Result (1e7, level 7, 150 waves): current ~1578, per-cell sync 1473 (0.93), ideal 1017
(0.64) — docs/ARCHITECTURE.md §2d, next steps.
"""
import sys, numpy as np, torch
sys.path.insert(0, '/root/repo')
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from scipy.spatial import cKDTree
n = int(float(sys.argv[1])); k = 100; lvl = int(sys.argv[2]); nw = int(sys.argv[3])
g = torch.Generator().manual_seed(1)
p = torch.rand((n, 3), generator=g)
idx = E.build_index(p)
pts = idx.pts[:n].numpy().astype(np.float64)
box = idx.box.numpy()
sh = 10 - lvl
q = np.clip(((pts - box[0:3]) * box[6]), 0, 1023).astype(np.int64) >> sh
side = (box[7] / 1024.0) * (1 << sh)
keys = (q[:, 0] << 20) | (q[:, 1] << 10) | q[:, 2]
uk, cnt = np.unique(keys, return_counts=True)
cq = np.stack([uk >> 20, (uk >> 10) & 1023, uk & 1023], 1)
parent = (cq >> 2)
pkey = (parent[:, 0] << 20) | (parent[:, 1] << 10) | parent[:, 2]
lo = box[0:3] + cq * side; hi = lo + side
tree = cKDTree(pts)
rng = np.random.default_rng(0)
waves = rng.choice(n // 64, nw, replace=False)
cur = []; rows = []; rows_ideal = []
def gap2(blo, bhi):
    gap = np.maximum(0, np.maximum(lo - bhi, blo - hi))
    return (gap ** 2).sum(1)
for w in waves:
    Q = pts[w*64:(w+1)*64]
    d, _ = tree.query(Q, k)
    kth = d[:, -1] * 1.045
    gw = gap2(Q.min(0), Q.max(0)) <= kth.max() ** 2
    # current: per cell, needed counts in 4-batches (approx: per grandchild run, ceil/4*4 at segment level ~ +2)
    cur.append(cnt[gw].sum() + 2 * len(np.unique(pkey[gw])) * 2)
    need = [gap2(Q[r*16:(r+1)*16].min(0), Q[r*16:(r+1)*16].max(0)) <= kth[r*16:(r+1)*16].max() ** 2 for r in range(4)]
    cost = 0
    for pc in np.unique(pkey[gw]):
        m = pkey == pc
        steps = max(int(np.ceil(cnt[m & need[r]].sum() / 16)) for r in range(4))
        cost += 16 * steps
    rows.append(cost)
    rows_ideal.append(max(cnt[need[r]].sum() for r in range(4)))
print(f"n={n} lvl {lvl}: current ~{np.mean(cur):.0f}  rows/cell-sync {np.mean(rows):.0f} ({np.mean(rows)/np.mean(cur):.2f})  rows ideal {np.mean(rows_ideal):.0f} ({np.mean(rows_ideal)/np.mean(cur):.2f})")
