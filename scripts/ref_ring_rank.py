"""One rank's whole share of the reference algorithm's ring at N points over P ranks,
on one GPU: the rank's N/P queries against each of the P trees of N/P points (its own,
then the ones the ring would bring), k-heaps persisted across rounds — the per-rank
compute of the P-GPU ring, without the tree transfers (P-1 sends of N/P·12 B over xGMI,
added in BASELINE.md). Prints per-round times and checks the result against this
framework's k-NN of the whole set.

    python scripts/ref_ring_rank.py [N] [P] [k]"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import refalgo as R  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 8
k = int(sys.argv[3]) if len(sys.argv) > 3 else 100
m = n // P
g = torch.Generator(device="cuda").manual_seed(1)
pts = torch.rand((m * P, 3), generator=g, device="cuda")  # rank r holds rows [r*m, (r+1)*m)
q = pts[:m]  # rank 0's queries


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


t_all = time.perf_counter()
heaps = R.alloc_heaps(m, k, pts.device)
rounds = []
for rnd in range(P):
    src = (0 - rnd) % P  # the ring brings rank -rnd's tree in round rnd
    a = ev()
    tree, _ = R.build_lbt(pts[src * m:(src + 1) * m])
    b = ev()
    R.run_query(tree, m, q, heaps, k, float("inf"), init=(rnd == 0))
    c = ev()
    c.synchronize()
    rounds.append({"round": rnd, "tree_build_ms": round(a.elapsed_time(b), 1), "query_ms": round(b.elapsed_time(c), 1)})
    print(json.dumps(rounds[-1]), flush=True)
    del tree
out = R.extract(heaps, m, k)
torch.cuda.synchronize()
wall = time.perf_counter() - t_all
del heaps
torch.cuda.empty_cache()
ref = E.knn_distances(pts, k)[:m]
equal = bool(torch.equal(out, ref))
q_ms = sum(r["query_ms"] for r in rounds)
print("SUMMARY", json.dumps({"n": m * P, "ranks": P, "k": k, "queries_per_rank": m, "query_ms_total": round(q_ms, 1),
                             "own_tree_build_ms": rounds[0]["tree_build_ms"], "wall_s": round(wall, 2),
                             "equal_to_framework": equal}), flush=True)
