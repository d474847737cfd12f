"""Reference-faithful distributed schedules ("--mode ring" / "--mode peer").

These reproduce the reference's communication structure on top of the ref-algo kernels
(ops/refalgo.py) — they are the measured baseline of BASELINE.md and a fidelity check,
not the fast path (pipelines.py):

* ``ring_knn`` — unorderedData variant (unorderedDataVariant.cu:173-205):
  every rank builds a left-balanced tree over its block of the file; queries stay put
  while trees rotate rank -> rank+1 for P-1 rounds (count exchange, then payload, as
  grouped point-to-point sends over RCCL); each round resumes every query's persisted
  k-heap.
* ``peer_knn`` — prePartitionedData variant (prePartitionedDataVariant.cu:284-357, S3):
  rank AABBs and counts are all-gathered; each round every rank pulls at most one unseen
  peer tree — the closest by box gap among peers closer than its current max k-NN
  radius (Sattolo tie-break permutation) — and serves its own tree to every requester;
  the job ends when every request is -1.
"""
from __future__ import annotations

import math

import torch

from .. import _native
from ..models import knn_engine as E
from ..ops import kernels as K
from ..ops import refalgo as R
from .comm import Comm
from .pipelines import PhaseTimer, RunInfo


# Per query and rank, besides its k-heap: the point in the left-balanced tree copy and in
# the query array (2 x 12 B), its output (4 B) and the builder's tag and sort scratch.
REF_BYTES_PER_POINT = 40
REF_SLACK = 2 << 30


def ref_memory_bytes(n_local: int, k: int) -> int:
    """Device bytes a ref-algo rank needs for n_local points: the reference's N·k·8 B of
    candidate heaps (unorderedDataVariant.cu:168, D4) plus the trees and queries."""
    return n_local * k * 8 + n_local * REF_BYTES_PER_POINT + REF_SLACK


def check_ref_fits(n_local: int, k: int, capacity: int, ranks: int = 1) -> None:
    """Refuse a ref-algo run whose heaps do not fit (raises ValueError with the arithmetic):
    the reference allocates N/P·k·8 B of heaps per rank up front and would fail there."""
    need = ref_memory_bytes(n_local, k)
    if need > capacity:
        heaps = n_local * k * 8
        raise ValueError(
            f"ref-algo (ring/peer) does not fit: {n_local:,} queries per rank x k={k} x 8 B = "
            f"{heaps / 1e9:.1f} GB of k-heaps (the reference's N/P*k*8 B, unorderedDataVariant.cu:168) "
            f"+ {(need - heaps) / 1e9:.1f} GB of trees/queries/scratch = {need / 1e9:.1f} GB > "
            f"{capacity / 1e9:.1f} GB of device memory per rank; use at least "
            f"{max(ranks + 1, math.ceil(ranks * need / max(capacity, 1)))} ranks or --mode halo")


def ring_knn(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig, info: RunInfo | None = None,
             overlap: bool = True) -> torch.Tensor:
    """Ring rotation (unorderedDataVariant.cu:173-205), double-buffered: the tree sizes
    are all-gathered once up front (the reference exchanges one count per round,
    :183-187 — the same numbers), and round r+1's tree exchange (send the tree held in
    round r to rank+1, receive rank-1's into the other buffer) is posted on a
    high-priority side stream before round r's query is launched, so the xGMI transfer
    runs under the k-NN kernel (the reference waits for each exchange, D6). `overlap`
    False: the reference's sequential order (same results)."""
    info = info or RunInfo(PhaseTimer(False, points.device))
    info.timer.start()
    points = points.contiguous()
    n = points.shape[0]
    dev = points.device
    size, rank = comm.size, comm.rank
    tree, _ = R.build_lbt(points)
    info.timer.mark("build")
    heaps = R.alloc_heaps(n, cfg.k, dev)
    counts = comm.allgather(torch.tensor([n], dtype=torch.int64, device=comm.device)).view(-1).cpu().tolist()
    nxt, prv = (rank + 1) % size, (rank - 1 + size) % size
    gpu = dev.type == "cuda"
    side = torch.cuda.Stream(dev, priority=torch.cuda.Stream.priority_range()[1]) if gpu and overlap else None
    compute = torch.cuda.current_stream(dev) if gpu else None
    cur, cur_n = tree, n
    for rnd in range(size):
        got = None
        if rnd + 1 < size:
            recv_n = counts[(rank - rnd - 1) % size]  # the tree rank-1 holds this round
            if side is not None:
                side.wait_stream(compute)  # `cur` complete (received / built) on the device
                with torch.cuda.stream(side):
                    (got,) = comm.p2p([(nxt, cur[:cur_n])], [(prv, (recv_n, 3), torch.float32)])
                cur.record_stream(side)
            else:
                (got,) = comm.p2p([(nxt, cur[:cur_n])], [(prv, (recv_n, 3), torch.float32)])
            info.timer.mark("ring_exchange")
        R.run_query(cur, cur_n, points, heaps, cfg.k, cfg.cut2, init=(rnd == 0))
        info.timer.mark("knn_rounds")
        if got is not None:
            if side is not None:
                compute.wait_stream(side)  # round r+1 reads the received tree
                got.record_stream(compute)
            cur, cur_n = got, recv_n
    out = R.extract(heaps, n, cfg.k)
    info.timer.mark("return")
    return out


def peer_knn(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig, info: RunInfo | None = None,
             log=None) -> torch.Tensor:
    info = info or RunInfo(PhaseTimer(False, points.device))
    info.timer.start()
    points = points.contiguous()
    n = points.shape[0]
    dev = points.device
    size, me = comm.size, comm.rank
    host = _native.host()
    box = K.bounds(points)[0:6].float().cpu().contiguous()
    all_boxes = comm.allgather(box.to(comm.device)).cpu().contiguous()          # [P, 6]
    counts = comm.allgather(torch.tensor([n], dtype=torch.int64, device=comm.device)).view(-1).cpu().tolist()
    perm = (torch.zeros(size, dtype=torch.int32)).contiguous()
    host.lsk_peer_permutation(me, size, perm.data_ptr())
    my_tree, _ = R.build_lbt(points)
    info.timer.mark("build")
    heaps = R.alloc_heaps(n, cfg.k, dev)
    rmax = torch.zeros(1, dtype=torch.float32, device=dev)
    seen = torch.zeros(size, dtype=torch.uint8)
    initialised = False
    for rnd in range(size):
        comm.barrier()
        if me == 0 and log is not None:
            log(f"round {rnd}")
        if rnd == 0:
            work, wn = my_tree, n
            seen[me] = 1
        else:
            cutoff = float(rmax.cpu().item())
            peer = host.lsk_peer_choose(box.data_ptr(), all_boxes.data_ptr(), size, cutoff,
                                        seen.data_ptr(), perm.data_ptr())
            req = comm.allgather(torch.tensor([peer], dtype=torch.int64, device=comm.device)).view(-1).cpu().tolist()
            if all(r == -1 for r in req):
                break
            sends = [(j, my_tree) for j in range(size) if req[j] == me]
            recvs = [(peer, (counts[peer], 3), torch.float32)] if peer >= 0 else []
            got = comm.p2p(sends, recvs)
            info.timer.mark("peer_exchange")
            if peer >= 0:
                seen[peer] = 1
                work, wn = got[0], counts[peer]
            else:
                wn = 0
        if wn:
            rmax.zero_()
            R.run_query(work, wn, points, heaps, cfg.k, cfg.cut2, init=not initialised, rmax=rmax)
            initialised = True
        info.timer.mark("knn_rounds")
    if not initialised:  # empty rank: nothing queried
        R.run_query(my_tree, 0, points, heaps, cfg.k, cfg.cut2, init=True)
    out = R.extract(heaps, n, cfg.k)
    info.timer.mark("return")
    info.counts["peer_rounds"] = rnd
    return out
