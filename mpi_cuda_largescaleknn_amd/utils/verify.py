"""Sampled brute-force verification of a distributed k-th-NN distance result.

The reference's only check is a disabled dump of every 16th result
(unorderedDataVariant.cu:215-227, prePartitionedDataVariant.cu:366-378). Here
:func:`sampled_exact` verifies S sampled outputs of a finished run against ALL points,
without trusting any part of the pipeline (no tree, no selection, no sort):

1. the owners of the sampled global ids contribute (x, y, z, claimed value) to one
   all-reduced [S, 4] table (every other rank contributes zeros);
2. for each claimed value v the host finds the float thresholds
   t_lo = min{x : sqrtf(x) >= v} and t_hi = min{x : sqrtf(x) > v} (bisection on the
   float bits; numpy's float32 sqrt is IEEE correctly rounded like the kernels' sqrtf);
3. every rank counts, over its own shard, the canonical squared distances below both
   thresholds (``lsk_hip_count_below`` / ``lsk_cpu_count_below``); the counts are summed;
4. v is exact iff lt < k <= le (sqrtf is monotone, so v = sqrtf(k-th smallest d2)
   exactly when fewer than k values map below v and at least k map to <= v); an `inf`
   claim is exact iff fewer than k points exist.

Cost: S x N canonical distances, ~20-30 ms for 256 samples over 1B points on one MI355X.
No ``-r`` cutoff (the bench has none).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import _native
from ..ops import kernels as K

INF_BITS = 0x7F800000


def sample_ids(n_total: int, nsamp: int = 256) -> list[int]:
    """Deterministic, well-spread global ids (independent of the rank count)."""
    if n_total <= 0:
        return []
    ids = {(i * 2654435761 + 40503) % n_total for i in range(min(nsamp, n_total))}
    return sorted(ids)


def sqrt_thresholds(v: np.ndarray) -> np.ndarray:
    """[S] float32 claimed distances -> [S, 2] float32 (t_lo, t_hi), see module doc."""
    v = np.asarray(v, dtype=np.float32)

    def first_bits(pred):
        lo = np.zeros(v.shape, dtype=np.int64)               # pred(lo) may be false
        hi = np.full(v.shape, INF_BITS, dtype=np.int64)      # pred(inf) assumed true
        for _ in range(32):
            mid = (lo + hi) // 2
            x = mid.astype(np.uint32).view(np.float32)
            with np.errstate(invalid="ignore"):
                ok = pred(np.sqrt(x))
            hi = np.where(ok, mid, hi)
            lo = np.where(ok, lo, mid)
        # smallest bits with pred true: lo < answer <= hi; 0 itself may qualify
        zero_ok = pred(np.zeros_like(v))
        return np.where(zero_ok, 0, hi).astype(np.uint32).view(np.float32)

    t_lo = first_bits(lambda s: s >= v)
    t_hi = first_bits(lambda s: s > v)
    inf = ~np.isfinite(v)
    t_lo = np.where(inf, np.float32(np.inf), t_lo)
    t_hi = np.where(inf, np.float32(np.inf), t_hi)
    return np.stack([t_lo, t_hi], axis=1).astype(np.float32)


def count_below(pts: torch.Tensor, q: torch.Tensor, thr: torch.Tensor, counts: torch.Tensor,
                chunk: int = 1 << 26) -> None:
    """counts[j] += (#d2 < thr[j,0], #d2 < thr[j,1]) over pts (device: q/thr/counts live on
    the counting device; host `pts` are streamed to it in chunks)."""
    nq = q.shape[0]
    if counts.device.type == "cuda":
        lib = _native.hip()
        dev = counts.device
        n = pts.shape[0]
        for s in range(0, n, chunk):
            part = pts[s:s + chunk]
            part = part.to(dev, non_blocking=True) if part.device != dev else part
            part = part.contiguous()
            for j in range(0, nq, 1024):  # (the kernel takes <= 1024 queries per launch)
                m = min(1024, nq - j)
                K.check(lib.lsk_hip_count_below(part.data_ptr(), part.shape[0], q[j:].data_ptr(), thr[j:].data_ptr(),
                                                m, counts[j:].data_ptr(), K._stream(part)), "count_below")
        return
    c = np.zeros((nq, 2), dtype=np.uint64)
    p = pts.contiguous().float()
    _native.host().lsk_cpu_count_below(p.data_ptr(), p.shape[0], q.contiguous().data_ptr(),
                                       thr.contiguous().data_ptr(), nq, c.ctypes.data, K._nthreads())
    counts += torch.from_numpy(c.astype(np.int64))


def sampled_exact(comm, local_pts: torch.Tensor, local_out: torch.Tensor, begin: int, n_total: int,
                  k: int, nsamp: int = 256) -> dict:
    """Check `nsamp` sampled outputs of a block-partitioned run (this rank holds global ids
    [begin, begin + len)) against all points. Collective: every rank must call it.
    Returns {"samples", "exact", "mismatch_ids"} (equal on every rank)."""
    dev = comm.device
    ids = sample_ids(n_total, nsamp)
    S = len(ids)
    n_local = local_pts.shape[0]
    tab = torch.zeros((max(S, 1), 4), dtype=torch.float32)
    mine = [(j, g - begin) for j, g in enumerate(ids) if begin <= g < begin + n_local]
    if mine:
        rows = torch.tensor([r for _, r in mine], dtype=torch.int64)
        js = torch.tensor([j for j, _ in mine], dtype=torch.int64)
        tab[js, 0:3] = local_pts[rows.to(local_pts.device)].float().cpu()
        tab[js, 3] = local_out[rows.to(local_out.device)].float().cpu()
    tab = tab.to(dev)
    comm.allreduce_(tab, "sum")
    tab = tab.cpu()[:S]
    v = tab[:, 3].numpy()
    thr = torch.from_numpy(sqrt_thresholds(v))
    q = tab[:, 0:3].contiguous()
    counts = torch.zeros((S, 2), dtype=torch.int64, device=dev)
    if S:
        count_below(local_pts, q.to(dev), thr.to(dev), counts)
    comm.allreduce_(counts, "sum")
    c = counts.cpu().numpy()
    exact = []
    for j in range(S):
        lt, le = int(c[j, 0]), int(c[j, 1])
        if np.isnan(v[j]):
            ok = False
        elif np.isinf(v[j]):
            ok = lt < k               # inf: fewer than k points in total
        else:
            ok = lt < k <= le
        exact.append(ok)
    bad = [ids[j] for j in range(S) if not exact[j]]
    return {"samples": S, "exact": S - len(bad), "mismatch_ids": bad[:16]}
