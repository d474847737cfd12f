"""Sampled brute-force verification (utils/verify.py): threshold math and the
all-ranks count check, on the CPU (LoopbackComm ranks) against the CPU oracle."""
import math

import numpy as np
import pytest
import torch

from mpi_cuda_largescaleknn_amd.ops import kernels as K
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm, run_loopback
from mpi_cuda_largescaleknn_amd.utils import verify as V


def test_sqrt_thresholds_bracket_exactly():
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.random(200, dtype=np.float32) * 3, [0.0, 1.0, 1e-20, 3e30]]).astype(np.float32)
    thr = V.sqrt_thresholds(v)
    for j, x in enumerate(v):
        lo, hi = thr[j]
        assert np.sqrt(lo) >= x and np.sqrt(hi) > x
        # nothing below lo maps to >= x, nothing below hi maps to > x
        below_lo = np.nextafter(lo, np.float32(0)) if lo > 0 else None
        if below_lo is not None:
            assert np.sqrt(below_lo) < x
        below_hi = np.nextafter(hi, np.float32(0)) if hi > 0 else None
        if below_hi is not None:
            assert np.sqrt(below_hi) <= x
    inf = V.sqrt_thresholds(np.array([np.inf], dtype=np.float32))
    assert np.isinf(inf).all()


def test_sample_ids_spread_and_deterministic():
    ids = V.sample_ids(10**9, 256)
    assert ids == V.sample_ids(10**9, 256) and len(ids) == 256
    assert min(ids) >= 0 and max(ids) < 10**9 and max(ids) - min(ids) > 9 * 10**8
    assert V.sample_ids(10, 256) == list(range(10))


@pytest.mark.parametrize("size", [1, 3])
def test_sampled_exact_accepts_oracle_and_rejects_wrong(size):
    g = torch.Generator().manual_seed(3)
    pts = torch.rand((6000, 3), generator=g)
    pts[100:140] = pts[7]  # exact copies: zero distances and ties
    k = 16
    ref = K.finalize_distances(K.kth_cpu(pts, pts, k, math.inf))
    bad = ref.clone()
    ids = V.sample_ids(6000, 64)
    bad[ids[5]] = torch.nextafter(bad[ids[5]], torch.tensor(2.0))  # one ulp off
    bad[ids[9]] = float("nan")

    def fn(comm, out):
        b, e = 6000 * comm.rank // comm.size, 6000 * (comm.rank + 1) // comm.size
        return V.sampled_exact(comm, pts[b:e], out[b:e], b, 6000, k, 64)

    for out, want_bad in ((ref, []), (bad, sorted([ids[5], ids[9]]))):
        res = [fn(SingleComm(), out)] if size == 1 else run_loopback(size, lambda c: fn(c, out))
        for r in res:
            assert r["samples"] == 64
            assert r["mismatch_ids"] == want_bad


def test_sampled_exact_inf_when_k_exceeds_n():
    pts = torch.rand((50, 3))
    out = torch.full((50,), float("inf"))
    r = V.sampled_exact(SingleComm(), pts, out, 0, 50, 51, 20)
    assert r["exact"] == r["samples"] == 20
    r = V.sampled_exact(SingleComm(), pts, out, 0, 50, 50, 20)
    assert r["exact"] == 0
