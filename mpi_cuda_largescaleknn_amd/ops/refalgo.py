"""Tensor wrappers of the "ref-algo" kernels (csrc/hip/refalgo.hip, CPU twin in
csrc/host/refalgo_cpu.cpp): the reference's algorithm — left-balanced k-d tree,
stack-free traversal, k-max-heaps persisted in global memory — re-implemented for
gfx950 as the measured baseline and as the engine of the reference-faithful ring /
peer schedules."""
from __future__ import annotations

import ctypes as C

import torch

from .. import _native
from . import kernels as K


def _levels(n: int) -> int:
    d = 0
    while ((1 << d) - 1) < n:
        d += 1
    return d


def build_lbt(points: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Left-balanced k-d tree (cukd::buildTree semantics) -> (tree points [n,3] in tree
    order, int32 ids: tree node i holds input row ids[i])."""
    points = points.contiguous()
    n = points.shape[0]
    if not K.is_gpu(points):
        out = torch.empty_like(points)
        ids = torch.empty(n, dtype=torch.int32)
        _native.host().lsk_cpu_lbt_build(points.data_ptr(), n, out.data_ptr(), ids.data_ptr())
        return out, ids
    lib = _native.hip()
    dev = points.device
    s = K._stream(points)
    pts = points
    ids = torch.arange(n, dtype=torch.int32, device=dev)
    tags = torch.zeros(n, dtype=torch.int32, device=dev)
    levels = _levels(n)
    keys = torch.empty(n, dtype=torch.int32, device=dev)
    iota = torch.empty(n, dtype=torch.int32, device=dev)
    for level in range(levels):
        # stable sort by coord, then stable sort by tag => order by (tag, coord)
        K.check(lib.lsk_hip_lbt_keys(pts.data_ptr(), n, level % 3, keys.data_ptr(), iota.data_ptr(), s), "lbt_keys")
        _, perm1 = K.sort_pairs(keys, iota, 32)
        t1 = torch.empty_like(tags)
        K.check(lib.lsk_hip_gather_u32(tags.data_ptr(), perm1.data_ptr(), n, t1.data_ptr(), s), "gather_u32")
        iota2 = torch.arange(n, dtype=torch.int32, device=dev)
        tags, perm2 = K.sort_pairs(t1, iota2, max(1, level + 1))
        perm = torch.empty_like(perm2)
        K.check(lib.lsk_hip_gather_u32(perm1.data_ptr(), perm2.data_ptr(), n, perm.data_ptr(), s), "gather_u32")
        pts = K.gather3(pts, perm)
        ids2 = torch.empty_like(ids)
        K.check(lib.lsk_hip_gather_u32(ids.data_ptr(), perm.data_ptr(), n, ids2.data_ptr(), s), "gather_u32")
        ids = ids2
        tags = tags.clone()
        K.check(lib.lsk_hip_lbt_retag(tags.data_ptr(), n, level, s), "lbt_retag")
    # every point now carries its node id: final order = sort by tag
    iota3 = torch.arange(n, dtype=torch.int32, device=dev)
    _, perm = K.sort_pairs(tags, iota3, max(1, levels + 1))
    pts = K.gather3(pts, perm)
    ids2 = torch.empty_like(ids)
    K.check(lib.lsk_hip_gather_u32(ids.data_ptr(), perm.data_ptr(), n, ids2.data_ptr(), s), "gather_u32")
    return pts, ids2


def alloc_heaps(nq: int, k: int, device) -> torch.Tensor:
    """N·k·8 B of candidate heaps (the reference's d_cand, U:168)."""
    return torch.empty(nq * k, dtype=torch.int64, device=device)


def run_query(tree: torch.Tensor, n: int, queries: torch.Tensor, heaps: torch.Tensor, k: int,
              cut2: float, init: bool, rmax: torch.Tensor | None = None, id_base: int = 0) -> None:
    """runQuery: add every point of `tree` into each query's persisted heap."""
    nq = queries.shape[0]
    if K.is_gpu(queries):
        K.check(_native.hip().lsk_hip_refalgo_knn(tree.data_ptr(), n, queries.data_ptr(), nq, heaps.data_ptr(),
                                                  k, C.c_float(cut2), int(init),
                                                  None if rmax is None else rmax.data_ptr(), id_base,
                                                  K._stream(queries)), "refalgo_knn")
        return
    _native.host().lsk_cpu_refalgo_knn(tree.data_ptr(), n, queries.data_ptr(), nq, heaps.data_ptr(), k,
                                       C.c_float(cut2), int(init), None if rmax is None else rmax.data_ptr(),
                                       id_base, K._nthreads())


def extract(heaps: torch.Tensor, nq: int, k: int) -> torch.Tensor:
    """extractFinalResult: sqrt of each heap's top unless inf."""
    out = torch.empty(nq, dtype=torch.float32, device=heaps.device)
    if K.is_gpu(heaps):
        K.check(_native.hip().lsk_hip_refalgo_extract(heaps.data_ptr(), nq, k, out.data_ptr(), K._stream(heaps)),
                "refalgo_extract")
    else:
        _native.host().lsk_cpu_refalgo_extract(heaps.data_ptr(), nq, k, out.data_ptr())
    return out
