"""Tensor-level wrappers around the gfx950 kernels (and their CPU counterparts).

Every function takes/returns torch tensors. CUDA (ROCm) tensors run the hand-written
HIP kernels of ``csrc/hip`` on torch's current stream; CPU tensors run the C++ host
runtime (``csrc/host``) or plain torch — that path exists for the CPU oracle, the
``--device cpu`` mode and multi-process ``gloo`` tests. A CUDA tensor never falls back
to the CPU path: if the kernel library is missing the call raises.

uint32 data (Morton keys, indices) is stored in ``torch.int32`` tensors (same bits).
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from .. import _native
from .._native import GridView, KnnArgs, TreeView, check

BUCKET = 64
PAD_POINTS = 64  # readable padding required after point arrays read by the knn kernel


def _nthreads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


# --------------------------------------------------------------------------- bounds
def bounds(pts: torch.Tensor) -> torch.Tensor:
    """AABB + Morton cube of an [n,3] float32 tensor -> [8] (lo.xyz, hi.xyz, scale, extent)."""
    n = pts.shape[0]
    if is_gpu(pts):
        lib = _native.hip()
        box = torch.empty(8, dtype=torch.float32, device=pts.device)
        ws = torch.empty(lib.lsk_hip_bounds_ws_bytes(n) // 4 + 1, dtype=torch.float32, device=pts.device)
        check(lib.lsk_hip_bounds(_ptr(pts), n, _ptr(box), _ptr(ws), _stream(pts)), "bounds")
        return box
    box = torch.empty(8, dtype=torch.float32)
    _native.host().lsk_cpu_bounds(_ptr(pts.contiguous()), n, _ptr(box), _nthreads())
    return box_finalize(box)


def box_finalize(box: torch.Tensor) -> torch.Tensor:
    """Recompute the Morton cube (box[6:8]) from box[0:6]."""
    if is_gpu(box):
        check(_native.hip().lsk_hip_box_finalize(_ptr(box), _stream(box)), "box_finalize")
        return box
    lo, hi = box[0:3], box[3:6]
    ex = float(torch.max(hi - lo)) if bool(torch.all(torch.isfinite(box[0:6]))) else 0.0
    ok = ex > 0 and math.isfinite(ex)
    box[6] = 1024.0 / ex if ok else 0.0
    box[7] = ex if ok else 0.0
    return box


# --------------------------------------------------------------------------- curve keys + sort
CURVES = {"morton": 0, "hilbert": 1}
# Space-filling curve of the sort keys: Hilbert runs are spatially much tighter than
# Z-order runs (fewer tree nodes and quarters per query, smaller halos); Morton kept
# for A/B measurements (LSKNN_CURVE=morton).
CURVE = os.environ.get("LSKNN_CURVE", "hilbert")


def morton(pts: torch.Tensor, box: torch.Tensor, with_iota: bool = True, curve: str | None = None):
    """30-bit space-filling-curve keys (Hilbert by default, `CURVE`) of pts in the cube
    of `box`; returns (keys, iota)."""
    cid = CURVES[curve or CURVE]
    n = pts.shape[0]
    keys = torch.empty(n, dtype=torch.int32, device=pts.device)
    vals = torch.empty(n, dtype=torch.int32, device=pts.device) if with_iota else None
    if is_gpu(pts):
        check(_native.hip().lsk_hip_morton(_ptr(pts), n, _ptr(box), _ptr(keys), _ptr(vals), cid,
                                           _stream(pts)), "morton")
        return keys, vals
    b = box.detach().cpu()
    origin = b[0:3].contiguous()
    _native.host().lsk_cpu_morton(_ptr(pts.contiguous()), n, _ptr(origin), C.c_float(float(b[6])),
                                  _ptr(keys), cid, _nthreads())
    if vals is not None:
        vals.copy_(torch.arange(n, dtype=torch.int32))
    return keys, vals


def morton_into(pts: torch.Tensor, box: torch.Tensor, keys: torch.Tensor, vals: torch.Tensor | None,
                base: int, flag: torch.Tensor | None = None, curve: str | None = None) -> None:
    """GPU: keys of pts (and vals = base + i) written into the given (slice) tensors; with
    a device int32 `flag` nothing is written unless flag != 0 (decided on the device)."""
    check(_native.hip().lsk_hip_morton_ex(_ptr(pts), pts.shape[0], _ptr(box), _ptr(keys),
                                          _ptr(vals) if vals is not None else None, CURVES[curve or CURVE],
                                          int(base), _ptr(flag) if flag is not None else None,
                                          _stream(pts)), "morton_ex")


def sort_pairs(keys: torch.Tensor, vals: torch.Tensor, key_bits: int = 30):
    """Stable sort of (key, value) int32 pairs by the low `key_bits` bits of key (unsigned)."""
    n = keys.shape[0]
    if not is_gpu(keys):
        k64 = keys.to(torch.int64) & ((1 << 32) - 1)
        if key_bits < 32:
            k64 = k64 & ((1 << key_bits) - 1)
        order = torch.sort(k64, stable=True).indices
        return keys[order], vals[order]
    lib = _native.hip()
    ka = torch.empty_like(keys)
    va = torch.empty_like(vals)
    ws = torch.empty(lib.lsk_hip_sort_ws_bytes(n), dtype=torch.uint8, device=keys.device)
    alt = C.c_int(0)
    check(lib.lsk_hip_sort_pairs(_ptr(keys), _ptr(vals), _ptr(ka), _ptr(va), n, key_bits, _ptr(ws),
                                 C.byref(alt), _stream(keys)), "sort_pairs")
    return (ka, va) if alt.value else (keys, vals)


def sort_keys_iota(keys: torch.Tensor, key_bits: int = 30):
    """sort_pairs(keys, arange(n)) without the arange: the GPU sort's first pass generates
    the values (no 4-byte-per-point array written and read back)."""
    n = keys.shape[0]
    if not is_gpu(keys):
        return sort_pairs(keys, torch.arange(n, dtype=torch.int32), key_bits)
    lib = _native.hip()
    vals = torch.empty_like(keys)
    ka = torch.empty_like(keys)
    va = torch.empty_like(keys)
    ws = torch.empty(lib.lsk_hip_sort_ws_bytes(n), dtype=torch.uint8, device=keys.device)
    alt = C.c_int(0)
    check(lib.lsk_hip_sort_keys_iota(_ptr(keys), _ptr(vals), _ptr(ka), _ptr(va), n, key_bits, _ptr(ws),
                                     C.byref(alt), _stream(keys)), "sort_keys_iota")
    return (ka, va) if alt.value else (keys, vals)


def sort_keys_iota_gather(keys: torch.Tensor, points: torch.Tensor, key_bits: int = 30, pad: int = 0):
    """sort_keys_iota + the points in sorted order (`pad` extra zero rows), gathered by the
    sort's last pass instead of a separate gather3 over the permutation. Returns (sorted
    keys, permutation, sorted points)."""
    n = keys.shape[0]
    if not is_gpu(keys) or n < 2:
        sk, perm = sort_keys_iota(keys, key_bits)
        return sk, perm, gather3(points, perm, pad=pad)
    lib = _native.hip()
    vals = torch.empty_like(keys)
    ka = torch.empty_like(keys)
    va = torch.empty_like(keys)
    ws = torch.empty(lib.lsk_hip_sort_ws_bytes(n), dtype=torch.uint8, device=keys.device)
    pts = torch.empty((n + pad, 3), dtype=torch.float32, device=keys.device)
    if pad:
        pts[n:].zero_()
    points = points.contiguous()
    alt = C.c_int(0)
    check(lib.lsk_hip_sort_keys_iota_gather(_ptr(keys), _ptr(vals), _ptr(ka), _ptr(va), n, key_bits, _ptr(ws),
                                            C.byref(alt), _ptr(points), _ptr(pts), _stream(keys)),
          "sort_keys_iota_gather")
    return ((ka, va) if alt.value else (keys, vals)) + (pts,)


def key_census(skeys: torch.Tensor, run: int) -> tuple[torch.Tensor, torch.Tensor]:
    """One device pass over sorted keys: (int64 [11] level counts as key_levels_dev, int32
    [1] heavy flag: some key equals the one `run` positions earlier). No host read."""
    cnt = torch.zeros(11, dtype=torch.int64, device=skeys.device)
    heavy = torch.zeros(1, dtype=torch.int32, device=skeys.device)
    check(_native.hip().lsk_hip_key_census(_ptr(skeys), skeys.shape[0], _ptr(cnt), int(run), _ptr(heavy),
                                           _stream(skeys)), "key_census")
    return cnt, heavy


def segment_bounds(p: torch.Tensor, seg: torch.Tensor, nseg: int):
    """Per-segment AABB of GPU points p [m,3] with contiguous segment ids seg (int32,
    non-decreasing runs) -> (lo, hi) [nseg, 3]."""
    lo = torch.empty((nseg, 3), dtype=torch.float32, device=p.device)
    hi = torch.empty((nseg, 3), dtype=torch.float32, device=p.device)
    check(_native.hip().lsk_hip_segment_bounds(_ptr(p.contiguous()), _ptr(seg.contiguous()), p.shape[0], nseg,
                                               _ptr(lo), _ptr(hi), _stream(p)), "segment_bounds")
    return lo, hi


def gather3(src: torch.Tensor, idx: torch.Tensor, pad: int = 0) -> torch.Tensor:
    """dst[i] = src[idx[i]] for float3 rows; dst gets `pad` extra zero rows."""
    n = idx.shape[0]
    dst = torch.empty((n + pad, 3), dtype=torch.float32, device=src.device)
    if pad:
        dst[n:].zero_()
    if is_gpu(src):
        check(_native.hip().lsk_hip_gather3(_ptr(src), _ptr(idx), n, _ptr(dst), _stream(src)), "gather3")
    else:
        dst[:n] = src[idx.to(torch.int64)]
    return dst


def scatter1(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, finalize: bool) -> torch.Tensor:
    """out[idx[i]] = f(src[i]) with f = sqrt-unless-inf when finalize."""
    n = src.shape[0]
    if is_gpu(src):
        check(_native.hip().lsk_hip_scatter1(_ptr(src), _ptr(idx), n, _ptr(out), int(finalize), _stream(src)),
              "scatter1")
    else:
        v = finalize_distances(src) if finalize else src
        out[idx.to(torch.int64)] = v
    return out


def finalize_distances(d2: torch.Tensor) -> torch.Tensor:
    """sqrt of the k-th squared distance unless it is +inf (reference extractFinalResult)."""
    if is_gpu(d2):
        out = torch.empty_like(d2)
        check(_native.hip().lsk_hip_finalize(_ptr(d2), d2.shape[0], _ptr(out), _stream(d2)), "finalize")
        return out
    # torch's float32 CPU sqrt is not correctly rounded (vectorised approximation);
    # sqrt in float64 then one rounding to float32 is (IEEE sqrtf, as on the GPU).
    return torch.where(torch.isinf(d2), d2, torch.sqrt(d2.double()).float())


# --------------------------------------------------------------------------- tree
def tree_depth(n: int) -> int:
    nb = (n + BUCKET - 1) // BUCKET
    d = 0
    while (1 << d) < nb:
        d += 1
    return d


def build_tree(sorted_pts: torch.Tensor, n: int) -> tuple[torch.Tensor, torch.Tensor, int]:
    """Bucket tree over the first n rows of sorted_pts -> (nodes [2^(D+1), 8],
    quarter boxes [2^D * 4, 8], depth)."""
    depth = tree_depth(n)
    slots = 1 << depth
    if is_gpu(sorted_pts):
        nodes = torch.empty((2 * slots, 8), dtype=torch.float32, device=sorted_pts.device)
        qnodes = torch.empty((4 * slots, 8), dtype=torch.float32, device=sorted_pts.device)
        check(_native.hip().lsk_hip_build_tree(_ptr(sorted_pts), n, _ptr(nodes), _ptr(qnodes),
                                               _stream(sorted_pts)), "build_tree")
        return nodes, qnodes, depth
    inf = float("inf")
    lo = torch.full((slots * BUCKET, 3), inf)
    hi = torch.full((slots * BUCKET, 3), -inf)
    lo[:n] = sorted_pts[:n]
    hi[:n] = sorted_pts[:n]
    qnodes = torch.zeros((4 * slots, 8), dtype=torch.float32)
    qnodes[:, 0:3] = lo.view(4 * slots, 16, 3).amin(dim=1)
    qnodes[:, 4:7] = hi.view(4 * slots, 16, 3).amax(dim=1)
    nodes = torch.zeros((2 * slots, 8), dtype=torch.float32)
    nodes[slots:, 0:3] = lo.view(slots, BUCKET, 3).amin(dim=1)
    nodes[slots:, 4:7] = hi.view(slots, BUCKET, 3).amax(dim=1)
    for level in range(depth - 1, -1, -1):
        a = 1 << level
        ch = nodes[2 * a: 4 * a].view(a, 2, 8)
        nodes[a:2 * a, 0:3] = torch.minimum(ch[:, 0, 0:3], ch[:, 1, 0:3])
        nodes[a:2 * a, 4:7] = torch.maximum(ch[:, 0, 4:7], ch[:, 1, 4:7])
        nodes[a:2 * a, 3] = torch.maximum(ch[:, 0, 3], ch[:, 1, 3])
    return nodes, qnodes, depth


def tree_set_radii(nodes: torch.Tensor, n: int, d2_sorted: torch.Tensor) -> torch.Tensor:
    """Store per-node max k-th squared radius (lo.w) of the queries below each node."""
    if is_gpu(nodes):
        check(_native.hip().lsk_hip_tree_set_radii(_ptr(nodes), n, _ptr(d2_sorted), _stream(nodes)),
              "tree_set_radii")
        return nodes
    depth = tree_depth(n)
    slots = 1 << depth
    r = torch.zeros(slots * BUCKET, dtype=torch.float32)
    r[:n] = d2_sorted[:n]
    nodes[slots:, 3] = r.view(slots, BUCKET).amax(dim=1)
    for level in range(depth - 1, -1, -1):
        a = 1 << level
        ch = nodes[2 * a: 4 * a].view(a, 2, 8)
        nodes[a:2 * a, 3] = torch.maximum(ch[:, 0, 3], ch[:, 1, 3])
    return nodes


# --------------------------------------------------------------------------- kNN
def radius_hint(box: torch.Tensor, n_total: int, k: int) -> torch.Tensor:
    """Device [1] float32: uniform-density k-th squared distance estimate of a GPU box."""
    out = torch.empty(1, dtype=torch.float32, device=box.device)
    check(_native.hip().lsk_hip_radius_hint(_ptr(box), int(n_total), int(k), _ptr(out), _stream(box)),
          "radius_hint")
    return out


ROWS_MAX_K = 65535  # 16-bit histogram bins of knn_rows; larger k go to the exact kernel
FAIL_CAP_OVERRIDE: int | None = None  # tests: force failure-list overflows (whole reruns)


def fail_capacity(work: int) -> int:
    """Capacity of the failure list of one knn_rows launch over `work` queries: all of
    them up to 64M, then 1/16 of them (a failure count above it makes the host rerun the
    whole query on the exact kernel, see knn_engine.query)."""
    if FAIL_CAP_OVERRIDE is not None:
        return max(1, min(work, FAIL_CAP_OVERRIDE))
    return max(1, min(work, max(1 << 26, work >> 4)))


class FailWord:
    """Always-on failure word of one k-NN launch: count (device int32) of the queries the
    16-bit kernel handed to the exact backstop, and the list capacity. Reading it syncs."""

    def __init__(self, count: torch.Tensor | None, cap: int):
        self.count = count
        self.cap = cap
        self._host = None
        self._ev = None
        self._gate = None
        self.flist = None

    def stage(self, gate: torch.Tensor | None = None) -> None:
        """Queue the word's copy to pinned host memory on the current stream (right behind
        the launch): a later value() waits for this launch only, not for work queued on
        the stream after it. `gate` (the device grid decision, int32 [1]) is staged with it
        (gate_value()): a .item() would wait for everything queued on the stream since."""
        if self.count is None or self.count.device.type != "cuda":
            return
        self._host = torch.empty(2, dtype=torch.int32, pin_memory=True)
        self._host[0:1].copy_(self.count.view(torch.int32), non_blocking=True)
        if gate is not None:
            self._host[1:2].copy_(gate.view(-1)[:1].to(torch.int32), non_blocking=True)
            self._gate = gate
        self._ev = torch.cuda.Event()
        self._ev.record()

    def gate_value(self, gate: torch.Tensor) -> int:
        """The staged grid decision (stage(gate)), else a direct read."""
        if self._gate is gate and self._ev is not None:
            self._ev.synchronize()
            return int(self._host[1])
        return int(gate.item())

    def value(self) -> int:
        # the kernels count in uint32 (a count >= 2^31 must not read as negative)
        if self.count is None:
            return 0
        if self._ev is not None:
            self._ev.synchronize()
            return int(self._host[0]) & 0xFFFFFFFF
        return int(self.count.item()) & 0xFFFFFFFF

    def overflowed(self) -> bool:
        return self.value() > self.cap


def knn_gpu(qpts: torch.Tensor, nq: int, trees: list, k: int, cut2: float,
            r_hint2: float | torch.Tensor,
            out_d2: torch.Tensor, groups: torch.Tensor | None = None, ngroups: int = 0,
            stats: torch.Tensor | None = None, qstatus: torch.Tensor | None = None,
            seed: int = 0, impl: str = "rows", init_d2: torch.Tensor | None = None,
            out_perm: torch.Tensor | None = None, out_final: torch.Tensor | None = None,
            debug_fail_mod: int = 0, grid=None, ngroups_dev: torch.Tensor | None = None,
            expect_grid: bool = True, short_list: bool = False, chunks: int = 1, grid2=None,
            qrot: torch.Tensor | None = None) -> FailWord:
    """k-th squared distance for sorted queries against up to two bucket trees.

    trees: list of (sorted_pts_padded, nodes, qnodes, n, depth). impl: "rows" (the
    production kernel: 4 x 16-query rows, 16-bit LDS histograms; every query it cannot
    resolve exactly goes to the failure list and is recomputed by the exact kernel in the
    same stream, no host round trip) or "exact" (the wave-per-query 32-bit backstop for
    every query; also used for k > 65535). seed > 0 declares that the queries are
    trees[0]'s points in tree order (pass 1 starts from neighbour buckets).
    init_d2 (optional, [nq]): a known upper bound of every query's k-th squared distance
    (e.g. the local result before a halo re-query) that places the first range.
    out_perm / out_final (optional, fused scatter): the kernels also write
    out_final[out_perm[q]] = final distance; out_d2 may then be None.
    debug_fail_mod (tests): the rows kernel also fails every query q with q % mod == 0.
    ngroups_dev (optional, with groups): int32 [1] on the device, the list's length
    (ngroups is then only the launch's upper bound).
    expect_grid (with a gate): which kernel the gate is expected to pick — that one gets the
    full launch, the other its persistent strided form (a small grid whose waves return at
    once when the gate rejects it; a misprediction costs speed, never exactness).
    short_list (with ngroups_dev): the device-side list is expected far shorter than
    ngroups (a rank's boundary groups): the kernel that runs takes its persistent strided
    form at full occupancy instead of one wave per possible group (most would be
    dispatched only to return: ~16 ms per 1M-block launch).
    chunks > 1: the pass goes out as that many launches over consecutive wave ranges —
    kernel boundaries at which the high-priority streams' kernels (the next set's
    redistribution, the halo exchange) get CU slots: a running k-NN grid keeps every slot
    until its last workgroup is dispatched.
    grid (impl "grid"): (slots, level, box, inf4[, gate]) of knn_engine.GridIndex — the
    cell-grid candidate source of knn_grid.hip for one tree whose points are the queries
    (same failure list and backstop as "rows"); with a device gate (int32 [1]) the grid
    kernel runs iff gate == 1 and knn_rows iff gate == 0.
    grid2 (impl "grid", two trees: the halo re-query): the second tree's grid (slots, level,
    box, inf4) — knn_grid2 walks both grids; init_d2 is allowed then.
    qrot (one tree, rows / exact): the queries in the rotated frame trees[0]'s boxes were
    built in (knn_engine.flat_frame); box tests use it, distances qpts.
    Returns the launch's FailWord.
    """
    if (out_perm is None) != (out_final is None):
        raise ValueError("knn_gpu: out_perm and out_final go together")
    if out_perm is not None and (out_perm.shape[0] < nq or out_perm.dtype != torch.int32
                                 or not out_perm.is_contiguous() or out_final.dtype != torch.float32):
        raise ValueError("knn_gpu: out_perm must be int32 [>= nq], out_final float32")
    if impl not in ("rows", "exact", "grid"):
        raise ValueError(f"knn_gpu: impl must be rows, exact or grid, not {impl!r}")
    if impl == "grid" and (grid is None or len(trees) != (2 if grid2 is not None else 1)
                           or (grid2 is None and init_d2 is not None)):
        raise ValueError("knn_gpu: impl grid needs a grid and one tree (no init_d2), or two trees and grid2")
    a = KnnArgs()
    a.qpts = _ptr(qpts)
    a.nq = nq
    a.groups = _ptr(groups)
    a.ngroups = ngroups
    a.ngroups_dev = _ptr(ngroups_dev) if groups is not None else None
    for i, (pts, nodes, qnodes, n, depth) in enumerate(trees):
        a.tree[i] = TreeView(_ptr(pts), _ptr(nodes), _ptr(qnodes), n, depth, 0)
    a.ntrees = len(trees)
    a.k = k
    a.cut2 = cut2
    if isinstance(r_hint2, torch.Tensor):
        # device value (K.radius_hint): parked in the unused node 0 of tree 0, which the
        # kernel reads when r_hint2 < 0 — no host round trip, no extra kernel argument
        trees[0][1].view(-1)[3:4].copy_(r_hint2.view(-1)[:1])
        a.r_hint2 = -1.0
    else:
        a.r_hint2 = max(float(r_hint2), 0.0)
    a.out_d2 = _ptr(out_d2)
    a.stats = _ptr(stats)
    a.qstatus = _ptr(qstatus)
    a.seed = seed
    a.init_d2 = _ptr(init_d2)
    if qrot is not None and (impl == "grid" or len(trees) != 1):
        raise ValueError("knn_gpu: qrot needs one tree and the rows / exact kernel")
    a.qrot = _ptr(qrot)
    a.out_perm = _ptr(out_perm)
    a.out_final = _ptr(out_final)
    a.debug_fail_mod = int(debug_fail_mod)
    lib = _native.hip()
    st = _stream(qpts)
    if impl == "exact" or k > ROWS_MAX_K:
        check(lib.lsk_hip_knn_exact(C.byref(a), None, None, 0, st), "knn_exact")
        return FailWord(None, 0)
    work = ngroups * BUCKET if groups is not None else nq
    cap = fail_capacity(work)
    count = torch.zeros(1, dtype=torch.int32, device=qpts.device)
    flist = torch.empty(cap, dtype=torch.int32, device=qpts.device)
    a.fail_list = _ptr(flist)
    a.fail_count = _ptr(count)
    a.fail_cap = cap
    full = 2 if short_list and groups is not None and ngroups_dev is not None else 0
    # a short device-counted list runs persistent waves that take their groups from a work
    # queue (one zeroed counter per launch): re-query groups differ widely in cost, and a
    # static stride left the halo re-query at 9.1 vs 6.9 ms with the exact-size launch
    # (1B / 8 ranks, scripts/rank_replay.py)
    wqs = torch.zeros(2 * max(1, int(chunks)), dtype=torch.int32, device=qpts.device) if full else None
    nw = ngroups if groups is not None else (nq + BUCKET - 1) // BUCKET
    chunks = max(1, min(int(chunks), nw))
    # the pass as `chunks` consecutive launches over wave ranges (0 = to the end)
    spans = [(0, 0)] if chunks == 1 else [(nw * c // chunks, nw * (c + 1) // chunks) for c in range(chunks)]
    def _wq(i: int, on: bool):
        a.wq = _ptr(wqs[i:i + 1]) if on and wqs is not None else None

    if impl == "grid":
        slots, level, gbox, inf4 = grid[:4]
        gate = grid[4] if len(grid) > 4 else None
        gv = GridView(_ptr(slots), None, _ptr(gbox), _ptr(inf4), int(level), 0)
        gv2 = GridView(_ptr(grid2[0]), None, _ptr(grid2[2]), _ptr(grid2[3]), int(grid2[1]), 0) if grid2 is not None else None
        for ci, (a.wave_base, a.wave_end) in enumerate(spans):
            if gate is not None:
                # the device decides (lsk_hip_grid_decide): both kernels are queued, the one
                # not chosen returns at its first instruction (no host read, graph-capturable)
                a.gate = _ptr(gate)
                a.gate_on = 1
                a.pad2 = full if expect_grid else 1
            else:
                a.pad2 = full
            _wq(2 * ci, a.pad2 == 2)
            if gv2 is not None:
                check(lib.lsk_hip_knn_grid2(C.byref(a), C.byref(gv), C.byref(gv2), st), "knn_grid2")
            else:
                check(lib.lsk_hip_knn_grid(C.byref(a), C.byref(gv), st), "knn_grid")
            if gate is not None:
                a.gate_on = 0
                a.pad2 = 1 if expect_grid else full
                _wq(2 * ci + 1, a.pad2 == 2)
                check(lib.lsk_hip_knn_rows(C.byref(a), st), "knn_rows")
            a.gate = None
            a.pad2 = 0
    else:
        for ci, (a.wave_base, a.wave_end) in enumerate(spans):
            a.pad2 = full
            _wq(ci, a.pad2 == 2)
            check(lib.lsk_hip_knn_rows(C.byref(a), st), "knn_rows")
            a.pad2 = 0
    a.wave_base = a.wave_end = 0
    a.wq = None
    # exact backstop over the failure list (device-side count: empty list = short no-op)
    check(lib.lsk_hip_knn_exact(C.byref(a), _ptr(flist), _ptr(count), cap, st), "knn_exact")
    fw = FailWord(count, cap)
    fw.flist = flist  # (debugging: the failed queries' positions, flist[:count])
    return fw


# --------------------------------------------------------------------------- cell grid
def key_levels(skeys: torch.Tensor) -> list[int]:
    """Distinct cells of each octree level 0..10 among sorted 30-bit curve keys (one
    device pass + one 88-byte read): [1, d1, ..., d10]."""
    n = skeys.shape[0]
    if n == 0:
        return [0] * 11
    cnt = torch.empty(11, dtype=torch.int64, device=skeys.device)
    check(_native.hip().lsk_hip_key_levels(_ptr(skeys), n, _ptr(cnt), _stream(skeys)), "key_levels")
    c = cnt.cpu().tolist()
    return [1] + [int(c[l]) + 1 for l in range(1, 11)]


def grid_build(sorted_pts: torch.Tensor, sorted_keys: torch.Tensor, n: int, box: torch.Tensor, level: int):
    """Grandchild runs of the octree grid over the curve-sorted points (knn_grid.hip): every
    level-`level` cell has 64 slots (its level+2 grandchildren in curve order), each
    (start, end, packed coords, 0) -> int32 [8^level * 64, 4]."""
    dev = sorted_pts.device
    slots = torch.empty((64 << (3 * level), 4), dtype=torch.int32, device=dev)
    check(_native.hip().lsk_hip_grid_build(_ptr(sorted_pts), _ptr(sorted_keys), n, _ptr(box), level, _ptr(slots),
                                           _stream(sorted_pts)), "grid_build")
    return slots


def key_levels_dev(skeys: torch.Tensor) -> torch.Tensor:
    """key_levels without the host read: int64 [11] on the device, counts[l] = distinct
    level-l cells - 1 (the raw lsk_hip_key_levels output)."""
    cnt = torch.zeros(11, dtype=torch.int64, device=skeys.device)
    if skeys.shape[0] > 0:
        check(_native.hip().lsk_hip_key_levels(_ptr(skeys), skeys.shape[0], _ptr(cnt), _stream(skeys)),
              "key_levels")
    return cnt


def grid_sq_dev(slots: torch.Tensor) -> torch.Tensor:
    """grid_sq without the host read: int64 [1] on the device."""
    out = torch.zeros(1, dtype=torch.int64, device=slots.device)
    check(_native.hip().lsk_hip_grid_sq(_ptr(slots), slots.shape[0], _ptr(out), _stream(slots)), "grid_sq")
    return out


def grid_decide(counts: torch.Tensor, sq: torch.Tensor, n: int, g: int, crowd: float, check_uniform: bool):
    """Device flag int32 [1]: 1 iff the grid applies (lsk_hip_grid_decide), no host read."""
    gate = torch.empty(1, dtype=torch.int32, device=counts.device)
    check(_native.hip().lsk_hip_grid_decide(_ptr(counts), _ptr(sq), n, g, C.c_float(crowd), int(check_uniform),
                                            _ptr(gate), _stream(counts)), "grid_decide")
    return gate


def grid_sq(slots: torch.Tensor) -> int:
    """Sum over grid slots of population^2 (host read)."""
    out = torch.zeros(1, dtype=torch.int64, device=slots.device)
    check(_native.hip().lsk_hip_grid_sq(_ptr(slots), slots.shape[0], _ptr(out), _stream(slots)), "grid_sq")
    return int(out.item())


def kth_cpu(points: torch.Tensor, queries: torch.Tensor, k: int, cut2: float, method: str = "kdtree") -> torch.Tensor:
    """CPU oracle: k-th squared distance of each query among points (self counted if present)."""
    pts = points.contiguous().float()
    q = queries.contiguous().float()
    out = torch.empty(q.shape[0], dtype=torch.float32)
    f = _native.host().lsk_cpu_kth_kdtree if method == "kdtree" else _native.host().lsk_cpu_kth_brute
    f(_ptr(pts), pts.shape[0], _ptr(q), q.shape[0], int(k), C.c_float(cut2), _ptr(out), _nthreads())
    return out


# --------------------------------------------------------------------------- halo
UB_MAX_W = 8  # tree.hip kUbMaxW: beyond it the box-pair bound


def tree_set_radii_ub(nodes: torch.Tensor, pts: torch.Tensor, n: int, k: int) -> torch.Tensor:
    """Per-node upper bound of the k-th squared radius before any query ran (tree.hip
    leaf_radius_ub_kernel): the ceil(k/64)+1 buckets around a leaf hold >= k points;
    with m(p) = farthest-corner distance from window point p to the leaf box, the k-th
    smallest m(p) bounds every leaf query's k-th neighbour distance (beyond UB_MAX_W
    buckets: the farthest corner pair of the leaf box and the window's union box).
    `pts`: the index's sorted points."""
    if is_gpu(nodes):
        check(_native.hip().lsk_hip_tree_set_radii_ub(_ptr(nodes), _ptr(pts), n, k, _stream(nodes)),
              "tree_set_radii_ub")
        return nodes
    depth = tree_depth(n)
    slots = 1 << depth
    nb = (n + BUCKET - 1) // BUCKET
    r = torch.zeros(slots, dtype=torch.float32)
    if nb and n < k:
        r[:nb] = math.inf
    elif nb:
        w = min(nb, (k + BUCKET - 1) // BUCKET + 1)
        leaf = torch.arange(nb)
        st = (leaf - (w - 1) // 2).clamp(0, nb - w)
        lo = nodes[slots:slots + nb, 0:3]
        hi = nodes[slots:slots + nb, 4:7]
        if w <= UB_MAX_W:
            idx = (st[:, None] * BUCKET + torch.arange(w * BUCKET)[None, :])   # [nb, 64w]
            valid = idx < n
            p = pts[:n][idx.clamp(max=n - 1)]                                   # [nb, 64w, 3]
            e = torch.maximum(p - lo[:, None, :], hi[:, None, :] - p)
            m = torch.addcmul(torch.addcmul(e[..., 0] * e[..., 0], e[..., 1], e[..., 1]), e[..., 2], e[..., 2])
            m = torch.where(valid, m, torch.full_like(m, math.inf))
            d2 = m.kthvalue(k, dim=1).values
        else:
            win = st[:, None] + torch.arange(w)[None, :]
            wlo = lo[win].amin(dim=1)
            whi = hi[win].amax(dim=1)
            e = torch.maximum(whi - lo, hi - wlo)
            d2 = torch.addcmul(torch.addcmul(e[:, 0] * e[:, 0], e[:, 1], e[:, 1]), e[:, 2], e[:, 2])
        r[:nb] = d2 * (1.0 + 2.0 ** -16)
    nodes[slots:, 3] = r
    for level in range(depth - 1, -1, -1):
        a = 1 << level
        ch = nodes[2 * a: 4 * a].view(a, 2, 8)
        nodes[a:2 * a, 3] = torch.maximum(ch[:, 0, 3], ch[:, 1, 3])
    return nodes


def boundary_groups(local_nodes: torch.Tensor, depth: int, ngroups: int, pub: torch.Tensor, pub_off: list[int],
                    pub_depth, self_rank: int) -> torch.Tensor:
    """int32 [ngroups]: 1 for the local query groups (buckets) whose leaf box, inflated by
    its squared radius bound (lo.w of local_nodes), comes closer than that bound to some
    node of another rank's published tree (halo.hip boundary_groups_kernel); 0 = the
    group's k nearest are all local, whatever the other ranks hold."""
    nranks = len(pub_off)
    flags = torch.zeros(max(ngroups, 0), dtype=torch.int32, device=local_nodes.device)
    if ngroups <= 0:
        return flags
    if is_gpu(local_nodes):
        off = torch.tensor(pub_off, dtype=torch.int64, device=local_nodes.device)
        dep = (pub_depth.to(device=local_nodes.device, dtype=torch.int32).contiguous()
               if isinstance(pub_depth, torch.Tensor)
               else torch.tensor(pub_depth, dtype=torch.int32, device=local_nodes.device))
        check(_native.hip().lsk_hip_boundary_groups(_ptr(local_nodes), int(depth), int(ngroups), _ptr(pub),
                                                    _ptr(off), _ptr(dep), nranks, self_rank, _ptr(flags),
                                                    _stream(local_nodes)), "boundary_groups")
        return flags
    # CPU: every group against the leaf level of each published tree, in float64 with the
    # squared gap shrunk by 2^-20 (a rounding of the canonical float d² cannot hide a
    # neighbour: the test only errs towards "boundary")
    if isinstance(pub_depth, torch.Tensor):
        pub_depth = [int(x) for x in pub_depth.cpu().tolist()]
    pub = pub.reshape(-1, 8)
    leaves = local_nodes[(1 << depth):(1 << depth) + ngroups].double()
    lo, hi, r2 = leaves[:, None, 0:3], leaves[:, None, 4:7], leaves[:, 3]
    hit = torch.zeros(ngroups, dtype=torch.bool)
    for j in range(nranks):
        if j == self_rank:
            continue
        d = pub_depth[j]
        base = pub_off[j] // 8
        nb = pub[base + (1 << d): base + (2 << d)].double()
        for s0 in range(0, ngroups, 4096):
            gap = torch.clamp(torch.maximum(lo[s0:s0 + 4096] - nb[None, :, 4:7], nb[None, :, 0:3] - hi[s0:s0 + 4096]),
                              min=0.0)
            g2 = (gap * gap).sum(-1) * (1.0 - 2.0 ** -20)
            hit[s0:s0 + 4096] |= (g2 < r2[s0:s0 + 4096, None]).any(1)
    flags[hit] = 1
    return flags


def compact_flags(flags: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """(list of the indices i with flags[i] != 0, their count as an int32 [1] tensor on the
    flags' device: no host read on the GPU)."""
    n = flags.shape[0]
    if is_gpu(flags):
        lst = torch.empty(max(n, 1), dtype=torch.int32, device=flags.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=flags.device)
        if n:
            check(_native.hip().lsk_hip_compact_flags(_ptr(flags), n, _ptr(lst), _ptr(cnt), _stream(flags)),
                  "compact_flags")
        return lst, cnt
    idx = torch.nonzero(flags != 0).view(-1).to(torch.int32)
    return idx, torch.tensor([idx.shape[0]], dtype=torch.int32)


def halo_mask(pts: torch.Tensor, pub: torch.Tensor, pub_off: list[int], pub_depth, self_rank: int) -> torch.Tensor:
    """Per point bitmask of ranks whose published radius-inflated boxes contain it.
    pub_depth: published tree depth per rank (list, or an int32 tensor — a device tensor
    keeps the GPU path free of a host read)."""
    n = pts.shape[0]
    nranks = len(pub_off)
    mask = torch.empty(n, dtype=torch.int64, device=pts.device)
    if isinstance(pub_depth, torch.Tensor) and not (is_gpu(pts) and pub_depth.device == pts.device):
        pub_depth = [int(x) for x in pub_depth.cpu().tolist()]
    if is_gpu(pts):
        off = torch.tensor(pub_off, dtype=torch.int64, device=pts.device)
        dep = (pub_depth.to(torch.int32).contiguous() if isinstance(pub_depth, torch.Tensor)
               else torch.tensor(pub_depth, dtype=torch.int32, device=pts.device))
        check(_native.hip().lsk_hip_halo_mask(_ptr(pts), n, _ptr(pub), _ptr(off), _ptr(dep), nranks,
                                              self_rank, _ptr(mask), _stream(pts)), "halo_mask")
        return mask
    # CPU: test against the leaf level of each published tree
    boxes, offs = [], [0]
    pub = pub.reshape(-1, 8)
    for j in range(nranks):
        d = pub_depth[j]
        base = pub_off[j] // 8
        leaves = pub[base + (1 << d): base + (2 << d)]
        boxes.append(leaves)
        offs.append(offs[-1] + leaves.shape[0])
    allb = torch.cat(boxes).contiguous() if boxes else torch.zeros((0, 8))
    offs_t = torch.tensor(offs, dtype=torch.int64)
    _native.host().lsk_cpu_halo_mask(_ptr(pts.contiguous()), n, _ptr(allb), _ptr(offs_t), nranks, self_rank,
                                     _ptr(mask), _nthreads())
    return mask
