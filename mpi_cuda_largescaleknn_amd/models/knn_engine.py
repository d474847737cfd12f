"""Single-rank k-th-nearest-neighbour distance engine.

The "model" of this framework is the reference's per-rank work (SURVEY §1, L2+L4):
build a k-d tree over the rank's points (cukd::buildTree, unorderedDataVariant.cu:161)
and answer one k-NN query per point (runQuery/extractFinalResult, :75-103). Pipeline
on the GPU — every step a hand-written gfx950 kernel on torch's current stream:

    bounds -> Hilbert keys -> LSD radix sort -> gather -> bucket tree (+ cell grid) -> radix-select k-NN

``LocalIndex`` is the reusable product of the first five steps (also used for the
halo tree in the distributed pipelines).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import NamedTuple

import numpy as np
import torch

from ..ops import kernels as K


def cut2_of(max_radius: float) -> float:
    """The reference stores maxRadius as float and compares squared distances against
    cutOff*cutOff evaluated in float (FlexHeapCandidateList init, U:84-85)."""
    r = np.float32(max_radius)
    with np.errstate(over="ignore"):
        return float(r * r)


SEED_BUCKETS = 1  # curve-neighbour buckets (each side) that seed the first pass (1e8 k=100: 0/1/2 -> 0.126/0.125/0.126 s)
KNN_IMPL = "rows"  # "rows" (production kernel + exact backstop) or "exact" (backstop only)
DEBUG_FAIL_MOD = 0  # tests: make the rows kernel hand every m-th query to the backstop
# HIP-graph captures: the failure words of captured launches, checked after a replay
# (verify_captured_failures) — during a capture the host cannot read them. A replay
# re-zeroes each launch's counter, so every captured launch also folds its count into a
# peak slot of CAPTURE_PEAKS (allocated and zeroed by prepare_capture, outside the graph):
# the check then covers every replay, not only the last one.
CAPTURED_FAIL_WORDS: list = []
CAPTURE_PEAKS: torch.Tensor | None = None


def prepare_capture(device: torch.device, slots: int = 64) -> None:
    """Call before capturing k-NN launches into a graph (see CAPTURED_FAIL_WORDS)."""
    global CAPTURE_PEAKS
    CAPTURE_PEAKS = torch.zeros(slots, dtype=torch.int64, device=device)


@dataclass
class KnnConfig:
    k: int
    max_radius: float = math.inf
    publish_levels: int = 15       # top tree levels published for halo filtering (~1K pts/box)
    collect_stats: bool = False

    @property
    def cut2(self) -> float:
        return cut2_of(self.max_radius)


# Cell-grid candidate source of the local k-NN pass (knn_grid.hip): "auto" = built for
# GPU indexes whose sub-cell populations look near-uniform (GRID_CROWD), "on" = always,
# "off" = never (the bucket-tree kernel knn_rows serves every query).
GRID = os.environ.get("LSKNN_GRID", "auto")
GRID_MS = float(os.environ.get("LSKNN_GRID_MS", "6"))  # target mean points per finest cell
# auto: a point's sub-cell holds on average at most this many times the mean (+1)
GRID_CROWD = float(os.environ.get("LSKNN_GRID_CROWD", "2"))
# Which kernel the device gate is expected to pick (the last decision read on the host):
# that one gets the full launch, the other a small persistent one (kernels.knn_gpu).
GRID_EXPECT = [True]


@dataclass
class GridIndex:
    slots: torch.Tensor      # int32 [8^level * 64, 4]: per level-`level` cell, its 64
                             # grandchildren's runs of the sorted array in curve order
    level: int               # cell level (grandchildren at level + 2)
    box: torch.Tensor        # the cube of the sort keys (device)
    inf4: torch.Tensor | None = None  # 4 x +inf on the device (candidate padding)
    gate: torch.Tensor | None = None  # device int32 [1]: 1 = the grid applies (decided on
                                      # the device, GRID=auto), None = always (GRID=on)
    census: tuple | None = None       # (level counts, crowding sum) the gate came from

    def view(self) -> tuple:
        if self.inf4 is None:
            self.inf4 = torch.full((4,), math.inf, dtype=torch.float32, device=self.slots.device)
        return (self.slots, self.level, self.box, self.inf4, self.gate)

    def decision(self) -> dict:
        """Host read of what the device decided from (debugging / reporting)."""
        out = {"level": self.level + 2, "applies": self.applies()}
        if self.census is not None:
            c = [int(x) for x in self.census[0].cpu().tolist()]
            out.update(distinct_g=c[self.level + 2] + 1, distinct_g1=c[self.level + 1] + 1,
                       crowd_sum=int(self.census[1].item()))
        return out

    def applies(self) -> bool:
        """Host read of the device decision (reporting only; never on the hot path)."""
        return self.gate is None or bool(int(self.gate.item()))


@dataclass
class LocalIndex:
    n: int
    pts: torch.Tensor        # [n + PAD, 3] curve-sorted (Hilbert) points (padded)
    perm: torch.Tensor       # int32 [n]: sorted position -> row of the input array
    nodes: torch.Tensor      # [2^(depth+1), 8] bucket-tree node boxes (lo.w = radius²)
    qnodes: torch.Tensor     # [2^depth * 4, 8] boxes of each bucket's four 16-point quarters
    depth: int
    box: torch.Tensor        # [8] cube used for the curve keys
    grid: GridIndex | None = None
    qrot: torch.Tensor | None = None  # [n + PAD, 3]: the sorted points in the rotated frame the
                                      # keys, tree boxes and box tests use (flat_frame), or None

    @property
    def device(self) -> torch.device:
        return self.pts.device

    def tree(self) -> tuple:
        return (self.pts, self.nodes, self.qnodes, self.n, self.depth)


@dataclass
class KnnStats:
    counters: dict = field(default_factory=dict)

    def add(self, raw: torch.Tensor) -> None:
        names = ["evals", "leaves", "nodes", "hist_passes", "overflow_lanes", "underflow_lanes",
                 "refine_lanes", "mismatch_lanes", "pass_limit_waves", "list_invalid_waves", "waves",
                 "hint_lanes", "recorded_leaves", "collect_steps", "collect_nodes", "guard_trips",
                 # cycle profile (LSK_PROFILE kernel builds only)
                 "prof_proc_hist", "prof_proc_collect", "prof_walk_hist", "prof_walk_collect",
                 "prof_quarters", "prof_inner_nodes", "prof_select", "prof_wave",
                 "prof_rows_entry", "prof_rows_in", "failed_lanes", "binovf_lanes",
                 "prof_dead_slots", "prof_slots", "prof_crows_entry", "prof_crows_in"]
        vals = raw.cpu().tolist()
        for i, nm in enumerate(names):
            self.counters[nm] = self.counters.get(nm, 0) + int(vals[i])

    def add_fallback(self, n: int) -> None:
        self.counters["fallback_queries"] = self.counters.get("fallback_queries", 0) + int(n)


# The point gather fused into the key sort's last pass (kernels.sort_keys_iota_gather)
# instead of a gather3 pass over the permutation: 1B build 74.9 vs 71.9 ms,
# bench neutral (profiles/r6_sort/), so off by default.
FUSED_GATHER = os.environ.get("LSKNN_FUSED_GATHER", "0") == "1"


# Flat data in any orientation (a tilted plane, a slanted line): the bucket tree's axis-
# aligned boxes around a slanted patch are as thick as they are wide, so they cull like 3-D
# boxes around 2-D data (2e7 points, k = 100: tilted plane 649.6 vs axis-aligned plane
# 1239.0 Mpts/s). flat_frame finds the principal axes of such a set; build_index then sorts
# and boxes the points in that frame (keys, tree boxes, box tests) while every distance stays
# canonical in the points' own coordinates, so outputs are bit-identical. The boxes are
# widened by a bound on the rotation's rounding (rotate_margin): culling stays conservative.
# 0: off (A/B).
FLAT_FRAME = os.environ.get("LSKNN_FLAT_FRAME", "1") != "0"
FLAT_RATIO = 1e-6        # smallest / largest principal variance of a flat set
FRAME_SAMPLE = 1 << 13   # points sampled for the covariance (strided)
# The frame pays from k ~ 48 (2e7 tilted plane, k = 100: 647 -> 1012 Mpts/s; k = 16: 1485 ->
# 1366, the rotated build's extra passes outweigh its cheaper walk); the probe is then read
# before the build (FRAME_EARLY: non-flat data pay a ~1 % host wait; read after the build
# instead, a plane pays a wasted build: 911 vs 1012). profiles/r6_nonuniform/flat_frame_ab.txt
FRAME_MIN_K = int(os.environ.get("LSKNN_FRAME_MIN_K", "48"))
FRAME_EARLY = os.environ.get("LSKNN_FRAME_EARLY", "1") == "1"
# ... and only while the plane's k-NN radius (sqrt(k * area / (pi * n))) is >= FRAME_RADIUS_X
# times the boxes' widening (rotate_margin); measured wins down to a ratio of ~4 (5e8, k = 48).
FRAME_RADIUS_X = float(os.environ.get("LSKNN_FRAME_RADIUS_X", "2"))
# Curve keys in the plane's frame: above PLANE_2D_MIN points, 2-D Morton keys of the two
# in-plane coordinates, 15 bits each — 3-D keys spend a third of their 30 bits on the flat
# axis: 1024^2 cells, ~200 points each at 2e8, wider than the k-NN radius (tilted plane,
# k = 100, 3-D -> 2-D keys: 2e8 379 -> 878, 5e8 167 -> 856 Mpts/s; at 2e7 the 3-D Hilbert
# keys' locality wins, 987 vs 880; profiles/r6_nonuniform/plane_frame_scale.txt). Above it,
# axis-aligned planes take the frame too for the same keys, and every k does (2e8, frame vs
# own: tilted 875 / 1227 vs 630 / 912 at k = 100 / 16, axis-aligned 884 / 1248 vs 649 / 897).
# LSKNN_PLANE_KEYS: auto | 2d | 3d.
PLANE_KEYS = os.environ.get("LSKNN_PLANE_KEYS", "auto")
PLANE_2D_MIN = 1 << 26


# A line (two principal variances negligible) keeps its own frame (rotated fp32 coordinates
# cannot resolve a dense line: profiles/r6_nonuniform/line_frame_ab.txt) but is sorted by its
# position along the axis (line_keys) instead of 3-D curve keys. LSKNN_LINE_KEYS=0: off.
LINE_KEYS = os.environ.get("LSKNN_LINE_KEYS", "1") != "0"


class LineAxis(NamedTuple):
    """FrameProbe's verdict for a line: its unit direction (float32 [3], device)."""
    a: torch.Tensor


def line_keys(points: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
    """30-bit keys of points by their projection on the direction a (float32 arithmetic:
    ~24 significant bits; ties in any order)."""
    t = points[:, 0] * a[0] + points[:, 1] * a[1] + points[:, 2] * a[2]
    lo, hi = t.min(), t.max()
    t = (t - lo) * (float(1 << 30) / (hi - lo).clamp_min(1e-30))
    return t.clamp_(0.0, float((1 << 30) - 64)).to(torch.int32)


def _plane_2d(n: int) -> bool:
    return PLANE_KEYS == "2d" or (PLANE_KEYS == "auto" and n > PLANE_2D_MIN)


class FrameProbe:
    """The flatness test of flat_frame: a strided sample's 3x3 covariance is computed on
    the device (float64 sums); result() reads it (one small host read) and returns the
    rotation, or None."""

    def __init__(self, points: torch.Tensor, k: int = FRAME_MIN_K):
        self.cov = None
        self.k = k
        n = points.shape[0]
        if not FLAT_FRAME or (k < FRAME_MIN_K and not _plane_2d(n) and not LINE_KEYS) or not K.is_gpu(points) or n < 1024 \
                or _SYNC_FREE[0] \
                or torch.cuda.is_current_stream_capturing():
            return
        smp = points[::max(1, n // FRAME_SAMPLE)][:FRAME_SAMPLE].to(torch.float64)
        self.n, self.m = n, smp.shape[0]
        c = smp - smp.mean(0)
        # (read by result() with one small blocking copy: the probe is read before the build
        # anyway, FRAME_EARLY, so a pinned buffer + event saved nothing)
        self.cov = torch.stack([(c[:, i] * c[:, j]).sum() for i, j in ((0, 0), (0, 1), (0, 2), (1, 1), (1, 2),
                                                                         (2, 2))] + [smp.abs().max()])
        self.device = points.device

    def result(self) -> torch.Tensor | None:
        if self.cov is None:
            return None
        a = self.cov.cpu().numpy()
        cov = np.array([[a[0], a[1], a[2]], [a[1], a[3], a[4]], [a[2], a[4], a[5]]])
        if not np.isfinite(cov).all():
            return None
        w, v = np.linalg.eigh(cov)  # ascending
        if not (w[2] > 0) or w[0] > FLAT_RATIO * w[2]:
            return None
        if w[1] <= FLAT_RATIO * w[2]:  # a line: sorted along its axis, in its own frame
            return LineAxis(torch.tensor(v[:, 2].copy(), dtype=torch.float32, device=self.device)) \
                if LINE_KEYS else None
        # a plane: one principal variance negligible, the other two not
        if w[1] < 1e-3 * w[2] or (self.k < FRAME_MIN_K and not _plane_2d(self.n)):
            return None
        if np.max(np.abs(v[:, 0])) > 1.0 - 1e-6 and not _plane_2d(self.n):
            return None  # already axis-aligned: the tree is thin as is (3-D keys either way)
        # the k-NN radius against rotate_margin (extents of a uniform spread: sqrt(12 var))
        e1, e2 = math.sqrt(12.0 * w[1] / self.m), math.sqrt(12.0 * w[2] / self.m)
        radius = math.sqrt(self.k * e1 * e2 / (math.pi * max(self.n, 1)))
        if radius < FRAME_RADIUS_X * (a[6] * 1.7320508 + e2) * 2.0 ** -16:
            return None
        R = v[:, ::-1].T.copy()  # rows: axes by decreasing variance
        return torch.tensor(R, dtype=torch.float32, device=self.device)


def flat_frame(points: torch.Tensor) -> torch.Tensor | None:
    """3x3 float32 rotation (rows: principal axes, largest variance first) when `points`
    (GPU) lie on a plane that is not already aligned with the coordinate axes, else None
    (FrameProbe, read at once; eager paths only: never inside a HIP-graph capture or a
    stream of sets)."""
    return FrameProbe(points).result()


def rotate(points: torch.Tensor, R: torch.Tensor) -> torch.Tensor:
    """points @ R^T with explicit fp32 multiply-adds (no reduced-precision GEMM path)."""
    p0, p1, p2 = points[:, 0:1], points[:, 1:2], points[:, 2:3]
    return p0 * R[:, 0] + p1 * R[:, 1] + p2 * R[:, 2]


def rotate_margin(rbox: torch.Tensor) -> torch.Tensor:
    """Per-side widening of every box built from rotated points (device scalar): bounds the
    difference between distances in the rotated frame (float-evaluated, non-orthonormal
    float matrix) and the canonical float distances in the points' own frame — ~9 ulp of the
    largest coordinate for the rotation, a few ulp of the extent for the distances — with a
    wide safety factor (2^-16 of |coordinate| + extent)."""
    mag = torch.maximum(rbox[0:3].abs(), rbox[3:6].abs()).max()
    ext = (rbox[3:6] - rbox[0:3]).max()
    return (mag * 1.7320508 + ext) * (2.0 ** -16)


def build_index(points: torch.Tensor, box: torch.Tensor | None = None,
                keys: tuple | None = None, grid: bool = False, density_n: int | None = None,
                grid_level: int | None = None, grid_gated: bool = True,
                frame: torch.Tensor | None = None) -> LocalIndex:
    """Sort points along the space-filling curve of `box` (default: their own bounds) and
    build the bucket tree. `keys` = (keys, iota) computed already (SetStream's PRE_KEYS:
    the next set's box and curve keys on the side stream beside the current k-NN). `grid`: also index the sorted points by the cell grid of
    the fast local k-NN pass (build_grid, GPU). `density_n`: the number of points that
    fill `box` (a rank's share of a global box: the global count; default: n).
    `grid_level`: force the grid's grandchild level (tests; a halo index takes the local
    grid's); `grid_gated=False`: no census / device gate for the grid (build_grid).
    `frame` (flat_frame, GPU, with no keys or box given): the index is built in that rotated
    frame (no grid) — see FLAT_FRAME.
    No host read on the way unless an over-full key cell needs the eager refinement
    (refine_heavy_cells; under host_sync_free() not even that)."""
    points = points.contiguous()
    n = points.shape[0]
    if isinstance(frame, LineAxis):  # a line: its own frame, keys along its axis, no grid
        if keys is None and K.is_gpu(points) and n >= 2:
            keys, grid = (line_keys(points, frame.a), None), False
        frame = None
    if frame is not None and K.is_gpu(points) and keys is None and box is None and n >= 2:
        return _build_rotated(points, frame)
    if box is None:
        box = K.bounds(points)
    gpu = K.is_gpu(points)
    spts = None  # points in sorted order, gathered by the sort's last pass (FUSED_GATHER)
    if keys is not None and keys[1] is not None:
        skeys, perm = K.sort_pairs(keys[0], keys[1], 30)
    elif gpu or keys is not None:  # (the sort's first pass generates the values: no iota array)
        kk = keys[0] if keys is not None else K.morton(points, box, with_iota=False)[0]
        if FUSED_GATHER and gpu and n >= 2:
            skeys, perm, spts = K.sort_keys_iota_gather(kk, points, 30, pad=K.PAD_POINTS)
        else:
            skeys, perm = K.sort_keys_iota(kk, 30)
    else:
        skeys, perm = K.sort_pairs(*K.morton(points, box), 30)
    # level census (grid) and over-full-cell flag (refinement) in one pass over the keys
    census = K.key_census(skeys[:n], HEAVY_RUN) if gpu and n > 1 else None
    sorted_perm = perm
    perm = refine_heavy_cells(points, skeys, perm, heavy=census[1] if census is not None else None)
    # (a refinement reorders over-full cells: the fused gather's order is then stale)
    pts = spts if spts is not None and perm is sorted_perm else K.gather3(points, perm, pad=K.PAD_POINTS)
    nodes, qnodes, depth = K.build_tree(pts, n)
    index = LocalIndex(n, pts, perm, nodes, qnodes, depth, box)
    if grid:
        index.grid = build_grid(index, skeys, density_n, grid_level,
                                counts=census[0] if census is not None else None, gated=grid_gated)
    return index


def _spread15(v: torch.Tensor) -> torch.Tensor:
    """The low 15 bits of int32 v moved to the even bit positions."""
    v = (v | (v << 8)) & 0x00FF00FF
    v = (v | (v << 4)) & 0x0F0F0F0F
    v = (v | (v << 2)) & 0x33333333
    return (v | (v << 1)) & 0x55555555


def plane_keys(rp: torch.Tensor, rbox: torch.Tensor) -> torch.Tensor:
    """30-bit 2-D Morton keys of rotated points by their first two coordinates (the plane's
    own axes), 15 bits each over the square of the larger in-plane extent."""
    s = float(1 << 15) / torch.maximum(rbox[3] - rbox[0], rbox[4] - rbox[1]).clamp_min(1e-30)
    x = ((rp[:, 0] - rbox[0]) * s).clamp_(0.0, 32767.0).to(torch.int32)
    y = ((rp[:, 1] - rbox[1]) * s).clamp_(0.0, 32767.0).to(torch.int32)
    return _spread15(x) | (_spread15(y) << 1)


def _build_rotated(points: torch.Tensor, R: torch.Tensor) -> LocalIndex:
    """build_index in the frame R: curve keys, sort and tree boxes from the rotated points
    (boxes widened by rotate_margin), the index's points (the candidates' coordinates) in
    their own frame, qrot the queries in the rotated one. No grid (flat data)."""
    n = points.shape[0]
    rp = rotate(points, R).contiguous()
    rbox = K.bounds(rp)
    keys = plane_keys(rp, rbox) if _plane_2d(n) else K.morton(rp, rbox, with_iota=False)[0]
    skeys, perm = K.sort_keys_iota(keys, 30)
    census = K.key_census(skeys[:n], HEAVY_RUN) if n > 1 else None
    perm = refine_heavy_cells(rp, skeys, perm, heavy=census[1] if census is not None else None)
    pts = K.gather3(points, perm, pad=K.PAD_POINTS)
    qrot = K.gather3(rp, perm, pad=K.PAD_POINTS)
    nodes, qnodes, depth = K.build_tree(qrot, n)
    m = rotate_margin(rbox)
    for t in (nodes, qnodes):
        t[:, 0:3] -= m
        t[:, 4:7] += m
    return LocalIndex(n, pts, perm, nodes, qnodes, depth, rbox, qrot=qrot)


def grid_level_for(density_n: int, n_local: int, ms: float = GRID_MS) -> int:
    """Grandchild level of the grid from point counts alone (no census, no host read):
    the level whose occupied cells would hold closest to `ms` points on average, in log
    scale, for `density_n` uniform points filling the cube (mean population of the
    occupied cells = lam / (1 - e^-lam), lam = density_n / 8^g; 1B -> 9, 1e8 -> 8,
    1e7 -> 7 — what the census picks for uniform data), then capped so that the slot
    table (16 KiB... 1 KiB per level g-2 cell) stays within 48 B per local point + 64 MiB:
    a rank's share of a large global cube does not allocate the whole cube's finest table
    (a capped level is coarser, hence slower, never wrong)."""
    best, err = 2, math.inf
    for g in range(2, 11):
        lam = max(density_n, 1) / float(8 ** g)
        mean = lam / -math.expm1(-lam) if lam > 1e-12 else 1.0
        e = abs(math.log(max(mean, 1e-9) / ms))
        if e < err:
            best, err = g, e
    while best > 2 and 1024 * 8 ** (best - 2) > 48 * max(n_local, 1) + (64 << 20):
        best -= 1
    return best


def grid_level(distinct: list[int], n: int, ms: float = GRID_MS) -> int:
    """Level of the grid's finest cells (the grandchildren whose runs the k-NN pass
    streams; enumerated through their level-2 ancestors): the level whose occupied cells
    hold closest to `ms` points on average, in log scale (uniform points in a cube, ms = 6:
    1B -> 9 (7.5 per cell), 1e8 -> 8 (6.0), 1e7 -> 7 (4.8)), in [2, 10]. Finer levels cull
    more candidates (at 1e8, k=100: level 8 3.6K evaluations per query vs 4.6K at 7), and
    merged runs keep the segments long."""
    best, err = 2, math.inf
    for lvl in range(2, 11):
        if distinct[lvl] <= 0:
            continue
        e = abs(math.log(max(n / distinct[lvl], 1e-9) / ms))
        if e < err:
            best, err = lvl, e
    return best


def grid_applies(distinct: list[int], n: int, g: int) -> bool:
    """GRID=auto: near-uniform 3-D data at the grid's scale — occupied cells multiply by
    >= 6 from level g-1 to g (planar data: 4, exact copies: 1), and the level's mean
    population is within [2, 256] points."""
    mean = n / max(1, distinct[g])
    return distinct[g] >= 6 * distinct[g - 1] and 2.0 <= mean <= 256.0


def build_grid(index: LocalIndex, skeys: torch.Tensor, density_n: int | None = None,
               level: int | None = None, counts: torch.Tensor | None = None,
               gated: bool = True) -> GridIndex | None:
    """Cell grid over index's sorted points (knn_grid.hip), or None (CPU, GRID=off).

    The level comes from the point counts (grid_level_for); whether the grid applies is
    decided ON THE DEVICE (GRID=auto: lsk_hip_grid_decide from the level census and the
    crowding sum — clustered or multi-scale data keeps the bucket-tree walk of knn_rows,
    which adapts to density): the k-NN launch queues both kernels and the device runs the
    chosen one. No host read, so the build is graph-capturable and a stream of sets never
    waits for the previous set's k-NN here. `gated=False` (a halo index: whether its grid
    serves is the local index's gate): no census, no gate."""
    n = index.n
    if GRID == "off" or n == 0 or not K.is_gpu(index.pts):
        return None
    g = level if level is not None else grid_level_for(density_n if density_n is not None else n, n)
    slots = K.grid_build(index.pts, skeys, n, index.box, g - 2)
    gate = None
    if GRID == "auto" and gated:
        if counts is None:
            counts = K.key_levels_dev(skeys[:n])
        sq = K.grid_sq_dev(slots)
        gate = K.grid_decide(counts, sq, n, g, GRID_CROWD, True)
        census = (counts, sq)
    else:
        census = None
    return GridIndex(slots, g - 2, index.box, gate=gate, census=census)


HEAVY_RUN = 4096  # sorted points sharing one 30-bit key that trigger a second-level key
# HIP-graph captures cannot ask the host whether a cell is over-full. REFINE_CAPTURE
# (set by the caller from an eager warmup on the same kind of data, see LAST_REFINED)
# captures the refinement with fixed, data-independent sizes; otherwise the capture
# records a device flag (CAPTURED_HEAVY) that says after a replay whether some cell
# would have needed it (results stay exact either way, only the speed differs).
REFINE_CAPTURE = False
LAST_REFINED = False
CAPTURED_HEAVY: list = []
# Under host_sync_free() (a stream of point sets) the eager over-full-cell check does not
# read its flag either: it is kept here like a captured one (results stay exact, an
# unrefined cell only costs speed) and the stream reports it once the sets are done.
_SYNC_FREE = [0]
DEFERRED_HEAVY: list = []
# What a stream of sets knows about over-full cells: the flags of its sync-free builds in
# flight (pinned host copy, event) and the last one known. The first set of a stream, and
# every set once a known flag says the data has over-full cells, takes the eager check
# (one host read: refining such a set costs ~55 ms at 5e6 mixed-scale points, leaving it
# unrefined ~105 s, profiles/r5_stream/heavy_ab_deferred.log, heavy_ab_learned.log); sets after a known clean one stay
# sync-free.
_HEAVY_PENDING: list = []
_HEAVY_KNOWN: list = [None]


class host_sync_free:
    """Context: index builds queue no host read (see DEFERRED_HEAVY)."""

    def __enter__(self):
        _SYNC_FREE[0] += 1
        return self

    def __exit__(self, *exc):
        _SYNC_FREE[0] -= 1
        return False


def new_heavy_stream() -> None:
    """A new stream of sets starts knowing nothing about over-full cells: its first set
    takes the eager check (SetStream.run). The DEFERRED_HEAVY report is kept."""
    _HEAVY_PENDING.clear()
    _HEAVY_KNOWN[0] = None


def deferred_heavy_cells(clear: bool = False) -> bool:
    """Whether a build under host_sync_free() met an over-full cell it did not refine."""
    hit = any(bool(f) for f in DEFERRED_HEAVY)
    if clear:
        DEFERRED_HEAVY.clear()
        _HEAVY_PENDING.clear()
        _HEAVY_KNOWN[0] = None
    return hit


def refine_heavy_cells(points: torch.Tensor, skeys: torch.Tensor, perm: torch.Tensor,
                       heavy: torch.Tensor | None = None) -> torch.Tensor:
    """Order inside over-full key cells (docs/ARCHITECTURE.md §2a).

    Keys have 10 bits per axis of the global cube, so a cluster much smaller than one
    cell (huge dynamic range, e.g. a dense core in a large box) shares a single key and
    its buckets all overlap: the k-NN walk cannot cull inside it. The points of every
    run of more than HEAVY_RUN equal keys are re-keyed on the curve of the run's own
    bounding box and re-sorted by (run, local key) with the same radix sort; only the
    order changes (results are exact in any order). Eager: one compare pass + one host
    sync, then work and memory proportional to the over-full runs only. Inside a HIP
    graph capture: see REFINE_CAPTURE. `heavy`: the flag computed already (key_census)."""
    global LAST_REFINED
    n = skeys.shape[0]
    if n <= HEAVY_RUN:
        return perm
    heavy_any = heavy[0] != 0 if heavy is not None else (skeys[HEAVY_RUN:] == skeys[:-HEAVY_RUN]).any()
    if K.is_gpu(skeys) and torch.cuda.is_current_stream_capturing():
        if REFINE_CAPTURE:
            return _refine_all_cells(points, skeys, perm)
        CAPTURED_HEAVY.append(heavy_any)
        return perm
    if _SYNC_FREE[0] and K.is_gpu(skeys):
        while _HEAVY_PENDING and _HEAVY_PENDING[0][1].query():  # flags that landed (no wait)
            _HEAVY_KNOWN[0] = int(_HEAVY_PENDING.pop(0)[0][0]) != 0
        if _HEAVY_KNOWN[0] is False:
            flag = torch.empty(1, dtype=torch.int32, pin_memory=True)
            flag.copy_(heavy_any.reshape(1).to(torch.int32), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            _HEAVY_PENDING.append((flag, ev))
            DEFERRED_HEAVY.append(heavy_any)
            del DEFERRED_HEAVY[:-1024]
            return perm
        # first set of the stream, or the data is known to have over-full cells: eager
        # (the host read waits for this stream's queue)
        _HEAVY_KNOWN[0] = bool(heavy_any)
        if not _HEAVY_KNOWN[0]:
            return perm
        LAST_REFINED = True
        return _refine_heavy_runs(points, skeys, perm)
    if not bool(heavy_any):
        return perm
    LAST_REFINED = True
    return _refine_heavy_runs(points, skeys, perm)


def _local_keys(p: torch.Tensor, seg: torch.Tensor, nseg: int) -> torch.Tensor:
    """30-bit curve keys of points p on the bounding box of their segment."""
    dev = p.device
    if K.is_gpu(p):
        lo, hi = K.segment_bounds(p, seg, nseg)
    else:
        idx3 = seg.long()[:, None].expand(-1, 3)
        lo = torch.full((nseg, 3), math.inf, device=dev).scatter_reduce(0, idx3, p, "amin")
        hi = torch.full((nseg, 3), -math.inf, device=dev).scatter_reduce(0, idx3, p, "amax")
    ext = hi - lo
    ext = torch.where(ext > 0, ext, torch.ones_like(ext))
    sl = seg.long()
    q = ((p - lo[sl]) / ext[sl]).clamp_(0.0, 1.0).contiguous()
    del sl
    del lo, hi, ext
    # unit cube, scale just under 1024 cells so q = 1 stays in the last cell
    # (filled on the device: a host-to-device copy is not allowed inside a graph capture)
    unit = torch.ones(8, dtype=torch.float32, device=dev)
    unit[0:3].zero_()
    unit[6:7].fill_(1023.5)
    k2, _ = K.morton(q, unit, with_iota=False)
    return k2


def _refine_heavy_runs(points, skeys, perm):
    """Eager refinement restricted to the over-full runs (m points): O(m) memory."""
    n = skeys.shape[0]
    dev = skeys.device
    brk = torch.ones(n, dtype=torch.bool, device=dev)
    brk[1:] = skeys[1:] != skeys[:-1]
    starts = torch.nonzero(brk).view(-1)
    ends = torch.cat([starts[1:], torch.tensor([n], dtype=starts.dtype, device=dev)])
    lens = ends - starts
    heavy = lens > HEAVY_RUN
    hs, hl = starts[heavy], lens[heavy]
    nh = int(hs.shape[0])
    m = int(hl.sum())
    first = torch.cumsum(hl, 0) - hl                                          # run offsets in [m]
    # run id of every position: a 1 at each run's first offset, prefix-summed (torch's
    # repeat_interleave gives each run one thread: 3.9 ms for one 1e7-point run)
    seg = torch.zeros(m, dtype=torch.int32, device=dev)
    seg[first[1:]] = 1
    seg = torch.cumsum(seg, 0, dtype=torch.int32)                              # [m]
    pos = hs[seg] + (torch.arange(m, device=dev) - first[seg])                # sorted positions
    del brk, starts, ends, lens, heavy
    src = perm[pos].long()
    k2 = _local_keys(points[src], seg, nh)
    loc = torch.arange(m, dtype=torch.int32, device=dev)
    _, o1 = K.sort_pairs(k2, loc, 30)  # by local key ...
    sbits = max(1, (nh - 1).bit_length())
    _, o2 = K.sort_pairs(seg[o1.long()], o1, sbits)  # ... then stably by run
    out = perm.clone()
    out[pos] = perm[pos[o2.long()]]
    return out


def _refine_all_cells(points, skeys, perm):
    """Graph-capturable refinement: every cell re-keyed, all sizes bounded by n (no host
    sync; ~100 B per point of temporaries — used only when an eager warmup refined)."""
    n = skeys.shape[0]
    dev = skeys.device
    brk = torch.ones(n, dtype=torch.bool, device=dev)
    brk[1:] = skeys[1:] != skeys[:-1]
    rid = (torch.cumsum(brk, 0, dtype=torch.int32) - 1).contiguous()
    del brk
    k2 = _local_keys(points[perm.long()], rid, n)
    pos = torch.arange(n, dtype=torch.int32, device=dev)
    _, o1 = K.sort_pairs(k2, pos, 30)
    rbits = max(1, (n - 1).bit_length())
    _, o2 = K.sort_pairs(rid[o1.long()], o1, rbits)
    return perm[o2.long()].contiguous()


def captured_heavy_cells(clear: bool = False) -> bool:
    """After a replay: whether a captured build met an over-full cell it did not refine."""
    hit = any(bool(f) for f in CAPTURED_HEAVY)
    if clear:
        CAPTURED_HEAVY.clear()
    return hit


def radius_hint2(box: torch.Tensor, n_total: int, k: int) -> float:
    """Uniform-density estimate of the k-th squared distance (only used for groups
    whose own extent is zero)."""
    b = box.detach().cpu().tolist()
    ext = [max(b[3 + a] - b[a], 0.0) for a in range(3)]
    if not all(math.isfinite(e) for e in ext) or n_total <= 0:
        return 1.0
    nz = [e for e in ext if e > 0]
    if not nz:
        return 1.0
    measure = math.prod(nz)
    dim = len(nz)
    rho = n_total / measure
    unit = {1: 2.0, 2: math.pi, 3: 4.0 * math.pi / 3.0}[dim]
    r = (k / (unit * rho)) ** (1.0 / dim)
    return float(r * r)


def radius_hint(box: torch.Tensor, n_total: int, k: int) -> float | torch.Tensor:
    """radius_hint2 without a host round trip: for a GPU box a 1-element device tensor
    computed by a kernel (the k-NN kernel reads it in place), else the host float. Keeps
    the single-rank pipeline free of device->host syncs (HIP-graph capturable)."""
    if K.is_gpu(box):
        return K.radius_hint(box, n_total, k)
    return radius_hint2(box, n_total, k)


def query(index: LocalIndex, cfg: KnnConfig, hint2: float | torch.Tensor = 0.0, extra: LocalIndex | None = None,
          groups: torch.Tensor | None = None, ngroups: int = 0, out: torch.Tensor | None = None,
          stats: KnnStats | None = None, qstatus: torch.Tensor | None = None,
          init_d2: torch.Tensor | None = None, final_out: torch.Tensor | None = None,
          keep_d2: bool = False, deferred: list | None = None,
          ngroups_dev: torch.Tensor | None = None, short_list: bool = False, chunks: int = 1) -> torch.Tensor:
    """k-th squared distance of every (or every listed group of) sorted query of
    `index` against index's tree (+ `extra`'s tree). Returns d2 in sorted order.

    With `final_out` the kernel also writes the final distances in input order
    (final_out[index.perm[q]], fused scatter); then the sorted d2 is only produced (and
    returned) when `keep_d2` or `out` is given, else final_out is returned.

    `deferred` (a list): the failure-word read (a host sync) is not done here but queued
    on the list; `settle(deferred)` does it later — the launch stays asynchronous, so the
    host can queue other work (the overlapped halo exchange) behind it.
    `ngroups_dev` (with `groups`): the list's length as an int32 [1] tensor (on the GPU it
    stays on the device; `ngroups` is then the launch's upper bound); `short_list`: that
    length is expected far below ngroups; `chunks`: the pass as that many launches
    (kernels.knn_gpu)."""
    n = index.n
    want_d2 = final_out is None or keep_d2 or out is not None
    if out is None and want_d2:
        out = torch.empty(n, dtype=torch.float32, device=index.device)
    if n == 0:
        return out if want_d2 else final_out
    if not K.is_gpu(index.pts):
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=index.device)
        pts = index.pts[:n]
        if extra is not None and extra.n > 0:
            pts = torch.cat([pts, extra.pts[:extra.n]])
        if groups is None:
            out.copy_(K.kth_cpu(pts, index.pts[:n], cfg.k, cfg.cut2))
            rows = None
            KERNELS_USED.add("cpu")
        else:
            if ngroups_dev is not None:
                ngroups = int(ngroups_dev.view(-1)[0])
            g = groups[:ngroups].to(torch.int64)
            rows = (g[:, None] * 64 + torch.arange(64)[None, :]).reshape(-1)
            rows = rows[rows < n]
            out[rows] = K.kth_cpu(pts, index.pts[:n][rows], cfg.k, cfg.cut2)
        if final_out is not None:
            if rows is None:
                K.scatter1(out, index.perm, final_out, finalize=True)
            else:
                final_out[index.perm[rows].to(torch.int64)] = K.finalize_distances(out[rows])
        return out if want_d2 else final_out
    trees = [index.tree()] + ([extra.tree()] if extra is not None and extra.n > 0 else [])
    raw = torch.zeros(32, dtype=torch.int64, device=index.device) if stats is not None else None
    kw = dict(groups=groups, ngroups=ngroups, seed=SEED_BUCKETS, init_d2=init_d2,
              out_perm=index.perm if final_out is not None else None, out_final=final_out,
              qrot=index.qrot if len(trees) == 1 else None)
    impl = KNN_IMPL
    # two grids: the halo re-query of a distributed run (the halo index has a grid of its
    # own, pipelines._halo_requery); the local index's gate still picks grid or rows
    if index.qrot is not None and len(trees) != 1:
        raise ValueError("query: an index built in a rotated frame serves its own points only (no extra tree)")
    two_grid = (impl == "rows" and index.grid is not None and len(trees) == 2 and extra.grid is not None
                and cfg.k <= K.ROWS_MAX_K)
    use_grid = two_grid or (impl == "rows" and index.grid is not None and len(trees) == 1
                            and init_d2 is None and cfg.k <= K.ROWS_MAX_K)
    if len(trees) == 1 and init_d2 is None:  # (a local pass, not a halo re-query)
        if use_grid and index.grid.gate is not None:
            GATES_SEEN.append(index.grid.gate)  # grid or rows: resolved by kernels_used()
            GRIDS_SEEN[:] = [index.grid]  # (the last one: debugging)
            del GATES_SEEN[:-1024]  # (reporting only: a long stream keeps the last sets)
        else:
            KERNELS_USED.add("grid" if use_grid else impl)
    fw = K.knn_gpu(index.pts, n, trees, cfg.k, cfg.cut2, hint2, out, stats=raw, qstatus=qstatus,
                   impl="grid" if use_grid else impl, debug_fail_mod=DEBUG_FAIL_MOD,
                   grid=index.grid.view() if use_grid else None, ngroups_dev=ngroups_dev,
                   expect_grid=GRID_EXPECT[0], short_list=short_list, chunks=chunks,
                   grid2=extra.grid.view()[:4] if two_grid else None, **kw)
    gate = index.grid.gate if use_grid else None
    def check() -> bool:
        # one 4-byte read: failures beyond the list capacity (pathological input) rerun
        # the whole query on the exact kernel (on the current stream; returns True then)
        nfail = fw.value()
        rerun = nfail > fw.cap
        if gate is not None:  # (staged with the failure word: no wait for later work)
            GRID_EXPECT[0] = bool(fw.gate_value(gate))
        if rerun:
            K.knn_gpu(index.pts, n, trees, cfg.k, cfg.cut2, hint2, out, impl="exact", ngroups_dev=ngroups_dev,
                      **kw)
        if stats is not None:
            stats.add_fallback(nfail)
            stats.add(raw)
        return rerun

    if torch.cuda.is_current_stream_capturing():
        slot = len(CAPTURED_FAIL_WORDS)
        if fw.count is not None and CAPTURE_PEAKS is not None and slot < CAPTURE_PEAKS.numel():
            fw.peak = CAPTURE_PEAKS[slot:slot + 1]
            torch.maximum(fw.peak, fw.count.to(torch.int64) & 0xFFFFFFFF, out=fw.peak)
        CAPTURED_FAIL_WORDS.append(fw)
        if stats is not None:
            stats.add(raw)
    elif fw.count is None:
        if stats is not None:
            stats.add(raw)
    elif deferred is not None:
        fw.stage(gate)  # the later read waits for this launch only
        deferred.append(check)
    else:
        check()
    return out if want_d2 else final_out


# k-NN kernels the whole-set passes of this process used ("grid", "rows", "exact"): the
# bench reports them next to its number. Passes whose kernel the device picks leave their
# gate in GATES_SEEN; kernels_used() reads them (a host read: after the timed region).
KERNELS_USED: set = set()
GATES_SEEN: list = []
GRIDS_SEEN: list = []


def kernels_used() -> list:
    used = set(KERNELS_USED)
    for gate in GATES_SEEN:
        used.add("grid" if int(gate.item()) else "rows")
    return sorted(used)


def reset_kernels_used() -> None:
    KERNELS_USED.clear()
    GATES_SEEN.clear()


def settle(deferred: list) -> bool:
    """Run the failure checks `query(..., deferred=...)` queued (in launch order). True
    when one of them queued a rerun (its output is rewritten behind the current stream's
    work: a copy of it queued earlier is stale)."""
    rerun = False
    while deferred:
        rerun = bool(deferred.pop(0)()) or rerun
    return rerun


def verify_captured_failures(clear: bool = False) -> int:
    """After replaying a captured graph: total backstop queries of the captured launches;
    raises if one overflowed its failure list (the graph's output is then incomplete)."""
    total = 0
    for fw in CAPTURED_FAIL_WORDS:
        v = fw.value()
        peak = getattr(fw, "peak", None)
        if peak is not None:
            v = max(v, int(peak.item()))  # the worst replay
        if v > fw.cap:
            raise RuntimeError(f"k-NN failure list overflow in a captured graph ({v} > {fw.cap}): "
                               "rerun eagerly")
        total += v
    if clear:
        CAPTURED_FAIL_WORDS.clear()
    return total


def knn_distances(points: torch.Tensor, k: int, max_radius: float = math.inf,
                  stats: KnnStats | None = None) -> torch.Tensor:
    """Distance from every point to its k-th nearest neighbour among `points`
    (itself counted), in input order — the single-rank reference output."""
    cfg = KnnConfig(k=k, max_radius=max_radius)
    probe = FrameProbe(points, k)
    if FRAME_EARLY:  # the probe read before the build (a short host wait, no wasted build)
        frame = probe.result()
        index = build_index(points, grid=frame is None, frame=frame)
    else:  # read after the unrotated build: no host wait before it
        index = build_index(points, grid=True)
        frame = probe.result()
        if frame is not None:  # a tilted plane: rebuilt in its principal-axes frame
            index = build_index(points, frame=frame)
    hint2 = radius_hint(index.box, index.n, k)
    out = torch.empty(index.n, dtype=torch.float32, device=points.device)
    return query(index, cfg, hint2, stats=stats, final_out=out)
