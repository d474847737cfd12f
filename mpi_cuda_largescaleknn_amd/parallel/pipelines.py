"""Distributed k-th-NN distance pipelines (one rank per GPU).

Fast path ("halo" mode), shared by both entrypoints:

1. (unordered only) spatial redistribution — global bounds (all-reduce), 30-bit Hilbert
   curve keys in the global cube, global histogram of the top 16 key bits (all-reduce) ->
   P-1 balanced splitters, destination-rank partition (radix sort by rank), rows moved
   with all-to-all-v. This is the sequence-parallel/Ulysses-style reshard of SURVEY §5.7a
   and replaces the reference's P-round ring of whole trees (unorderedDataVariant.cu:
   173-205, P kNN passes per query, O(P) traffic).
2. local index (Hilbert sort + bucket tree + cell grid) and local k-NN on the owned
   points (knn_grid.hip for near-uniform data, knn_rows.hip otherwise).
3. halo exchange — each rank publishes the top levels of its tree with per-node max
   k-NN radius (all-gather, tiny); every rank sends exactly the points that fall
   inside another rank's radius-inflated boxes (halo_mask kernel, all-to-all-v); the
   receiver builds a halo tree and re-queries only the query groups that have a halo
   point closer than their current k-th distance (2-tree k-NN kernel). Exact, because
   local radii are upper bounds and the filter is conservative (halo.hip).
   Replaces the bounds-culled whole-tree pulls of prePartitionedDataVariant.cu:304-357.
4. (unordered only) distances return to the origin rank with the reverse all-to-all-v
   and are scattered to input order.

The reference-faithful schedules (ring rotation, peer pulls) live in ``refalgo.py``.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import torch

from ..models import knn_engine as E
from ..ops import kernels as K
from ..utils import trace
from .comm import Comm
from .faults import HEARTBEAT

SPLIT_BITS = 16  # splitter resolution: top 16 of the 30 curve-key bits


@dataclass
class PhaseTimer:
    """Per-phase wall times (device-synchronised when enabled)."""
    enabled: bool = False
    device: torch.device | None = None
    times: dict = field(default_factory=dict)
    _t: float = 0.0

    def start(self):
        if self.enabled:
            self._sync()
            self._t = time.perf_counter()

    def mark(self, name: str):
        HEARTBEAT.beat(name)
        trace.mark("lsknn:" + name)
        if self.enabled:
            self._sync()
            now = time.perf_counter()
            self.times[name] = self.times.get(name, 0.0) + (now - self._t)
            self._t = now

    def _sync(self):
        if self.device is not None and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


@dataclass
class RunInfo:
    timer: PhaseTimer
    stats: E.KnnStats = field(default_factory=E.KnnStats)
    # plain ints, or 1-element device tensors for counts the pipeline does not read back
    # itself (the re-query's group count: no host sync on the hot path); plain_counts()
    # resolves them for reporting
    counts: dict = field(default_factory=dict)

    def plain_counts(self) -> dict:
        return {c: (int(v.reshape(-1)[0]) if isinstance(v, torch.Tensor) else v) for c, v in self.counts.items()}


# --------------------------------------------------------------------------- helpers
def global_box(points: torch.Tensor, comm: Comm) -> torch.Tensor:
    box = K.bounds(points)
    if comm.distributed:
        v = torch.cat([box[0:3], -box[3:6]])
        comm.allreduce_(v, "min")
        box = torch.cat([v[0:3], -v[3:6], box[6:8]])
        box = K.box_finalize(box)
    return box


SPLIT_TOL = 0.02  # accepted load imbalance per rank when snapping splitters to coarse cells
HIST_SAMPLE = 8   # splitter histogram over every 8th key of ranks holding >= 2^20 points


def _hist_sample(n: int) -> int:
    """Key sampling stride of the splitter histogram (balance only; exactness does not
    depend on the splitters)."""
    if n < (1 << 20):
        return 1
    # at most ~8M sampled keys: their atomics into the shared histogram cost 2.6 ms per
    # 500M-point rank at stride 8 (profiles/archive/r1_v20/lb_scaling), and 8M samples already
    # place the splitters far inside the 2 % tolerance
    return max(HIST_SAMPLE, n >> 23)


def _splitters(hist: torch.Tensor, total: int, size: int) -> list[int]:
    """Bin starts of ranks 1..P-1 so that each rank owns ~total/P points.

    Each splitter is snapped to the coarsest octree cell boundary (level m: 8^m cells,
    2^(SPLIT_BITS-3m) histogram bins) whose count stays within SPLIT_TOL of the ideal
    share. A rank range ending mid-cell owns a sliver of a distant cell; bucket-tree
    nodes spanning that Z-order jump have huge boxes and blow up the halo (uniform data,
    8 ranks: exact octants instead of octants + slivers, ~3x smaller halos)."""
    cum = torch.cumsum(hist.to(torch.int64), 0)
    excl_t = torch.cat([torch.zeros(1, dtype=torch.int64), cum])  # excl[b] = count below bin b
    nb = hist.shape[0]
    tol = max(1, int(SPLIT_TOL * total / max(size, 1)))
    targets = torch.tensor([(total * j) // size for j in range(1, size)], dtype=torch.int64)
    firsts = torch.searchsorted(excl_t[:-1], targets, right=False).tolist()
    excl = excl_t.tolist()
    out = []
    for j in range(1, size):
        target = (total * j) // size
        b = int(firsts[j - 1])
        best = b
        for m in range(1, SPLIT_BITS // 3 + 1):
            step = 1 << (SPLIT_BITS - 3 * m)
            lo = (b // step) * step
            cands = [c for c in (lo, min(lo + step, nb)) if 0 <= c <= nb]
            c = min(cands, key=lambda x: abs(excl[x] - target))
            if abs(excl[c] - target) <= tol:
                best = c
                break
        out.append(min(max(best, out[-1] if out else 0), nb))
    return out


def _dest_and_perm(keys: torch.Tensor, splitters: list[int], size: int):
    n = keys.shape[0]
    dev = keys.device
    shift = 30 - SPLIT_BITS
    if K.is_gpu(keys):
        from .. import _native
        lib = _native.hip()
        split_t = torch.tensor(splitters if splitters else [0], dtype=torch.int32, device=dev)
        dest = torch.empty(n, dtype=torch.int32, device=dev)
        iota = torch.empty(n, dtype=torch.int32, device=dev)
        K.check(lib.lsk_hip_dest_rank(keys.data_ptr(), n, split_t.data_ptr(), len(splitters), shift,
                                      dest.data_ptr(), iota.data_ptr(), K._stream(keys)), "dest_rank")
        counts = torch.zeros(size, dtype=torch.int32, device=dev)
        K.check(lib.lsk_hip_count_dest(dest.data_ptr(), n, size, counts.data_ptr(), K._stream(keys)),
                "count_dest")
    else:
        bins = (keys.to(torch.int64) >> shift)
        split_t = torch.tensor(splitters, dtype=torch.int64)
        dest = torch.searchsorted(split_t, bins, right=True).to(torch.int32)
        iota = torch.arange(n, dtype=torch.int32)
        counts = torch.bincount(dest.to(torch.int64), minlength=size).to(torch.int32)
    bits = max(1, (size - 1).bit_length())
    _, perm = K.sort_pairs(dest, iota, bits)
    return perm, counts


def redistribute(points: torch.Tensor, comm: Comm, box: torch.Tensor, info: RunInfo):
    """Move every point to the rank owning its curve-key range.
    Returns (owned points, recv_counts, send permutation, send counts)."""
    size = comm.size
    keys, _ = K.morton(points, box, with_iota=False)
    nb = 1 << SPLIT_BITS
    hist = torch.zeros(nb, dtype=torch.int32, device=points.device)
    if K.is_gpu(keys):
        from .. import _native
        K.check(_native.hip().lsk_hip_key_histogram(keys.data_ptr(), keys.shape[0], 30 - SPLIT_BITS,
                                                   _hist_sample(keys.shape[0]), hist.data_ptr(),
                                                   K._stream(keys)), "key_histogram")
    else:
        sk = keys[::_hist_sample(keys.shape[0])]
        hist += torch.bincount((sk.to(torch.int64) >> (30 - SPLIT_BITS)), minlength=nb).to(torch.int32)
    comm.allreduce_(hist, "sum")
    hist_h = hist.cpu()
    total = int(hist_h.to(torch.int64).sum())
    splitters = _splitters(hist_h, total, size)
    perm, counts = _dest_and_perm(keys, splitters, size)
    send = K.gather3(points, perm)
    send_counts, recv_counts = comm.count_exchange(counts)  # one host read
    info.timer.mark("partition")
    recv, recv_counts = comm.alltoallv(send, send_counts, recv_counts)
    info.timer.mark("alltoallv_points")
    info.counts["sent_points"] = sum(send_counts) - send_counts[comm.rank]
    info.counts["owned_points"] = int(recv.shape[0])
    return recv, recv_counts, perm, send_counts


# points per host->device chunk of the streamed redistribution (env LSKNN_STREAM_CHUNK);
# smaller chunks shorten the tail after the last copy (forced 1-rank RCCL, 1e8 points:
# 32M / 16M / 8M -> 170.6 / 169.5 / 169.3 ms per step; profiles/archive/r2_return)
STREAM_CHUNK = int(os.environ.get("LSKNN_STREAM_CHUNK", str(1 << 24)))


@dataclass
class Redist:
    """Bookkeeping of a (streamed) redistribution, for the result return."""
    owned: torch.Tensor           # [m, 3] points this rank owns (received-row order)
    ret_index: torch.Tensor       # int64: owned-row order -> return-send order (by dest)
    ret_counts: list              # rows returned to each rank
    origin_index: torch.Tensor    # int64: return-receive order -> local input row
    back_counts: list             # rows coming back from each rank
    box: torch.Tensor             # global box of all points (exact)
    # per stream chunk (grouped return): local input span, send permutation, rows sent
    # to / received from each rank, first owned row of the chunk
    spans: list = field(default_factory=list)
    perms: list = field(default_factory=list)
    scs: list = field(default_factory=list)
    rcs: list = field(default_factory=list)
    bases: list = field(default_factory=list)


def redistribute_stream(host_pts: torch.Tensor, comm: Comm, info: RunInfo,
                        chunk: int | None = None) -> Redist:
    """Spatial redistribution fed in chunks straight from host memory: the host->device
    copies of all chunks are queued on a copy stream up front, and chunk c is keyed,
    partitioned and sent (all-to-all-v) while chunks c+1.. are still in flight, so the
    PCIe transfer hides the partitioning and most of the xGMI exchange.

    Ownership uses the cube of the ranks' FIRST chunks (all-reduced) and splitters from
    their key histogram; points outside that cube get clamped keys. Neither affects
    exactness (the k-NN is exact for any ownership); they only shape the load balance, so
    a first chunk that is unrepresentative of the rest (e.g. input sorted in space) costs
    speed, not correctness. The exact global box is all-reduced after the last chunk."""
    dev = comm.device
    n = host_pts.shape[0]
    gpu = dev.type == "cuda"
    size = comm.size
    chunk = max(1, int(chunk or STREAM_CHUNK))
    # every chunk is one all-to-all-v (and one return group member): all ranks must run
    # the same number of them, so the count is the maximum over ranks and ranks with fewer
    # points get empty trailing chunks (uneven inputs: prePartitioned files, empty ranks)
    nch = torch.tensor([max(1, -(-n // chunk))], dtype=torch.int64, device=dev)
    comm.allreduce_(nch, "max")
    nch = int(nch.item())
    spans = [(min(c * chunk, n), min((c + 1) * chunk, n)) for c in range(nch)]
    cur = torch.cuda.current_stream(dev) if gpu else None
    copy_stream = torch.cuda.Stream(dev) if gpu else None
    dchunks, events = [], []
    for s, e in spans:
        if gpu:
            d = torch.empty((e - s, 3), dtype=torch.float32, device=dev)  # allocated on `cur`
            copy_stream.wait_stream(cur)
            with torch.cuda.stream(copy_stream):
                d.copy_(host_pts[s:e], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(copy_stream)
        else:
            d, ev = host_pts[s:e], None
        dchunks.append(d)
        events.append(ev)

    def ready(c):
        if events[c] is not None:
            cur.wait_event(events[c])
        return dchunks[c]

    # ownership cube from every rank's first chunk; exact bounds accumulate per chunk
    first = ready(0)
    box0 = global_box(first, comm)
    lo_hi = K.bounds(first)[0:6].clone()
    nb = 1 << SPLIT_BITS
    keys0, _ = K.morton(first, box0, with_iota=False)
    hist = torch.zeros(nb, dtype=torch.int32, device=dev)
    if K.is_gpu(keys0):
        from .. import _native
        K.check(_native.hip().lsk_hip_key_histogram(keys0.data_ptr(), keys0.shape[0], 30 - SPLIT_BITS,
                                                   _hist_sample(keys0.shape[0]), hist.data_ptr(),
                                                   K._stream(keys0)), "key_histogram")
    elif keys0.numel():
        sk = keys0[::_hist_sample(keys0.shape[0])]
        hist += torch.bincount((sk.to(torch.int64) >> (30 - SPLIT_BITS)), minlength=nb).to(torch.int32)
    comm.allreduce_(hist, "sum")
    hist_h = hist.cpu()
    splitters = _splitters(hist_h, max(1, int(hist_h.to(torch.int64).sum())), size)
    info.timer.mark("partition")
    recvs, rcs, perms, scs = [], [], [], []
    for c, (s, e) in enumerate(spans):
        pts_c = first if c == 0 else ready(c)
        if c:
            b = K.bounds(pts_c)
            lo_hi = torch.cat([torch.minimum(lo_hi[0:3], b[0:3]), torch.maximum(lo_hi[3:6], b[3:6])])
        keys_c = keys0 if c == 0 else K.morton(pts_c, box0, with_iota=False)[0]
        perm_c, counts_c = _dest_and_perm(keys_c, splitters, size)
        send_c = K.gather3(pts_c, perm_c)
        sc, rc = comm.count_exchange(counts_c)  # one host read per chunk
        recv_c, rc = comm.alltoallv(send_c, sc, rc)
        recvs.append(recv_c)
        rcs.append(rc)
        perms.append(perm_c)
        scs.append(sc)
    info.timer.mark("alltoallv_points")
    owned = torch.cat(recvs) if len(recvs) > 1 else recvs[0]
    # exact global box (radius hint, local index keys)
    v = torch.cat([lo_hi[0:3], -lo_hi[3:6]])
    comm.allreduce_(v, "min")
    box = torch.zeros(8, dtype=torch.float32, device=dev)
    box[0:3] = v[0:3]
    box[3:6] = -v[3:6]
    box = K.box_finalize(box)
    # return plan: owned rows are chunk-major, rank-minor; the return sends each rank its
    # rows chunk by chunk, and the origin maps them back through the chunk permutations
    ret_parts, ret_counts = [[] for _ in range(size)], [0] * size
    orig_parts, back_counts = [[] for _ in range(size)], [0] * size
    base = 0
    bases = []
    for c, (s, e) in enumerate(spans):
        bases.append(base)
        ro = _offsets(rcs[c])
        so = _offsets(scs[c])
        for j in range(size):
            if rcs[c][j]:
                ret_parts[j].append(torch.arange(base + ro[j], base + ro[j + 1], device=dev))
                ret_counts[j] += rcs[c][j]
            if scs[c][j]:
                orig_parts[j].append(perms[c][so[j]:so[j + 1]].to(torch.int64) + s)
                back_counts[j] += scs[c][j]
        base += ro[-1]
    empty = torch.zeros(0, dtype=torch.int64, device=dev)
    ret_index = torch.cat([t for parts in ret_parts for t in parts] or [empty])
    origin_index = torch.cat([t for parts in orig_parts for t in parts] or [empty])
    info.counts["sent_points"] = sum(sum(sc) - sc[comm.rank] for sc in scs)
    info.counts["owned_points"] = int(owned.shape[0])
    info.counts["stream_chunks"] = len(spans)
    return Redist(owned, ret_index, ret_counts, origin_index, back_counts, box,
                  spans=spans, perms=perms, scs=scs, rcs=rcs, bases=bases)


RETURN_GROUPS = 4  # result-return groups of stream chunks (each: all-to-all-v, scatter, D2H)


def _return_grouped(R: Redist, dist_owned: torch.Tensor, comm: Comm, res: torch.Tensor,
                    out: torch.Tensor) -> None:
    """Result return in groups of stream chunks: group g's all-to-all-v and scatter
    complete the local rows of its chunks, whose device-to-host copy into the pinned
    `out` then runs on a copy stream while group g+1 is exchanged (the PCIe copy of the
    results hides under the xGMI return). Counts are known from the redistribution."""
    dev = res.device
    size = comm.size
    nch = len(R.spans)
    ng = max(1, min(RETURN_GROUPS, nch))
    bounds = [nch * g // ng for g in range(ng + 1)]
    cur = torch.cuda.current_stream(dev)
    copy_stream = torch.cuda.Stream(dev)
    empty = torch.zeros(0, dtype=torch.int64, device=dev)
    for g in range(ng):
        cs = range(bounds[g], bounds[g + 1])
        ret, orig, rc, bc = [], [], [0] * size, [0] * size
        for j in range(size):
            for c in cs:
                ro, so = _offsets(R.rcs[c]), _offsets(R.scs[c])
                if R.rcs[c][j]:
                    ret.append(torch.arange(R.bases[c] + ro[j], R.bases[c] + ro[j + 1], device=dev))
                    rc[j] += R.rcs[c][j]
                if R.scs[c][j]:
                    orig.append(R.perms[c][so[j]:so[j + 1]].to(torch.int64) + R.spans[c][0])
                    bc[j] += R.scs[c][j]
        ret_i = torch.cat(ret) if ret else empty
        orig_i = torch.cat(orig) if orig else empty
        back, _ = comm.alltoallv(dist_owned[ret_i], rc, recv_counts=bc)
        K.scatter1(back, orig_i.to(torch.int32), res, finalize=False)
        s0, s1 = R.spans[cs[0]][0], R.spans[cs[-1]][1]
        if s1 > s0:
            copy_stream.wait_stream(cur)
            with torch.cuda.stream(copy_stream):
                out[s0:s1].copy_(res[s0:s1], non_blocking=True)
    res.record_stream(copy_stream)
    cur.wait_stream(copy_stream)


def _offsets(counts):
    o = [0]
    for x in counts:
        o.append(o[-1] + int(x))
    return o


def _publish(index: E.LocalIndex, radii_nodes: torch.Tensor, comm: Comm, cfg: E.KnnConfig):
    """All-gather the top cfg.publish_levels levels of every rank's tree (`radii_nodes`:
    index's tree with per-node k-th squared radius bounds in lo.w). Returns (pub_all
    [P, rows, 8], published depths (device int32 [P]), per-rank float offsets)."""
    levels = cfg.publish_levels
    my_levels = min(levels, index.depth)
    rows = 2 << levels
    pub = torch.zeros((rows, 8), dtype=torch.float32, device=index.device)
    pub[:, 0:3] = math.inf
    pub[:, 4:7] = -math.inf
    take = min(rows, radii_nodes.shape[0], 2 << my_levels)
    pub[:take] = radii_nodes[:take]
    # the published depth rides in node 0's unused hi.w: one all-gather, no host read
    pub[0, 7] = float(my_levels)
    pub_all = comm.allgather(pub)                       # [P, rows, 8]
    depths = pub_all[:, 0, 7].to(torch.int32)           # (device)
    return pub_all, depths, [j * rows * 8 for j in range(comm.size)]


def _halo_send(index: E.LocalIndex, radii_nodes: torch.Tensor, comm: Comm, cfg: E.KnnConfig, info: RunInfo,
               marks: bool = True) -> torch.Tensor:
    """Publish the top levels of `radii_nodes` (index's tree with per-node k-th squared
    radius bounds in lo.w), filter and pack own points for every other rank, exchange:
    returns the received halo points."""
    size, rank = comm.size, comm.rank
    n = index.n
    dev = index.device
    pub_all, depths, offs = _publish(index, radii_nodes, comm, cfg)
    if marks:
        info.timer.mark("halo_publish")
    pts = index.pts[:n]
    mask = K.halo_mask(pts, pub_all.reshape(-1), offs, depths, rank)
    recv_counts = None
    if K.is_gpu(pts):
        from .. import _native
        lib = _native.hip()
        counts = torch.zeros(size, dtype=torch.int32, device=dev)
        K.check(lib.lsk_hip_mask_counts(mask.data_ptr(), n, size, counts.data_ptr(), K._stream(pts)),
                "mask_counts")
        send_counts, recv_counts = comm.count_exchange(counts)  # one host read
        offsets = [0]
        for c in send_counts:
            offsets.append(offsets[-1] + c)
        send = torch.empty((offsets[-1], 3), dtype=torch.float32, device=dev)
        off_t = torch.tensor(offsets[:-1], dtype=torch.int64, device=dev)
        cursors = torch.zeros(size, dtype=torch.int32, device=dev)
        K.check(lib.lsk_hip_halo_pack(pts.data_ptr(), mask.data_ptr(), n, size, off_t.data_ptr(),
                                      cursors.data_ptr(), send.data_ptr(), K._stream(pts)), "halo_pack")
    else:
        parts, send_counts = [], []
        for j in range(size):
            sel = ((mask >> j) & 1).bool()
            parts.append(pts[sel])
            send_counts.append(int(sel.sum()))
        send = torch.cat(parts) if parts else pts[:0]
    if marks:
        info.timer.mark("halo_filter")
    recv, _ = comm.alltoallv(send, send_counts, recv_counts)
    info.counts["halo_sent"] = int(sum(send_counts))
    info.counts["halo_recv"] = int(recv.shape[0])
    if marks:
        info.timer.mark("halo_alltoallv")
    return recv


# The halo re-query on knn_grid2 (two grids: local + halo, see halo_index) instead of the
# bucket-tree kernel with two trees. 1B / 8 ranks, per-rank replay (profiles/r6_rank): the
# re-query launch 6.2 ms (rows) -> 4.85 ms with the halo grid one level coarser than the
# local one (its shell of points is thin: at the local level 2.4x the cells per wave, 5.8
# ms); the grid build adds ~0.4 ms; per-rank total 122.4 -> 120.5 ms. 0: knn_rows.
HALO_GRID = os.environ.get("LSKNN_HALO_GRID", "1") != "0"
HALO_GRID_DLEVEL = int(os.environ.get("LSKNN_HALO_GRID_DLEVEL", "-1"))  # halo grid level - local level
# the re-query's first range ends at the local k-th (0: the density estimate instead; A/B at
# 1B / 8: rows 6.2 vs 7.1 ms, grid 6.2 vs 6.5)
REQUERY_BOUND = os.environ.get("LSKNN_REQUERY_BOUND", "1") != "0"


def halo_index(index: E.LocalIndex, recv: torch.Tensor) -> E.LocalIndex:
    """Index of the received halo points. With a local grid the halo points get a grid of
    their own at the local grid's level (no gate: the local index's gate decides for both),
    so the re-query runs on the grid kernel over both sources when the local pass did
    (knn_grid2); the bucket-tree kernel with two trees otherwise."""
    g = HALO_GRID and index.grid is not None
    lvl = max(2, index.grid.level + 2 + HALO_GRID_DLEVEL) if g else None
    return E.build_index(recv, grid=g, grid_level=lvl, grid_gated=False)


def _halo_requery(index: E.LocalIndex, d2: torch.Tensor, recv: torch.Tensor, cfg: E.KnnConfig,
                  hint2: float | torch.Tensor, info: RunInfo, final_out: torch.Tensor | None,
                  hidx: E.LocalIndex | None = None) -> torch.Tensor:
    """Halo index from the received points (`hidx`: built already); re-query (against
    local + halo) every query group a halo point can reach within its local k-th radius
    (index.nodes must carry the final radii: tree_set_radii). Updates d2 / final_out in
    place."""
    n = index.n
    dev = index.device
    nh = recv.shape[0]
    if nh == 0 or n == 0:
        return d2
    if hidx is None:
        hidx = halo_index(index, recv)
    if K.is_gpu(index.pts):
        from .. import _native
        lib = _native.hip()
        ng = (n + 63) // 64
        flags = torch.zeros(ng, dtype=torch.int32, device=dev)
        # halo points against the local radius-annotated tree
        K.check(lib.lsk_hip_flag_groups_inverse(hidx.pts.data_ptr(), nh, index.nodes.data_ptr(), index.depth,
                                                ng, flags.data_ptr(), K._stream(index.pts)), "flag_groups")
        glist = torch.empty(ng, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        K.check(lib.lsk_hip_compact_flags(flags.data_ptr(), ng, glist.data_ptr(), cnt.data_ptr(),
                                          K._stream(index.pts)), "compact_flags")
        # the flagged-group count stays on the device (no host read here): the
        # re-query takes the device-counted list in the strided form sized for a short list
        # (~3 % of the groups at 1B / 8 ranks)
        info.counts["requery_groups"] = cnt
        info.timer.mark("halo_tree")
        # the local k-th distance bounds the true one from above: the re-query starts with
        # a tight first range
        E.query(index, cfg, hint2, extra=hidx, groups=glist, ngroups=ng, ngroups_dev=cnt, short_list=True,
                out=d2, stats=info.stats if cfg.collect_stats else None, init_d2=d2 if REQUERY_BOUND else None,
                final_out=final_out)
    else:
        info.timer.mark("halo_tree")
        E.query(index, cfg, hint2, extra=hidx, out=d2, final_out=final_out)
    info.timer.mark("halo_requery")
    return d2


def halo_refine(index: E.LocalIndex, d2: torch.Tensor, comm: Comm, cfg: E.KnnConfig,
                hint2: float | torch.Tensor,
                info: RunInfo, final_out: torch.Tensor | None = None) -> torch.Tensor:
    """Exchange boundary candidates and re-query the affected query groups (exact).
    `final_out` (input order of index.perm) already holds the local final distances; the
    re-query updates it in place together with the sorted d2."""
    K.tree_set_radii(index.nodes, index.n, d2)
    recv = _halo_send(index, index.nodes, comm, cfg, info)
    return _halo_requery(index, d2, recv, cfg, hint2, info, final_out)


# Overlapped halo exchange (the reference rotates shards only after the
# local query, unorderedDataVariant.cu:204). The halo filter needs per-node radius bounds;
# instead of waiting for the local k-NN's radii, a copy of the tree gets a-priori upper
# bounds from the bucket boxes (K.tree_set_radii_ub: the ceil(k/64)+1 buckets around a
# leaf hold >= k points), and publish / filter / pack / alltoallv run on a side stream
# while the local k-NN kernel runs on the compute stream. The halo is a superset of the
# exact one (looser radii); the re-query flags groups with the final radii, so the result
# is unchanged. Env LSKNN_OVERLAP_HALO=0 restores the sequential order.
OVERLAP_HALO = os.environ.get("LSKNN_OVERLAP_HALO", "1") != "0"
_SIDE_STREAMS: dict = {}


def _overlap_streams(dev: torch.device):
    """(compute, side) non-blocking streams of this thread (loopback ranks are threads).
    The k-NN also leaves the default stream: any implicit default-stream synchronisation
    on the side path (pageable copies) must not wait for the k-NN kernel. The side stream
    has the high priority: once the k-NN grid fills every CU, a side kernel only starts
    when the dispatcher prefers its queue as k-NN workgroups retire."""
    import threading
    key = (threading.get_ident(), dev.index)
    st = _SIDE_STREAMS.get(key)
    if st is None:
        hi = torch.cuda.Stream.priority_range()[1]  # (low, high): high is the smaller number
        st = _SIDE_STREAMS[key] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev, priority=hi))
    return st


def _radius_bounds(index: E.LocalIndex, cfg: E.KnnConfig) -> torch.Tensor:
    """A copy of the tree with a-priori per-node k-th squared radius bounds, capped at the
    cutoff (-r): candidates at or beyond it are never counted, so no query needs them."""
    ub = K.tree_set_radii_ub(index.nodes.clone(), index.pts, index.n, cfg.k)
    if math.isfinite(cfg.cut2):
        ub[:, 3].clamp_(max=cfg.cut2 * (1.0 + 2.0 ** -16))
    return ub


def knn_with_halo(index: E.LocalIndex, comm: Comm, cfg: E.KnnConfig, hint2: float | torch.Tensor,
                  info: RunInfo, final_out: torch.Tensor, hook=None) -> torch.Tensor:
    """Local k-NN of every owned query + halo exchange + re-query (distributed runs).
    Returns the sorted d2; `final_out` receives the final distances (index.perm order).
    `hook(after) -> stream | None` (overlapped GPU path): called right after the local
    k-NN is queued — independent work issued there (SetStream: the next point set's
    redistribution) runs under the k-NN, ordered after `after` (a stream, or an event
    recorded before the k-NN launch); the halo exchange / result return is ordered after
    the stream it returns."""
    stats = info.stats if cfg.collect_stats else None
    gpu = K.is_gpu(index.pts)
    capturing = gpu and torch.cuda.is_current_stream_capturing()
    if comm.size == 1 and not HALO_ONE_RANK:
        # one rank (a forced multi-rank run): no peer, so no halo — the local pass is the
        # result; the hook's work is issued right behind the k-NN launch, the failure
        # check after it
        pend: list = []
        pre = None
        if gpu and hook is not None and REDIST_UNDER_KNN:
            pre = torch.cuda.Event()
            pre.record(torch.cuda.current_stream(index.device))
        d2 = E.query(index, cfg, hint2, stats=stats, final_out=final_out, keep_d2=True,
                     deferred=None if capturing or not gpu else pend)
        if hook is not None:
            # the hook's work follows what precedes the k-NN (REDIST_UNDER_KNN), else the k-NN
            st = hook(pre if pre is not None else (torch.cuda.current_stream(index.device) if gpu else None))
            if st is not None:
                # the result return's collectives (queued on this stream next) follow the
                # hook's: one communicator, never two collectives in flight
                torch.cuda.current_stream(index.device).wait_stream(st)
        E.settle(pend)
        info.timer.mark("knn_local")
        return d2
    if not OVERLAP_HALO or capturing:
        d2 = E.query(index, cfg, hint2, stats=stats, final_out=final_out, keep_d2=True)
        info.timer.mark("knn_local")
        return halo_refine(index, d2, comm, cfg, hint2, info, final_out=final_out)
    n = index.n
    ng = (n + 63) // 64
    # 1. boundary groups: a-priori radius bounds (tree_set_radii_ub) against the other
    #    ranks' published tree tops; a group whose bound keeps it inside this rank's
    #    region needs no halo at all
    if gpu:
        dev = index.device
        cur = torch.cuda.current_stream(dev)
        comp, side = _overlap_streams(dev)
        comp.wait_stream(cur)
        side.wait_stream(cur)
        ctx = torch.cuda.stream(comp)
    else:
        import contextlib
        ctx = contextlib.nullcontext()
    with ctx:
        ub = _radius_bounds(index, cfg)
        pub_all, depths, offs = _publish(index, ub, comm, cfg)
        bflags = K.boundary_groups(ub, index.depth, ng, pub_all, offs, depths, comm.rank)
        blist, bcnt = K.compact_flags(bflags)
        ilist, icnt = K.compact_flags(1 - bflags)
        del ub, bflags
    if gpu:
        ev_pub = torch.cuda.Event()
        ev_pub.record(comp)
        cur.wait_event(ev_pub)  # (the hook's collectives follow the publish)
    pend: list = []
    with ctx:
        # (allocated and zeroed on the compute stream: the passes below write it there)
        d2 = torch.zeros(n, dtype=torch.float32, device=index.device)  # interior groups: radius 0 below
        # 2. the boundary groups' local pass first: their exact radii (interior leaves 0)
        #    are what the other ranks filter their points with
        E.query(index, cfg, hint2, stats=stats, final_out=final_out, out=d2, groups=blist, ngroups=ng,
                ngroups_dev=bcnt, deferred=pend if gpu else None, short_list=True)
        radii = K.tree_set_radii(index.nodes.clone(), n, d2)
        if gpu:
            ev_rad = torch.cuda.Event()
            ev_rad.record(comp)
        # 3. the interior groups (most of the work) ...
        if not gpu:
            recv = _halo_send(index, radii, comm, cfg, info, marks=False)
        E.query(index, cfg, hint2, stats=stats, final_out=final_out, out=d2, groups=ilist, ngroups=ng,
                ngroups_dev=icnt, deferred=pend if gpu else None)
        if gpu:
            ev_int = torch.cuda.Event()
            ev_int.record(comp)
    if gpu:
        if hook is not None:
            # independent work (SetStream: the next set's redistribution) beside the
            # interior pass (REDIST_UNDER_KNN, else after it); the halo exchange follows
            # the hook's collectives (one communicator: never two in flight)
            if not REDIST_UNDER_KNN:
                cur.wait_event(ev_int)
            st = hook(cur)
            if st is not None:
                side.wait_stream(st)
        # ... while the halo is filtered and exchanged on the side stream
        side.wait_event(ev_rad)
        with torch.cuda.stream(side):
            recv = _halo_send(index, radii, comm, cfg, info, marks=False)
        cur.wait_stream(comp)
        cur.wait_stream(side)
        recv.record_stream(cur)
        d2.record_stream(cur)
        # (the group lists: a failure-list overflow reruns the exact kernel on `cur` inside
        # E.settle, reading them)
        for t in (blist, ilist, bcnt, icnt):
            t.record_stream(cur)
        final_out.record_stream(comp)
        radii.record_stream(side)
        E.settle(pend)
        info.counts["halo_overlap"] = 1
    info.counts["boundary_groups"] = int(bcnt.view(-1)[0])
    info.timer.mark("knn_local+halo_exchange")
    K.tree_set_radii(index.nodes, index.n, d2)
    return _halo_requery(index, d2, recv, cfg, hint2, info, final_out)


# --------------------------------------------------------------------------- entrypoints
# Single-rank runs can let the k-NN kernel write the distances straight into pinned host
# memory (random 4-byte PCIe writes at perm[q], hidden under the kernel) instead of a
# device buffer + copy. The writes sustain ~0.9-1e9 points/s: they hide under the bucket-
# tree kernel only when it is slow enough per point, i.e. from k ~ 48 (the cell-grid
# kernel is faster than the writes at k = 100: local_query keeps its output on the device) (1e8 uniform points on one
# MI355X, step ms copy/direct: k=16 118/172, k=48 141/135, k=64 151/145, k=100
# 176/170; 1e7 k=16 12.5/17.9; profiles/archive/r1_v20/direct_out_ab.txt).
DIRECT_OUT_MIN_K = 48


def direct_host_out_pays(k: int) -> bool:
    return k >= DIRECT_OUT_MIN_K


def _check_out(out: torch.Tensor | None, n: int, points: torch.Tensor) -> torch.Tensor:
    """Output buffer of a single-rank run: given (device tensor, or pinned host memory the
    kernel writes over PCIe) or a new device tensor."""
    if out is None:
        return torch.empty(n, dtype=torch.float32, device=points.device)
    if out.shape != (n,) or out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("out must be a contiguous float32 tensor with one entry per point")
    if points.device.type == "cuda" and out.device.type == "cpu" and not out.is_pinned():
        raise ValueError("a host output buffer for a GPU run must be pinned")
    if points.device.type == "cpu" and out.device.type != "cpu":
        raise ValueError("a CPU run needs a CPU output buffer")
    return out



# (Splitting a pass into several launches so that high-priority streams' kernels get CU
# slots at the kernel boundaries was measured and dropped: no change at 1e8 with 8
# hardware queues, profiles/r4_s1/fd_c4, fd_c8.)
# The next set's redistribution (SetStream's hook) is ordered after what precedes the local
# k-NN launch, so it runs beside the k-NN once its upload has landed (forced 1-rank RCCL
# 1e8 stream with 8 hardware queues: 997.4 vs 980.5 Mpts/s ordered after the k-NN;
# with 4 shared queues it had measured slower, profiles/r4_s1/fd_o_*.log); 0: after the
# k-NN (env LSKNN_REDIST_UNDER_KNN)
REDIST_UNDER_KNN = os.environ.get("LSKNN_REDIST_UNDER_KNN", "1") == "1"

# A 1-rank group (forced multi-rank runs) has no peer, hence no halo: knn_with_halo skips
# the publish / filter / exchange / re-query. True: run them anyway (the RCCL call-site
# tests exercise the halo collectives on one GPU with it).
HALO_ONE_RANK = os.environ.get("LSKNN_HALO_ONE_RANK", "0") == "1"

# tests: streamed redistribution also for device-resident input (env LSKNN_FORCE_STREAM=1)
FORCE_STREAM = os.environ.get("LSKNN_FORCE_STREAM", "0") == "1"

def local_build(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig, n_total: int,
                info: RunInfo | None = None, pre: tuple | None = None) -> tuple[E.LocalIndex, float | torch.Tensor]:
    """Single-rank first half: points (host or device) -> device, bounds, radius hint,
    Hilbert-sorted bucket tree. Everything is enqueued on the current stream; the one host
    sync is the over-full-cell check after the sort (see knn_engine.refine_heavy_cells),
    which waits for this stream only — so a caller can build the next point set on a side
    stream while the current set's k-NN runs (bench.py --pipeline). `pre` = (box, curve
    keys) of these device points computed already (SetStream PRE_KEYS)."""
    info = info or RunInfo(PhaseTimer(False, comm.device))
    dev = comm.device
    n_local = points.shape[0]
    if pre is not None:
        box, keys = pre[0], (pre[1], None)
    else:
        points = points.to(dev, non_blocking=True) if points.device != dev else points
        box, keys = global_box(points, comm), None
    hint2 = E.radius_hint(box, n_total, cfg.k)
    info.timer.mark("bounds")
    info.counts["owned_points"] = n_local
    # a flat set in any orientation: the index in its principal-axes frame (eager runs only:
    # flat_frame reads a 3x3 covariance; never in a stream of sets or a graph capture)
    probe = E.FrameProbe(points, cfg.k) if pre is None and not comm.distributed and n_local == n_total else None
    frame = probe.result() if probe is not None else None
    if frame is not None:  # a tilted plane: indexed in its principal-axes frame
        index = E.build_index(points, frame=frame)
    else:
        index = E.build_index(points, box, keys=keys, grid=True, density_n=n_total)
    info.timer.mark("build")
    return index, hint2


def query_into(index: E.LocalIndex, hint2, cfg: E.KnnConfig, info: RunInfo, out: torch.Tensor,
               direct: bool | None = None, deferred: list | None = None) -> torch.Tensor:
    """The k-NN kernel writes the final distances in input order (fused scatter). `out`
    in pinned host memory: direct=True — the kernel writes it over PCIe while it runs;
    False — a device buffer, then one 4 B/point copy (returned is `out` either way);
    None — False when the index has a cell grid (the grid kernel outruns the random 4-byte
    PCIe writes: 1B uniform, k=100, 1321 ms direct vs ~950 ms for the kernel alone), for a
    deferred failure check (the caller copies after it) and below k = 48 (the bucket-tree
    kernel hides the writes only from there: direct_host_out_pays), else True."""
    stats = info.stats if cfg.collect_stats else None
    host = out.device.type == "cpu" and index.pts.device.type == "cuda"
    if host and direct is None:
        direct = index.grid is None and deferred is None and direct_host_out_pays(cfg.k)
    if host and not direct:
        dev_out = torch.empty(index.n, dtype=torch.float32, device=index.device)
        E.query(index, cfg, hint2, stats=stats, final_out=dev_out, deferred=deferred)
        if deferred is not None:
            return dev_out  # the caller copies it once the failure check has run
        out.copy_(dev_out, non_blocking=True)
        return out
    E.query(index, cfg, hint2, stats=stats, final_out=out, deferred=deferred)
    return out


def local_query(index: E.LocalIndex, hint2, cfg: E.KnnConfig, info: RunInfo | None = None,
                out: torch.Tensor | None = None, deferred: list | None = None,
                direct: bool | None = None) -> torch.Tensor:
    """Single-rank second half: the k-NN kernel writes the final distances in input order
    (fused scatter) into `out` (see unordered_knn; direct: query_into). `deferred`: as in
    knn_engine.query; a pinned host `out` then comes back as a device result unless
    direct=True (SetStream copies it after the check)."""
    info = info or RunInfo(PhaseTimer(False, index.device))
    out = _check_out(out, index.n, index.pts)
    out = query_into(index, hint2, cfg, info, out, direct=direct, deferred=deferred)
    info.timer.mark("knn_local")
    return out


def unordered_knn(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig, info: RunInfo | None = None,
                  n_total: int | None = None, out: torch.Tensor | None = None,
                  direct: bool | None = None) -> torch.Tensor:
    """k-th-NN distance of every local point (input order) for a globally unordered set
    block-partitioned over ranks (reference unorderedData variant).

    `points` may live in (pinned) host memory: on several ranks the redistribution then
    streams them to the device in chunks overlapped with the exchange
    (redistribute_stream); on one rank they are copied first.
    `out` (optional, float32 [n_local]): where the distances go. On one rank a pinned host
    `out` is written by the k-NN kernel over PCIe while it runs, or through a device buffer
    and one copy (`direct`, see query_into: by default the copy when the cell grid is
    built, the direct writes for the bucket-tree kernel)."""
    info = info or RunInfo(PhaseTimer(False, comm.device))
    info.timer.start()
    points = points.contiguous()
    n_local = points.shape[0]
    if n_total is None:
        t = torch.tensor([n_local], dtype=torch.int64, device=comm.device)
        comm.allreduce_(t, "sum")
        n_total = int(t.item())
    streamed = comm.distributed and (points.device != comm.device or FORCE_STREAM)
    dev = comm.device
    if not comm.distributed:
        index, hint2 = local_build(points, comm, cfg, n_total, info)
        return local_query(index, hint2, cfg, info, out, direct=direct)
    if not streamed:
        return compute_set(redistribute_set(points, comm, cfg, n_total, info), comm, cfg, info, out=out)
    R = redistribute_stream(points, comm, info)
    box, owned = R.box, R.owned
    hint2 = E.radius_hint(box, n_total, cfg.k)
    index = E.build_index(owned, box, grid=True, density_n=n_total)
    info.timer.mark("build")
    # final distances in received-row order straight from the kernels (fused scatter);
    # the sorted d2 feeds the halo radii and the re-query bounds
    dist_owned = torch.empty(index.n, dtype=torch.float32, device=dev)
    knn_with_halo(index, comm, cfg, hint2, info, dist_owned)
    res = torch.empty(n_local, dtype=torch.float32, device=dev)
    if streamed and out is not None and out.device.type == "cpu" and res.device.type == "cuda" \
            and RETURN_GROUPS > 1 and len(R.spans) > 1:
        _return_grouped(R, dist_owned, comm, res, out)
        info.timer.mark("return")
        return out
    # counts of the return are known from the send side: no count exchange
    back, _ = comm.alltoallv(dist_owned[R.ret_index], R.ret_counts, recv_counts=R.back_counts)
    K.scatter1(back, R.origin_index.to(torch.int32), res, finalize=False)
    info.timer.mark("return")
    if out is not None:
        out.copy_(res, non_blocking=True)
        return out
    return res


@dataclass
class Redistributed:
    """A point set after its spatial redistribution (non-streamed multi-rank path)."""
    n_local: int                 # this rank's input points
    box: torch.Tensor            # global box
    hint2: object                # radius hint (device tensor or float)
    owned: torch.Tensor          # [m, 3] points this rank owns (received-row order)
    recv_counts: list
    send_perm: torch.Tensor      # local input row of each sent row
    send_counts: list
    n_total: int | None = None         # points of the whole set (grid level of the global box)


def redistribute_set(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig, n_total: int,
                     info: RunInfo | None = None) -> Redistributed:
    """First half of the multi-rank unordered pipeline on device-resident points: global
    bounds, splitters, all-to-all-v of every point to its spatial owner. Everything is
    queued on the current stream (collectives included)."""
    info = info or RunInfo(PhaseTimer(False, comm.device))
    points = points.contiguous()
    if points.device != comm.device:
        points = points.to(comm.device, non_blocking=True)
    box = global_box(points, comm)
    hint2 = E.radius_hint(box, n_total, cfg.k)
    info.timer.mark("bounds")
    owned, recv_counts, send_perm, send_counts = redistribute(points, comm, box, info)
    return Redistributed(int(points.shape[0]), box, hint2, owned, recv_counts, send_perm, send_counts,
                         n_total=n_total)


def compute_set(P: Redistributed, comm: Comm, cfg: E.KnnConfig, info: RunInfo | None = None,
                out: torch.Tensor | None = None, hook=None) -> torch.Tensor:
    """Second half: bucket tree of the owned points, local k-NN + halo exchange + re-query,
    distances back to their origin ranks in input order (into `out` if given). `hook`:
    see knn_with_halo; it returns the stream its collectives ran on, and the result
    return is ordered after it (one communicator: no concurrent collectives)."""
    info = info or RunInfo(PhaseTimer(False, comm.device))
    dev = comm.device
    index = E.build_index(P.owned, P.box, grid=True, density_n=P.n_total)
    info.timer.mark("build")
    dist_owned = torch.empty(index.n, dtype=torch.float32, device=dev)
    used: list = []
    def _hook(after):
        st = hook(after)
        used.append(st)
        return st

    knn_with_halo(index, comm, cfg, P.hint2, info, dist_owned, hook=_hook if hook is not None else None)
    if hook is not None and not used:  # (a path without the overlap point: run it here)
        used.append(hook(torch.cuda.current_stream(dev)) if K.is_gpu(dist_owned) else hook(None))
    for st in used:
        if st is not None:
            torch.cuda.current_stream(dev).wait_stream(st)
    res = torch.empty(P.n_local, dtype=torch.float32, device=dev)
    back, _ = comm.alltoallv(dist_owned, P.recv_counts, recv_counts=P.send_counts)
    K.scatter1(back, P.send_perm, res, finalize=False)
    info.timer.mark("return")
    if out is not None:
        out.copy_(res, non_blocking=True)
        return out
    return res


IMBALANCE_LIMIT = 1.2  # --balance auto: rebalance when max/mean points per rank exceeds it


def prepartitioned_knn(points: torch.Tensor, comm: Comm, cfg: E.KnnConfig,
                       info: RunInfo | None = None, out: torch.Tensor | None = None,
                       balance: str = "auto", direct: bool | None = None) -> torch.Tensor:
    """k-th-NN distance of every local point (input order) when each rank holds one
    (spatially coherent) input file (reference prePartitionedData variant). `out` as in
    unordered_knn (on one rank a pinned host tensor is written by the kernel directly).

    Skewed file sets: the reference serves a hot rank's whole shard to
    every requester (prePartitionedDataVariant.cu:337-344) and its own queries stay on
    it. With balance="on" — or "auto" when max/mean points per rank > IMBALANCE_LIMIT —
    the files go through the unordered pipeline instead (count-balanced spatial
    redistribution, halo, return): every rank owns ~N/P points and each file's results
    still come back in its own order."""
    if balance not in ("auto", "on", "off"):
        raise ValueError(f"balance must be auto, on or off, not {balance!r}")
    info = info or RunInfo(PhaseTimer(False, points.device))
    info.timer.start()
    points = points.contiguous()
    n_local = points.shape[0]
    if not comm.distributed:
        n_total = n_local
    else:
        counts = comm.allgather(torch.tensor([n_local], dtype=torch.int64, device=comm.device)).view(-1).cpu()
        n_total = int(counts.sum())
        ratio = float(counts.max()) * comm.size / max(n_total, 1)
        info.counts["imbalance_x1000"] = int(round(ratio * 1000))
        if balance == "on" or (balance == "auto" and ratio > IMBALANCE_LIMIT):
            info.counts["rebalanced"] = 1
            return unordered_knn(points, comm, cfg, info, n_total=n_total, out=out)
    box = K.bounds(points)
    gbox = global_box(points, comm) if comm.distributed else box
    hint2 = E.radius_hint(gbox, n_total, cfg.k)
    info.timer.mark("bounds")
    index = E.build_index(points, box, grid=True)
    info.counts["owned_points"] = n_local
    info.timer.mark("build")
    if not comm.distributed:  # fused scatter: final distances straight from the k-NN kernel
        out = _check_out(out, n_local, points)
        out = query_into(index, hint2, cfg, info, out, direct=direct)
        info.timer.mark("knn_local")
        return out
    res = torch.empty(n_local, dtype=torch.float32, device=points.device)
    knn_with_halo(index, comm, cfg, hint2, info, res)
    info.timer.mark("return")
    if out is not None:
        out.copy_(res, non_blocking=True)
        return out
    return res
