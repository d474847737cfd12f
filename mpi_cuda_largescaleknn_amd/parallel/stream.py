"""A stream of point sets through the unordered k-th-NN pipeline (serving many sets).

Serving sets one after the other leaves PCIe idle while the GPU computes and the GPU idle
while PCIe copies: a 1B-point set is a 12 GB host-to-device copy (~210 ms at ~57 GB/s)
before ~1.4 s of index build and k-NN. `SetStream` overlaps them across sets:

* set i+1's points are copied host -> device on a copy stream while set i is built and
  queried on the compute stream (PCIe H2D runs on the DMA engines; the k-NN kernel is
  VALU-bound and does not notice it). Two device input buffers alternate; the copy into
  one waits for the set that last read it;
* one rank: the k-NN kernel writes set i's distances straight into its pinned host
  output while it runs (pipelines.local_query), nothing to copy afterwards;
* several ranks: set i+1's spatial redistribution (bounds, splitters, all-to-all-v of
  the points) is issued on a fourth, high-priority stream right after set i's local k-NN
  is queued, so it runs under set i's k-NN (pipelines.compute_set hook; set i's halo
  exchange and result return are ordered after its collectives, one communicator never
  has two collectives in flight); set i's returned distances go device -> host on a
  third stream, queued from set i+1's hook so the copy runs under set i+1's k-NN (kept
  alive with record_stream). No host sync between sets (events order the input-buffer
  reuse), and no host read inside an index build (knn_engine.host_sync_free).

Every set is still uploaded, redistributed (several ranks), built, queried and returned in
full; only the order in which independent work is issued changes. On a CPU device the sets
run one after the other (same results; used by the CPU tests).

Measured on one MI355X (1B uniform, k=100, two alternating sets): 1414 ms per set
(707.3 Mpts/s) vs 1573 ms (635.8) one set at a time; forced 1-rank RCCL group at 1e8:
683 vs 599 Mpts/s (profiles/archive/r2_s3_pipe, profiles/archive/r2_s3_d2h).
"""
from __future__ import annotations

import os
from typing import Callable, Sequence

import torch

from ..models import knn_engine as E
from ..ops import kernels as K
from ..utils import trace
from . import pipelines as PL
from .comm import Comm


# Measured and dropped (rounds 3-4; the A/Bs stay in profiles/): building set i+1's index
# on a side stream under set i's k-NN (1B k=100: 1168 vs 1106 ms per set — the build's
# workgroups hold CU slots among the k-NN's far longer than the build takes alone), and
# queueing set i-1's result copy behind set i's build instead of beside it
# (profiles/r4_final/README.md).
# One rank: set i+1's bounds and curve keys (two short memory-bound passes) are computed on
# the high-priority side stream beside set i's k-NN, once set i+1's upload has landed,
# instead of at the head of set i+1's build beside set i-1's result copy (env
# LSKNN_PRE_KEYS; 1 = on).
PRE_KEYS = os.environ.get("LSKNN_PRE_KEYS", "1") == "1"


def _index_tensors(index: E.LocalIndex):
    yield from (index.pts, index.perm, index.nodes, index.qnodes, index.box)
    if index.grid is not None:
        yield index.grid.slots


class SetStream:
    """Runs `unordered_knn` over a sequence of host point sets with the transfers of
    neighbouring sets overlapped (see module doc).

    comm / cfg: as for pipelines.unordered_knn. direct_out (one rank): the kernel writes
    the distances into the pinned host outputs itself (pipelines.query_into).
    variant: "unordered" (block-partitioned sets, spatially redistributed on several
    ranks) or "prepartitioned" (each rank's set is its own file: on one rank the same
    pipeline; on several, pipelines.prepartitioned_knn per set with the uploads and result
    copies overlapped).
    """

    def __init__(self, comm: Comm, cfg: E.KnnConfig, direct_out: bool = True,
                 variant: str = "unordered", pre_keys: bool | None = None):
        if variant not in ("unordered", "prepartitioned"):
            raise ValueError(f"SetStream: variant must be unordered or prepartitioned, not {variant!r}")
        self.comm = comm
        self.cfg = cfg
        self.variant = variant
        self.device = comm.device
        self.gpu = self.device.type == "cuda"
        self.direct_out = bool(direct_out) and not comm.distributed
        self.pre_keys = PRE_KEYS if pre_keys is None else bool(pre_keys)
        if self.gpu:
            self.copy_stream = torch.cuda.Stream(self.device)
            self.out_stream = torch.cuda.Stream(self.device)
            # high priority: its kernels get CU slots as the k-NN grid's workgroups retire
            self.redist_stream = torch.cuda.Stream(self.device, priority=torch.cuda.Stream.priority_range()[1])
        self._dbuf: list[torch.Tensor | None] = [None, None]
        self._copy_ev: dict = {}  # set index -> event right behind its upload
        self.last_info: PL.RunInfo | None = None

    def _buffer(self, slot: int, like: torch.Tensor) -> torch.Tensor:
        b = self._dbuf[slot]
        if b is None or b.shape != like.shape or b.dtype != like.dtype:
            b = torch.empty(like.shape, dtype=like.dtype, device=self.device)
            self._dbuf[slot] = b
        return b

    def _prefetch(self, j: int, host: torch.Tensor) -> None:
        # after everything issued so far on the compute stream (the set that last read
        # this buffer), copy on the copy stream
        self.copy_stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.copy_stream):
            self._buffer(j % 2, host).copy_(host, non_blocking=True)
        self._mark_copy(j)

    def _mark_copy(self, j: int) -> None:
        # an event right behind set j's upload: consumers wait for THAT, not for a marker
        # placed on the copy stream later — with 4 hardware queues per process the copy
        # stream shares one with the output stream, whose result copy (a blit kernel) gets
        # no CU slot while a k-NN grid is being dispatched, and a later marker would sit
        # behind it (the next set's redistribution then started only after the k-NN)
        ev = torch.cuda.Event()
        ev.record(self.copy_stream)
        self._copy_ev[j] = ev

    def _uploaded(self, stream, j: int) -> None:
        """`stream` waits for set j's upload."""
        ev = self._copy_ev.pop(j, None)
        if ev is not None:
            stream.wait_event(ev)
        else:
            stream.wait_stream(self.copy_stream)

    def run(self, inputs: Sequence[torch.Tensor], outputs: Sequence[torch.Tensor],
            n_totals: Sequence[int | None] | None = None,
            info_factory: Callable[[], PL.RunInfo] | None = None,
            on_done: Callable[[int], None] | None = None) -> None:
        """Set i: this rank's points inputs[i] (pinned host memory for GPU runs) ->
        distances in outputs[i] (float32, one per point, pinned for GPU runs). Returns
        when every output is in host memory. `n_totals[i]`: the set's global point count
        (None: summed over ranks).

        `inputs` / `outputs` are only indexed (in set order, a set or two ahead), so they
        may be lazy sequences that read / allocate on first access. `on_done(i)` is called
        once outputs[i] is complete in host memory and inputs[i] is no longer read — a
        caller can write the result and release both buffers there, so a long stream keeps
        only ~3 sets alive (apps/stream.py)."""
        n = len(inputs)
        if len(outputs) != n:
            raise ValueError("SetStream.run: one output per input")
        n_totals = list(n_totals) if n_totals is not None else [None] * n
        new_info = info_factory or (lambda: PL.RunInfo(PL.PhaseTimer(False, self.device)))
        done = on_done or (lambda i: None)
        if self.gpu:
            E.new_heavy_stream()  # an earlier stream's clean verdict says nothing about this one
            with E.host_sync_free():  # no host read inside a build (knn_engine.build_index)
                if self.comm.distributed and self.variant == "prepartitioned":
                    return self._run_prepartitioned(inputs, outputs, new_info, done)
                if self.comm.distributed:
                    return self._run_distributed(inputs, outputs, n_totals, new_info, done)
                return self._run_local(inputs, outputs, n_totals, new_info, done)
        for i in range(n):  # CPU: one set after the other
            info = new_info()
            if self.variant == "prepartitioned":
                out = PL.prepartitioned_knn(inputs[i], self.comm, self.cfg, info)
            else:
                out = PL.unordered_knn(inputs[i], self.comm, self.cfg, info, n_total=n_totals[i])
            outputs[i].copy_(out)
            self.last_info = info
            done(i)

    def _run_local(self, inputs, outputs, n_totals, new_info, done) -> None:
        n = len(inputs)
        cur = torch.cuda.current_stream(self.device)
        if n:
            self._prefetch(0, inputs[0])
        # no host sync between sets: set i+1's build is queued right behind set i's k-NN
        # (the stream orders them), and set i's failure-word read (a host sync on an event
        # right behind its k-NN, see knn_engine.query `deferred`) comes once set i+1's work
        # is queued; set i's output copy follows that check (a rerun rewrites the output)
        prev = None  # set i-1: see _query
        pre: dict = {}  # set index -> (box, keys, event) computed beside the previous k-NN
        for i in range(n):
            self._uploaded(cur, i)  # set i's points are on the device
            pts = self._dbuf[i % 2]
            if i + 1 < n:
                self._prefetch(i + 1, inputs[i + 1])
            info = new_info()
            pk = pre.pop(i, None)
            if pk is not None:
                cur.wait_event(pk[2])
            with trace.range(f"lsknn:set {i}"):
                info.timer.start()
                index, hint2 = PL.local_build(pts, self.comm, self.cfg, n_totals[i] or pts.shape[0], info,
                                              pre=pk[:2] if pk is not None else None)
                rel = self._release(prev, outputs) if prev is not None else None
                rec = self._query(i, index, hint2, info, outputs)
                del index
                if self.pre_keys and i + 1 < n:
                    pre[i + 1] = self._pre_keys(i + 1, cur)
            if rel is not None:  # set i-1's output, waited for once set i's k-NN is queued
                rel[1].synchronize()
                done(rel[0])
            self.last_info = info
            prev = rec
        if prev is not None:
            self._retire(prev, outputs, done)

    def _query(self, i, index, hint2, info, outputs):
        """Queue set i's k-NN (the kernel writes the pinned output itself when direct);
        returns (i, device result or None, event after the k-NN, its deferred failure
        checks)."""
        cur = torch.cuda.current_stream(self.device)
        pend: list = []
        res = PL.local_query(index, hint2, self.cfg, info, outputs[i] if self.direct_out else None,
                             deferred=pend, direct=True if self.direct_out else None)
        ev = torch.cuda.Event()
        ev.record(cur)
        return (i, None if res.data_ptr() == outputs[i].data_ptr() else res, ev, pend)

    def _retire(self, rec, outputs, done) -> None:
        j, ev = self._release(rec, outputs)
        ev.synchronize()
        done(j)

    def _release(self, rec, outputs, after=None):
        """Set j: its failure check (a 4-byte read behind its k-NN), then its device result
        to host on the output stream (behind its k-NN, or behind everything queued so far
        when the check queued a rerun). Returns (j, event after which outputs[j] is in
        host memory)."""
        j, res, ev, pend = rec
        cur = torch.cuda.current_stream(self.device)
        if E.settle(pend):
            ev = torch.cuda.Event()
            ev.record(cur)
        if res is not None:
            self.out_stream.wait_event(ev)
            if after is not None:
                self.out_stream.wait_event(after)
            with torch.cuda.stream(self.out_stream):
                outputs[j].copy_(res, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.out_stream)
            res.record_stream(self.out_stream)
        return j, ev

    def _pre_keys(self, j: int, cur):
        """Set j's box and curve keys on the side stream once its upload has landed (the
        upload event stays for the compute stream); -> (box, keys, event after them)."""
        s2 = self.redist_stream
        ev = self._copy_ev.get(j)
        if ev is not None:
            s2.wait_event(ev)
        else:
            s2.wait_stream(self.copy_stream)
        nxt = self._dbuf[j % 2]
        with torch.cuda.stream(s2):
            box = PL.global_box(nxt, self.comm)
            keys = K.morton(nxt, box, with_iota=False)[0]
            done = torch.cuda.Event()
            done.record(s2)
        box.record_stream(cur)
        keys.record_stream(cur)
        return box, keys, done

    def _prefetch_after(self, j: int, host: torch.Tensor, ev) -> None:
        # copy set j into its buffer once `ev` (the build that last read it) is done
        if ev is not None:
            self.copy_stream.wait_event(ev)
        with torch.cuda.stream(self.copy_stream):
            self._buffer(j % 2, host).copy_(host, non_blocking=True)
        self._mark_copy(j)

    def _run_prepartitioned(self, inputs, outputs, new_info, done) -> None:
        """Several ranks, one file per rank and set: set i+1's upload runs under set i
        (copy stream), set i's result copy under set i+1 (output stream, queued once set
        i+1's work is), no host sync between sets beyond the collectives' own."""
        n = len(inputs)
        cur = torch.cuda.current_stream(self.device)
        if n == 0:
            return
        self._prefetch(0, inputs[0])
        copies: list = []
        prev = None
        for i in range(n):
            self._uploaded(cur, i)  # set i's points are on the device
            pts = self._dbuf[i % 2]
            if i + 1 < n:
                self._prefetch(i + 1, inputs[i + 1])  # after set i-1's reads of that buffer
            info = new_info()
            with trace.range(f"lsknn:set {i}"):
                res = PL.prepartitioned_knn(pts, self.comm, self.cfg, info)
            ev = torch.cuda.Event()
            ev.record(cur)
            if prev is not None:
                j, r, e = prev
                self.out_stream.wait_event(e)
                with torch.cuda.stream(self.out_stream):
                    outputs[j].copy_(r, non_blocking=True)
                    ce = torch.cuda.Event()
                    ce.record(self.out_stream)
                r.record_stream(self.out_stream)
                copies.append((j, ce))
            prev = (i, res, ev)
            del res
            self.last_info = info
            while copies and copies[0][1].query():
                done(copies.pop(0)[0])
        j, r, e = prev
        with torch.cuda.stream(self.out_stream):
            self.out_stream.wait_event(e)
            outputs[j].copy_(r, non_blocking=True)
        self.out_stream.synchronize()
        for j, _ in copies:
            done(j)
        done(n - 1)

    def _run_distributed(self, inputs, outputs, n_totals, new_info, done) -> None:
        """Several ranks. Set i+1's redistribution runs under set i's k-NN (the compute_set
        hook), and set i-1's result goes to host memory on the output stream from the same
        hook, i.e. under set i's k-NN too (queued earlier, its PCIe writes slowed set i's
        index build). No host sync between sets: events order the buffer reuse, and the
        host only waits where a collective's sizes are needed."""
        comm, cfg, dev = self.comm, self.cfg, self.device
        cur = torch.cuda.current_stream(dev)
        redist = self.redist_stream
        n = len(inputs)
        for j in range(n):  # global point counts (one small all-reduce per unknown set)
            if n_totals[j] is None:
                t = torch.tensor([int(inputs[j].shape[0])], dtype=torch.int64, device=dev)
                comm.allreduce_(t, "sum")
                n_totals[j] = int(t.item())
        if n == 0:
            return
        red_ev: list = [None, None]  # event after the redistribution that read input buffer b
        self._prefetch(0, inputs[0])
        self._uploaded(cur, 0)
        P = PL.redistribute_set(self._dbuf[0], comm, cfg, n_totals[0], new_info())
        red_ev[0] = torch.cuda.Event()
        red_ev[0].record(cur)
        if n > 1:
            self._prefetch(1, inputs[1])
        pending: list = []  # [(j, device result, event after it)] not yet copied to host
        copies: list = []   # [(j, event after its copy to host)]

        def flush():
            # queue the pending results' copies to host (behind their own sets' work)
            while pending:
                j, res, ev = pending.pop(0)
                self.out_stream.wait_event(ev)
                with torch.cuda.stream(self.out_stream):
                    outputs[j].copy_(res, non_blocking=True)
                    e = torch.cuda.Event()
                    e.record(self.out_stream)
                res.record_stream(self.out_stream)  # kept until its copy is done
                copies.append((j, e))

        for i in range(n):
            info = new_info()
            nxt: dict = {}

            def hook(after, j=i + 1):
                flush()  # set i-1's result: its copy runs under set i's k-NN
                if j >= n:
                    return None
                # set j's redistribution under set i's k-NN (issued right after the k-NN
                # launch), once set j's points are on the device
                if isinstance(after, torch.cuda.Event):
                    redist.wait_event(after)  # (a 1-rank group: the k-NN runs on `cur`)
                else:
                    redist.wait_stream(after)
                self._uploaded(redist, j)
                with torch.cuda.stream(redist):
                    nxt["P"] = PL.redistribute_set(self._dbuf[j % 2], comm, cfg, n_totals[j])
                    e = torch.cuda.Event()
                    e.record(redist)
                red_ev[j % 2] = e
                return redist

            with trace.range(f"lsknn:set {i}"):
                res = PL.compute_set(P, comm, cfg, info, hook=hook)
            ev = torch.cuda.Event()
            ev.record(cur)
            pending.append((i, res, ev))
            del res
            if i + 2 < n:  # the buffer set i was redistributed from, once that is done
                self._prefetch_after(i + 2, inputs[i + 2], red_ev[i % 2])
            cur.wait_stream(redist)  # set i+1's points are redistributed (device-side wait)
            P = nxt.get("P")
            self.last_info = info
            while copies and copies[0][1].query():  # finished sets, without waiting
                done(copies.pop(0)[0])
        flush()
        for j, e in copies:
            e.synchronize()
            done(j)
