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
  third stream under set i+1 (kept alive with record_stream).

Every set is still uploaded, redistributed (several ranks), built, queried and returned in
full; only the order in which independent work is issued changes. On a CPU device the sets
run one after the other (same results; used by the CPU tests).

Measured on one MI355X (1B uniform, k=100, two alternating sets): 1414 ms per set
(707.3 Mpts/s) vs 1573 ms (635.8) one set at a time; forced 1-rank RCCL group at 1e8:
683 vs 599 Mpts/s (profiles/r2_s3_pipe, profiles/r2_s3_d2h).
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch

from ..models import knn_engine as E
from ..utils import trace
from . import pipelines as PL
from .comm import Comm


class SetStream:
    """Runs `unordered_knn` over a sequence of host point sets with the transfers of
    neighbouring sets overlapped (see module doc).

    comm / cfg: as for pipelines.unordered_knn. direct_out (one rank): the kernel writes
    the distances into the pinned host outputs itself (pipelines.direct_host_out_pays).
    """

    def __init__(self, comm: Comm, cfg: E.KnnConfig, direct_out: bool = True):
        self.comm = comm
        self.cfg = cfg
        self.device = comm.device
        self.gpu = self.device.type == "cuda"
        self.direct_out = bool(direct_out) and not comm.distributed
        if self.gpu:
            self.copy_stream = torch.cuda.Stream(self.device)
            self.out_stream = torch.cuda.Stream(self.device)
            # high priority: its kernels get CU slots as the k-NN grid's workgroups retire
            self.redist_stream = torch.cuda.Stream(self.device, priority=torch.cuda.Stream.priority_range()[1])
        self._dbuf: list[torch.Tensor | None] = [None, None]
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
        if not self.gpu:
            for i in range(n):
                info = new_info()
                out = PL.unordered_knn(inputs[i], self.comm, self.cfg, info, n_total=n_totals[i])
                outputs[i].copy_(out)
                self.last_info = info
                done(i)
            return
        if self.comm.distributed:
            return self._run_distributed(inputs, outputs, n_totals, new_info, done)
        cur = torch.cuda.current_stream(self.device)
        if n:
            self._prefetch(0, inputs[0])
        # no host sync between sets: set i+1's build is queued right behind set i's k-NN
        # (the stream orders them), and set i's failure-word read (a host sync, see
        # knn_engine.query `deferred`) waits until set i+1's work is queued
        pend: list = []
        fin: list = []  # (set, event after which its output is in host memory)
        for i in range(n):
            cur.wait_stream(self.copy_stream)  # set i's points are on the device
            pts = self._dbuf[i % 2]
            if i + 1 < n:
                self._prefetch(i + 1, inputs[i + 1])
            info = new_info()
            with trace.range(f"lsknn:set {i}"):
                info.timer.start()
                index, hint2 = PL.local_build(pts, self.comm, self.cfg, n_totals[i] or pts.shape[0], info)
                E.settle(pend)  # set i-1's failure word: its k-NN ran before this build
                direct = self.direct_out
                res = PL.local_query(index, hint2, self.cfg, info, outputs[i] if direct else None,
                                     deferred=pend)
                ev = torch.cuda.Event()
                if res.data_ptr() != outputs[i].data_ptr():
                    # device results: their copy to host runs on a side stream under the
                    # next set's build and k-NN
                    self.out_stream.wait_stream(cur)
                    with torch.cuda.stream(self.out_stream):
                        outputs[i].copy_(res, non_blocking=True)
                        ev.record(self.out_stream)
                    res.record_stream(self.out_stream)
                else:
                    ev.record(cur)
                del res, index
            self.last_info = info
            fin.append((i, ev))
            while len(fin) > 1:  # set i-1 (queued before set i's work) is retired
                j, e = fin.pop(0)
                e.synchronize()
                done(j)
        E.settle(pend)
        torch.cuda.synchronize(self.device)  # the last results are in host memory
        for j, _ in fin:
            done(j)

    def _run_distributed(self, inputs, outputs, n_totals, new_info, done) -> None:
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
        fin: list = []
        self._prefetch(0, inputs[0])
        cur.wait_stream(self.copy_stream)
        P = PL.redistribute_set(self._dbuf[0], comm, cfg, n_totals[0], new_info())
        if n > 1:
            self._prefetch(1, inputs[1])
        for i in range(n):
            info = new_info()
            nxt: dict = {}

            def hook(after, j=i + 1):
                # set j's redistribution under set i's k-NN (issued right after the k-NN
                # launch), once set j's points are on the device
                redist.wait_stream(after)
                redist.wait_stream(self.copy_stream)
                with torch.cuda.stream(redist):
                    nxt["P"] = PL.redistribute_set(self._dbuf[j % 2], comm, cfg, n_totals[j])
                return redist

            with trace.range(f"lsknn:set {i}"):
                res = PL.compute_set(P, comm, cfg, info, hook=hook if i + 1 < n else None)
            self.out_stream.wait_stream(cur)
            ev = torch.cuda.Event()
            with torch.cuda.stream(self.out_stream):
                outputs[i].copy_(res, non_blocking=True)
                ev.record(self.out_stream)
            res.record_stream(self.out_stream)  # kept until its copy is done
            del res
            cur.synchronize()
            redist.synchronize()
            if i + 2 < n:  # the buffer set i was redistributed from is free again
                self._prefetch(i + 2, inputs[i + 2])
            cur.wait_stream(redist)
            P = nxt.get("P")
            self.last_info = info
            fin.append((i, ev))
            while len(fin) > 1:  # set i-1's copy was queued before set i's
                j, e = fin.pop(0)
                e.synchronize()
                done(j)
        torch.cuda.synchronize(dev)  # the last results are in host memory
        for j, _ in fin:
            done(j)
