"""Communicator abstraction for the distributed pipelines.

The reference talks CUDA-aware MPI directly (MPIComm + CUKD_MPI_CALL,
unorderedDataVariant.cu:23-39; call-site inventory SURVEY §2.6). Here the pipelines
talk to a small interface with the four collectives the k-NN exchange needs:

* ``allreduce_(t, op)``      — in-place min / max / sum (bounds, histograms, flags)
* ``allgather(t)``           — equal-size gather (published halo trees, counts)
* ``alltoallv(send, counts)``— all-to-all-v of rows (spatial redistribution, halo
                               exchange, result return)
* ``barrier()``

Implementations:

* :class:`TorchComm` — one process per GPU over ``torch.distributed``; backend ``nccl``
  is RCCL on ROCm (xGMI peer-to-peer), ``gloo`` for CPU tensors / tests.
* :class:`LoopbackComm` — P virtual ranks as threads of one process sharing one device
  (SURVEY §4.2 T3): lets every multi-rank pipeline run on a single GPU or on CPU.
* :class:`SingleComm` — size 1.
"""
from __future__ import annotations

import math
import os
import threading
from typing import Sequence

import torch
import torch.distributed as dist


class Comm:
    rank: int = 0
    size: int = 1
    # True: run every collective through the backend even on a 1-rank group, and the
    # pipelines take their multi-rank path (tests: exercises each RCCL call site on one GPU)
    force: bool = False
    # collective / grouped point-to-point launches handed to the backend so far (bench.py
    # reports them per step: the control plane's cost on a real multi-GPU run)
    ncoll: int = 0

    def collectives(self) -> int:
        return self.ncoll

    @property
    def distributed(self) -> bool:
        """Multi-rank code path: more than one rank, or a forced 1-rank group."""
        return self.size > 1 or self.force

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """Returns a tensor of shape [size, *t.shape]."""
        raise NotImplementedError

    def alltoallv(self, send: torch.Tensor, send_counts: Sequence[int],
                  recv_counts: Sequence[int] | None = None) -> tuple[torch.Tensor, list[int]]:
        """Rows send[sum(counts[:j]) : sum(counts[:j+1])] go to rank j. Returns
        (recv rows ordered by source rank, recv counts per source). `recv_counts`, when the
        caller knows them (e.g. a result return), saves the count exchange."""
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    def p2p(self, sends: Sequence[tuple[int, torch.Tensor]],
            recvs: Sequence[tuple[int, tuple, torch.dtype]]) -> list[torch.Tensor]:
        """Grouped point-to-point exchange (the reference's Isend/Irecv/Waitall,
        unorderedDataVariant.cu:183-193, prePartitionedDataVariant.cu:326-345):
        sends = [(dst, tensor)], recvs = [(src, shape, dtype)] -> received tensors."""
        raise NotImplementedError

    # convenience -----------------------------------------------------------------
    def count_exchange(self, counts: torch.Tensor) -> tuple[list[int], list[int]]:
        """`counts` ([size] ints, device or host: this rank's rows for each rank) ->
        (send counts, recv counts) on the host, through one all-gather of the count
        vectors and ONE host read of the [size, size] matrix (the alternative, reading
        the local counts and then exchanging them, costs two host round trips)."""
        m = self.allgather(counts.reshape(-1).to(torch.int64)).cpu()
        return [int(x) for x in m[self.rank]], [int(x) for x in m[:, self.rank]]

    def exchange_counts(self, send_counts: Sequence[int]) -> list[int]:
        t = torch.tensor(list(send_counts), dtype=torch.int64)
        allc = self.allgather_host(t)
        return [int(allc[j, self.rank]) for j in range(self.size)]

    def allgather_host(self, t: torch.Tensor) -> torch.Tensor:
        """allgather of a small CPU tensor (moved to the comm device if needed)."""
        return self.allgather(t.to(self.device)).cpu()

    @property
    def device(self) -> torch.device:
        return torch.device("cpu")


class SingleComm(Comm):
    def __init__(self, device: torch.device | str = "cpu"):
        self.rank, self.size = 0, 1
        self._device = torch.device(device)

    @property
    def device(self) -> torch.device:
        return self._device

    def allreduce_(self, t, op="sum"):
        return t

    def allgather(self, t):
        return t.unsqueeze(0).clone()

    def alltoallv(self, send, send_counts, recv_counts=None):
        return send.clone(), [int(send_counts[0])]

    def barrier(self):
        pass

    def p2p(self, sends, recvs):
        box = {dst: t for dst, t in sends}
        return [box[src].clone() for src, _, _ in recvs]


_OPS = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}

# Largest single point-to-point message handed to the backend. RCCL 2.26 (torch 2.10's
# librccl) corrupts the second half of any send/recv above 1 GiB (measured on MI355X with
# a 1-rank group: 1024 MiB exact, 1025 MiB wrong from byte 2^29 on; all_to_all_single and
# batch_isend_irecv alike; profiles/archive/r2_rccl/README.txt). At 1B points on 2 ranks the
# redistribution sends ~3 GB to the peer, so every larger message is split into rounds of
# at most this many bytes per peer.
MAX_MSG_BYTES = int(os.environ.get("LSKNN_MAX_MSG_MB", "256")) << 20


class TorchComm(Comm):
    """torch.distributed process group (RCCL for GPU tensors, gloo for CPU).

    A gloo group with GPU-resident data (several processes sharing one GPU: RCCL refuses
    two ranks on one device) stages every collective through host memory, so the whole
    multi-process GPU pipeline can run on a one-GPU box (tests/test_gpu_multiprocess.py)."""

    def __init__(self, device: torch.device | str, group=None, force: bool = False):
        self.group = group
        self.force = bool(force)
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self._device = torch.device(device)
        self.backend = dist.get_backend(group)
        self.staged = self.backend == "gloo" and self._device.type != "cpu"
        self.max_msg_bytes = MAX_MSG_BYTES

    @property
    def device(self) -> torch.device:
        return self._device

    def allreduce_(self, t, op="sum"):
        if self.distributed:
            self.ncoll += 1
            if self.staged and t.device.type != "cpu":
                h = t.cpu()
                dist.all_reduce(h, op=_OPS[op], group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=_OPS[op], group=self.group)
        return t

    def allgather(self, t):
        t = t.contiguous()
        if self.staged and t.device.type != "cpu" and self.distributed:
            self.ncoll += 1
            return self._gather_gloo(t.cpu()).to(t.device)
        if not self.distributed:
            out = torch.empty((self.size, *t.shape), dtype=t.dtype, device=t.device)
            out[0].copy_(t)
            return out
        self.ncoll += 1
        if self.backend == "gloo":
            return self._gather_gloo(t)
        out = torch.empty((self.size, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def _gather_gloo(self, t):
        out = torch.empty((self.size, *t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather(list(out.unbind(0)), t, group=self.group)
        return out

    def alltoallv(self, send, send_counts, recv_counts=None):
        send_counts = [int(c) for c in send_counts]
        recv_counts = (self.exchange_counts(send_counts) if recv_counts is None
                       else [int(c) for c in recv_counts])
        row_shape = tuple(send.shape[1:])
        if not self.distributed:
            return send.clone(), recv_counts
        dev = send.device
        staged = self.staged and dev.type != "cpu"
        src = send.cpu() if staged else send.contiguous()
        recv = torch.empty((sum(recv_counts), *row_shape), dtype=send.dtype, device=src.device)
        # grouped send/recv (the all-to-all-v RCCL itself runs: ncclSend/ncclRecv per peer in
        # one group), every message cut into pieces of at most max_msg_bytes. Both ends of a
        # pair know that message's size, so the pieces match pair by pair with no agreement
        # on a global collective form first (no extra all-reduce or host sync per exchange)
        so, ro = _offsets(send_counts), _offsets(recv_counts)
        sends = [(j, src[so[j]:so[j + 1]]) for j in range(self.size)]
        recvs = [(j, recv[ro[j]:ro[j + 1]]) for j in range(self.size)]
        self._p2p_rounds(sends, recvs)
        return (recv.to(dev) if staged else recv), recv_counts

    def _p2p_rounds(self, sends, recvs):
        """Grouped send/recv of contiguous tensors, every message cut into pieces of at
        most max_msg_bytes: round r carries piece r of every pair (both ends know each
        message's size, so the pieces match pair by pair in posting order). Own-rank
        pairs are a local copy unless the group is forced (then RCCL carries them too)."""
        cap = max(1, self.max_msg_bytes)
        via_backend = self.force and self.backend == "nccl"  # own-rank pairs through RCCL

        def pieces(t):
            b = t.reshape(-1).view(torch.uint8)
            return [b[o:o + cap] for o in range(0, b.numel(), cap)]

        own = {}
        ps, pr = [], []
        for j, t in sends:
            if j == self.rank and not via_backend:
                own[j] = t
            elif t.numel():
                ps.append((j, pieces(t)))
        for j, t in recvs:
            if j == self.rank and not via_backend:
                if t.numel():
                    t.copy_(own[j])
            elif t.numel():
                pr.append((j, pieces(t)))
        rounds = max([len(p) for _, p in ps + pr] + [0])
        for r in range(rounds):
            ops = [dist.P2POp(dist.isend, p[r], j, group=self.group) for j, p in ps if r < len(p)]
            ops += [dist.P2POp(dist.irecv, p[r], j, group=self.group) for j, p in pr if r < len(p)]
            if ops:
                self.ncoll += 1
                for req in dist.batch_isend_irecv(ops):
                    req.wait()

    def p2p(self, sends, recvs):
        staged = self.staged
        bufdev = torch.device("cpu") if staged else self._device
        out = [torch.empty(shape, dtype=dt, device=bufdev) for _, shape, dt in recvs]
        # own-rank traffic is a local copy, except on a forced group where it goes through
        # the backend as well (RCCL send/recv to self inside the group); messages above
        # max_msg_bytes travel in pieces (_p2p_rounds)
        self._p2p_rounds([(dst, (t.cpu() if staged else t.contiguous())) for dst, t in sends],
                         list(zip([src for src, _, _ in recvs], out)))
        return [b.to(self._device) for b in out] if staged else out

    def barrier(self):
        if self.distributed:
            self.ncoll += 1
            if self.backend == "nccl":
                # device barrier via a 1-element all-reduce keeps RCCL the only channel
                t = torch.zeros(1, device=self._device)
                dist.all_reduce(t, group=self.group)
                torch.cuda.synchronize(self._device)
            else:
                if self._device.type == "cuda":
                    torch.cuda.synchronize(self._device)
                dist.barrier(group=self.group)


def _offsets(counts):
    o = [0]
    for c in counts:
        o.append(o[-1] + int(c))
    return o


class _Hub:
    def __init__(self, size: int):
        self.size = size
        self.barrier = threading.Barrier(size)
        self.slots: list = [None] * size


class LoopbackComm(Comm):
    """P virtual ranks as threads of one process (tests; one GPU or CPU)."""

    def __init__(self, hub: _Hub, rank: int, device: torch.device | str):
        self.hub = hub
        self.rank = rank
        self.size = hub.size
        self._device = torch.device(device)

    @staticmethod
    def create(size: int, device: torch.device | str = "cpu") -> list["LoopbackComm"]:
        hub = _Hub(size)
        return [LoopbackComm(hub, r, device) for r in range(size)]

    @property
    def device(self) -> torch.device:
        return self._device

    def _sync_device(self):
        if self._device.type == "cuda":
            torch.cuda.current_stream(self._device).synchronize()

    def _share(self, obj):
        self.ncoll += 1
        self._sync_device()
        self.hub.slots[self.rank] = obj
        self.hub.barrier.wait()
        allv = list(self.hub.slots)
        self.hub.barrier.wait()
        return allv

    def allreduce_(self, t, op="sum"):
        allv = self._share(t.clone())
        acc = allv[0].clone()
        for v in allv[1:]:
            v = v.to(acc.device)
            if op == "sum":
                acc += v
            elif op == "min":
                acc = torch.minimum(acc, v)
            else:
                acc = torch.maximum(acc, v)
        t.copy_(acc)
        self._sync_device()
        return t

    def allgather(self, t):
        allv = self._share(t.clone())
        out = torch.stack([v.to(t.device) for v in allv])
        self._sync_device()
        return out

    def alltoallv(self, send, send_counts, recv_counts=None):
        send_counts = [int(c) for c in send_counts]
        offs = [0]
        for c in send_counts:
            offs.append(offs[-1] + c)
        allv = self._share((send.clone(), offs))
        parts, counts = [], []
        for src in range(self.size):
            s, o = allv[src]
            parts.append(s[o[self.rank]:o[self.rank + 1]].to(send.device))
            counts.append(o[self.rank + 1] - o[self.rank])
        recv = torch.cat(parts) if parts else send[:0].clone()
        self._sync_device()
        return recv, counts

    def barrier(self):
        self.ncoll += 1
        self._sync_device()
        self.hub.barrier.wait()

    def p2p(self, sends, recvs):
        allv = self._share({dst: t.clone() for dst, t in sends})
        out = [allv[src][self.rank].to(self._device) for src, _, _ in recvs]
        self._sync_device()
        return out


def run_loopback(size: int, fn, device: torch.device | str = "cpu"):
    """Run fn(comm) on `size` virtual ranks (threads); returns the per-rank results."""
    comms = LoopbackComm.create(size, device)
    results: list = [None] * size
    errors: list = [None] * size

    def worker(r):
        try:
            if torch.device(device).type == "cuda":
                torch.cuda.set_device(torch.device(device))
            results[r] = fn(comms[r])
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e
            comms[r].hub.barrier.abort()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(size)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errors:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errors:
        if e is not None:
            raise e
    return results
