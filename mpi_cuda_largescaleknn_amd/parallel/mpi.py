"""Native MPI host communicator ("HostComm") on csrc/mpi/mpi_comm.cpp.

The reference is an MPI program end to end: MPI_Init, MPIComm, ring Isend/Irecv/Waitall
of device buffers, Allgather/Allreduce of the peer schedule and MPI_Barrier
(unorderedDataVariant.cu:30-39, 107, 183-193; prePartitionedDataVariant.cu:228-229,
318-345). It needs CUDA-aware MPI. The MPICH of this image (3.3.2, ch3:nemesis) is not
GPU-aware, so `MpiComm` stages GPU tensors through host memory, and the C++ library moves
host bytes with MPI:

* allreduce  -> MPI_Allreduce (in place; chunked below INT_MAX elements)
* allgather  -> MPI_Allgather (Isend/Irecv pieces above INT_MAX bytes)
* alltoallv  -> nonblocking Isend/Irecv of every (source, destination) block + Waitall
                (messages above `max_msg_bytes` in pieces: MPI counts are int)
* p2p        -> grouped Isend/Irecv + Waitall (the reference's rounds)
* barrier    -> MPI_Barrier

Use it with ``mpirun -n N bin/hipKNN_unorderedData ...`` and ``LSKNN_DIST_BACKEND=mpi``
(launch.init): rank and size then come from MPI_COMM_WORLD itself, rank 0 broadcasts a
free rendezvous port over MPI for the small gloo control group (key-value store,
watchdog, failure broadcast), and a failing rank ends the job with MPI_Abort — the
reference's failure behaviour. RCCL (`nccl`, `rccl`) stays the data path for GPU runs;
this backend is for hosts without RCCL peers (CPU runs, several ranks sharing one GPU,
debugging against the reference's transport).
"""
from __future__ import annotations

import ctypes as C
import math
import socket

import torch

from .. import _native
from .comm import MAX_MSG_BYTES, Comm, _offsets

_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float32: 7, torch.float64: 8}
_OPS = {"sum": 0, "max": 2, "min": 3}


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _native.mpi().lsk_mpi_last_error()
        raise _native.NativeError(f"{what} failed: {msg.decode() if msg else rc}")


def mpi_world() -> tuple[int, int]:
    """MPI_Init (once) -> (rank, size) in MPI_COMM_WORLD."""
    r, s = C.c_int(0), C.c_int(1)
    _check(_native.mpi().lsk_mpi_init(C.byref(r), C.byref(s)), "MPI_Init")
    return r.value, s.value


def bcast_port(rank: int) -> int:
    """Rank 0 picks a free TCP port on 127.0.0.1 and broadcasts it over MPI (the gloo
    control group's rendezvous; no fixed port to collide with another job)."""
    buf = (C.c_int32 * 1)(0)
    if rank == 0:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            buf[0] = s.getsockname()[1]
    _check(_native.mpi().lsk_mpi_bcast(buf, 4, 0), "MPI_Bcast")
    return int(buf[0])


def finalize() -> None:
    _check(_native.mpi().lsk_mpi_finalize(), "MPI_Finalize")


def abort(code: int = 1) -> None:
    _native.mpi().lsk_mpi_abort(int(code))


class MpiComm(Comm):
    """One rank of MPI_COMM_WORLD; GPU tensors are staged through host memory."""

    def __init__(self, device: torch.device | str, force: bool = False):
        self._device = torch.device(device)
        self.rank, self.size = mpi_world()
        self.force = bool(force)
        self.backend = "mpi"
        self.staged = self._device.type != "cpu"
        self.max_msg_bytes = MAX_MSG_BYTES

    @property
    def device(self) -> torch.device:
        return self._device

    def abort(self) -> None:
        abort(1)

    # ------------------------------------------------------------------ staging
    @staticmethod
    def _host(t: torch.Tensor) -> torch.Tensor:
        return t.contiguous() if t.device.type == "cpu" else t.cpu()

    # -------------------------------------------------------------- collectives
    def allreduce_(self, t, op="sum"):
        if not self.distributed:
            return t
        if t.dtype not in _DTYPES:
            raise TypeError(f"MpiComm.allreduce_: unsupported dtype {t.dtype}")
        h = self._host(t)
        self.ncoll += 1
        _check(_native.mpi().lsk_mpi_allreduce(h.data_ptr(), h.numel(), _DTYPES[h.dtype], _OPS[op]),
               "MPI_Allreduce")
        if h.data_ptr() != t.data_ptr():
            t.copy_(h)
        return t

    def allgather(self, t):
        h = self._host(t)
        out = torch.empty((self.size, *t.shape), dtype=t.dtype)
        if not self.distributed:
            out[0].copy_(h)
        else:
            self.ncoll += 1
            _check(_native.mpi().lsk_mpi_allgather(h.data_ptr(), out.data_ptr(), h.numel() * h.element_size(),
                                                   self.max_msg_bytes), "MPI_Allgather")
        return out if t.device.type == "cpu" else out.to(t.device)

    def alltoallv(self, send, send_counts, recv_counts=None):
        send_counts = [int(c) for c in send_counts]
        recv_counts = (self.exchange_counts(send_counts) if recv_counts is None
                       else [int(c) for c in recv_counts])
        if not self.distributed:
            return send.clone(), recv_counts
        src = self._host(send)
        row_shape = tuple(send.shape[1:])
        rb = src.element_size() * math.prod(row_shape)
        recv = torch.empty((sum(recv_counts), *row_shape), dtype=send.dtype)
        arr = lambda v: (C.c_int64 * len(v))(*v)  # noqa: E731
        so = [o * rb for o in _offsets(send_counts)[:-1]]
        ro = [o * rb for o in _offsets(recv_counts)[:-1]]
        self.ncoll += 1
        _check(_native.mpi().lsk_mpi_alltoallv(
            self.size, src.data_ptr(), arr(so), arr([c * rb for c in send_counts]), recv.data_ptr(), arr(ro),
            arr([c * rb for c in recv_counts]), self.max_msg_bytes, int(self.force)), "MPI all-to-all-v")
        return (recv if send.device.type == "cpu" else recv.to(send.device)), recv_counts

    def p2p(self, sends, recvs):
        out = [torch.empty(shape, dtype=dt) for _, shape, dt in recvs]
        ss = [(dst, self._host(t)) for dst, t in sends]
        own = {}
        sp, rp = [], []
        for dst, t in ss:
            if dst == self.rank and not self.force:
                own[dst] = t
            else:
                sp.append((dst, t))
        for (src, _, _), b in zip(recvs, out):
            if src == self.rank and not self.force:
                if b.numel():
                    b.copy_(own[src])
            else:
                rp.append((src, b))
        if sp or rp:
            ints = lambda v: (C.c_int * max(1, len(v)))(*v)  # noqa: E731
            ptrs = lambda v: (C.c_void_p * max(1, len(v)))(*v)  # noqa: E731
            i64s = lambda v: (C.c_int64 * max(1, len(v)))(*v)  # noqa: E731
            self.ncoll += 1
            _check(_native.mpi().lsk_mpi_sendrecv(
                len(sp), ints([d for d, _ in sp]), ptrs([t.data_ptr() for _, t in sp]),
                i64s([t.numel() * t.element_size() for _, t in sp]), len(rp), ints([s for s, _ in rp]),
                ptrs([b.data_ptr() for _, b in rp]), i64s([b.numel() * b.element_size() for _, b in rp]),
                self.max_msg_bytes), "MPI Isend/Irecv")
        return out if self._device.type == "cpu" else [b.to(self._device) for b in out]

    def barrier(self):
        if self.distributed:
            if self._device.type == "cuda":
                torch.cuda.synchronize(self._device)
            self.ncoll += 1
            _check(_native.mpi().lsk_mpi_barrier(), "MPI_Barrier")
