"""Native RCCL communicator: the pipelines' Comm interface on csrc/comm/rccl_comm.cpp.

SURVEY §5.8: the reference drives CUDA-aware MPI from C++ (MPIComm, Isend/Irecv,
Allreduce, Allgather, Barrier; unorderedDataVariant.cu:23-39, 183-193). `RcclComm` calls
RCCL directly through a small C++ library: every collective is enqueued on the caller's
current HIP stream (the overlapped halo exchange's high-priority side stream included),
with no process-group wrapper or internal stream in between. Bootstrap: rank 0 creates
the RCCL unique id and publishes it in the job's key-value store (the torch TCPStore that
the gloo control group of parallel/launch.py already runs); every rank then calls
ncclCommInitRank. The control group (gloo) stays for the watchdog and host barriers.

Which RCCL: `LSKNN_RCCL_LIB` (a path), else ROCm's /opt/rocm/lib/librccl.so.1 (2.27),
else torch's bundled copy (2.26). The library is dlopen'ed by path with local symbols, so
it does not clash with the copy torch itself loaded.

It is the default GPU data path of a multi-rank run (launch.default_gpu_backend: faster
than TorchComm on a forced 1-rank group, profiles/r5_rccl_ab/); ``LSKNN_DIST_BACKEND=nccl``
selects torch's ProcessGroupNCCL instead.
"""
from __future__ import annotations

import ctypes as C
import math
import os

import torch

from .. import _native
from .comm import MAX_MSG_BYTES, Comm, _offsets

_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
           torch.float32: 7, torch.float64: 8, torch.bfloat16: 9}
_OPS = {"sum": 0, "max": 2, "min": 3}


def rccl_path() -> str:
    env = os.environ.get("LSKNN_RCCL_LIB")
    if env:
        return env
    for cand in ("/opt/rocm/lib/librccl.so.1",):
        if os.path.exists(cand):
            return cand
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _native.comm().lsk_comm_last_error()
        raise _native.NativeError(f"{what} failed: {msg.decode() if msg else rc}")


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def plan_pieces(nbytes: list[int], piece: int) -> int:
    """Rounds a grouped exchange needs when every message goes in pieces of <= piece bytes."""
    piece = max(1, int(piece))
    return max([(b + piece - 1) // piece for b in nbytes] + [0])


class RcclComm(Comm):
    """One rank of a native RCCL communicator (GPU tensors only)."""

    def __init__(self, device: torch.device | str, rank: int, size: int, store, force: bool = False,
                 key: str = "lsknn/rccl_id", lib_path: str | None = None, connect: bool = True):
        """`connect=False`: only the local steps (load RCCL, its version; rank 0 creates and
        publishes the unique id); `connect()` then runs the blocking ncclCommInitRank, after
        the ranks agreed that every one of them got this far (launch.bring_up_native)."""
        self._device = torch.device(device)
        if self._device.type != "cuda":
            raise ValueError("RcclComm needs a GPU device")
        self.rank, self.size, self.force = int(rank), int(size), bool(force)
        self.backend = "rccl"
        self.staged = False
        self.max_msg_bytes = MAX_MSG_BYTES
        lib = _native.comm()
        self.lib_path = lib_path or rccl_path()
        _check(lib.lsk_comm_load(self.lib_path.encode()), f"loading {self.lib_path}")
        v = C.c_int(0)
        _check(lib.lsk_comm_version(C.byref(v)), "ncclGetVersion")
        self.version = v.value
        self._store, self._key, self._h = store, key, None
        if self.rank == 0:
            nid = lib.lsk_comm_id_bytes()
            buf = C.create_string_buffer(nid)
            _check(lib.lsk_comm_unique_id(buf, nid), "ncclGetUniqueId")
            store.set(key, buf.raw)
        if connect:
            self.connect()

    def connect(self) -> None:
        """ncclCommInitRank (a collective: blocks until every rank has called it)."""
        lib = _native.comm()
        nid = lib.lsk_comm_id_bytes()
        uid = bytes(self._store.get(self._key))  # rank 0 published it before any rank gets here
        if len(uid) != nid:
            raise RuntimeError("RCCL unique id of the wrong size in the store")
        h = C.c_void_p()
        _check(lib.lsk_comm_init(uid, self.size, self.rank, self._device.index, C.byref(h)), "ncclCommInitRank")
        self._h = h

    @property
    def device(self) -> torch.device:
        return self._device

    def destroy(self, abort: bool = False) -> None:
        if getattr(self, "_h", None):
            _check(_native.comm().lsk_comm_destroy(self._h, int(abort)), "ncclCommDestroy")
            self._h = None

    def async_error(self) -> str | None:
        """RCCL's asynchronous error state (None while healthy); safe from another thread
        (the watchdog polls it)."""
        h = getattr(self, "_h", None)
        if not h:
            return None
        err, msg = C.c_int(0), C.c_char_p()
        if _native.comm().lsk_comm_async_error(h, C.byref(err), C.byref(msg)) != 0:
            return "ncclCommGetAsyncError failed"
        if err.value == 0:
            return None
        return f"RCCL async error {err.value}: {msg.value.decode() if msg.value else ''}"

    def abort(self) -> None:
        """ncclCommAbort: unblocks this rank's pending RCCL work before the process exits."""
        h = getattr(self, "_h", None)
        if h:
            self._h = None
            _native.comm().lsk_comm_destroy(h, 1)

    # ---------------------------------------------------------------- collectives
    def _dev(self, t: torch.Tensor) -> torch.Tensor:
        return t if t.device == self._device else t.to(self._device)

    def allreduce_(self, t, op="sum"):
        if not self.distributed:
            return t
        d = self._dev(t).contiguous()
        self.ncoll += 1
        _check(_native.comm().lsk_comm_allreduce(self._h, d.data_ptr(), d.numel(), _DTYPES[d.dtype], _OPS[op],
                                                 _stream(self._device)), "allreduce")
        if d.data_ptr() != t.data_ptr():
            t.copy_(d)
        return t

    def allgather(self, t):
        d = self._dev(t).contiguous()
        out = torch.empty((self.size, *t.shape), dtype=t.dtype, device=self._device)
        if not self.distributed:
            out[0].copy_(d)
        else:
            self.ncoll += 1
            _check(_native.comm().lsk_comm_allgather(self._h, d.data_ptr(), out.data_ptr(),
                                                     d.numel() * d.element_size(), _stream(self._device)),
                   "allgather")
        return out if t.device == self._device else out.to(t.device)

    def alltoallv(self, send, send_counts, recv_counts=None):
        send_counts = [int(c) for c in send_counts]
        recv_counts = (self.exchange_counts(send_counts) if recv_counts is None
                       else [int(c) for c in recv_counts])
        if not self.distributed:
            return send.clone(), recv_counts
        src = self._dev(send).contiguous()
        row_shape = tuple(send.shape[1:])
        rb = src.element_size() * math.prod(row_shape)
        recv = torch.empty((sum(recv_counts), *row_shape), dtype=send.dtype, device=self._device)
        so = [o * rb for o in _offsets(send_counts)[:-1]]
        ro = [o * rb for o in _offsets(recv_counts)[:-1]]
        arr = lambda v: (C.c_int64 * len(v))(*v)  # noqa: E731
        self.ncoll += 1
        _check(_native.comm().lsk_comm_alltoallv(
            self._h, self.size, self.rank, src.data_ptr(), arr(so), arr([c * rb for c in send_counts]),
            recv.data_ptr(), arr(ro), arr([c * rb for c in recv_counts]), self.max_msg_bytes, int(self.force),
            _stream(self._device)), "alltoallv")
        return recv, recv_counts

    def p2p(self, sends, recvs):
        out = [torch.empty(shape, dtype=dt, device=self._device) for _, shape, dt in recvs]
        ss = [(dst, self._dev(t).contiguous()) for dst, t in sends]
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
            _check(_native.comm().lsk_comm_sendrecv(
                self._h, len(sp), ints([d for d, _ in sp]), ptrs([t.data_ptr() for _, t in sp]),
                i64s([t.numel() * t.element_size() for _, t in sp]), len(rp), ints([s for s, _ in rp]),
                ptrs([b.data_ptr() for _, b in rp]), i64s([b.numel() * b.element_size() for _, b in rp]),
                self.max_msg_bytes, _stream(self._device)), "sendrecv")
        return out

    def barrier(self):
        if self.distributed:
            t = torch.zeros(1, device=self._device)
            self.allreduce_(t)
            torch.cuda.current_stream(self._device).synchronize()
