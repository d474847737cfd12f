"""Failure detection, fault injection and the no-hang guarantee.

The reference has none: a failing MPI call throws through ``CUKD_MPI_CALL``
(unorderedDataVariant.cu:23-26), nothing catches it and the job relies on mpirun to
tear the other ranks down; a rank-count mismatch throws the same way
(prePartitionedDataVariant.cu:215-216). Here every multi-rank job gets:

* **abort broadcast** — a rank that fails sets ``lsknn/abort`` in the process group's
  TCP store (with its rank and message) before exiting non-zero;
* **watchdog** — a daemon thread per rank that (a) polls that key and (b) checks a
  progress heartbeat (every Comm call and phase mark beats it). On a peer's abort, or
  when no progress was made for ``LSKNN_TIMEOUT`` seconds (default 900), it prints
  ``#r/P: ...`` to stderr and ends the process with ``os._exit`` (exit code 3 for a
  peer abort, 124 for a timeout) — no rank is ever left blocked in a collective. The
  collective timeout of the process group is set to the same value, and RCCL's async
  error handling is enabled, as a second line;
* **fault injection** for tests — ``LSKNN_FAULT="rank=R,op=OP[,call=N][,kind=K]"``
  makes rank R fail its N-th (0-based, default 0) call of Comm method OP
  (``allreduce_``, ``allgather``, ``alltoallv``, ``p2p``, ``barrier``, ``allgather_host``
  or ``*``) with kind ``raise`` (default: an exception, handled like any error),
  ``exit`` (``os._exit(7)``, a crash without cleanup) or ``hang`` (blocks forever:
  exercises the watchdog).
"""
from __future__ import annotations

import os
import sys
import threading
import time

from .comm import Comm

ABORT_KEY = "lsknn/abort"
EXIT_PEER_ABORT = 3
EXIT_TIMEOUT = 124
EXIT_COMM_ERROR = 5  # the communicator reported an asynchronous error


class InjectedFault(RuntimeError):
    pass


def timeout_s() -> float:
    return float(os.environ.get("LSKNN_TIMEOUT", "900"))


class Heartbeat:
    def __init__(self):
        self.t = time.monotonic()
        self.what = "start"
        self.host = 0  # > 0: inside a long local host phase (host_phase), not idle

    def host_phase(self, what: str):
        """Context for a long local phase with no collective (data generation, the sampled
        check, a library build): the progress timeout does not run inside it, and the
        heartbeat is beaten on the way in and out (a 150 s bench timeout must
        only catch time spent waiting on peers)."""
        hb = self

        class _Phase:
            def __enter__(self):
                hb.host += 1
                hb.beat(what)
                return self

            def __exit__(self, *exc):
                hb.host -= 1
                hb.beat()
                return False

        return _Phase()

    def beat(self, what: str = "") -> None:
        self.t = time.monotonic()
        if what:
            self.what = what


HEARTBEAT = Heartbeat()


def parse_fault(spec: str | None) -> dict | None:
    if not spec:
        return None
    out = {"call": 0, "kind": "raise", "op": "*"}
    for part in spec.split(","):
        k, _, v = part.partition("=")
        k, v = k.strip(), v.strip()
        if k not in ("rank", "op", "call", "kind"):
            raise ValueError(f"LSKNN_FAULT: unknown key {k!r}")
        out[k] = int(v) if k in ("rank", "call") else v
    if "rank" not in out:
        raise ValueError("LSKNN_FAULT needs rank=R")
    if out["kind"] not in ("raise", "exit", "hang"):
        raise ValueError(f"LSKNN_FAULT: unknown kind {out['kind']!r}")
    return out


class MonitoredComm(Comm):
    """Wraps a Comm: beats the heartbeat around every call and injects the configured
    fault (if any) on this rank."""

    _OPS = ("allreduce_", "allgather", "alltoallv", "barrier", "p2p", "exchange_counts", "allgather_host",
            "count_exchange")

    def __init__(self, inner: Comm, fault: dict | None = None):
        self.inner = inner
        self.rank = inner.rank
        self.size = inner.size
        self.force = inner.force
        self.fault = fault if fault and fault["rank"] == inner.rank else None
        self.calls: dict[str, int] = {}

    @property
    def device(self):
        return self.inner.device

    def collectives(self) -> int:
        return self.inner.collectives()

    def _enter(self, op: str) -> None:
        HEARTBEAT.beat(op)
        n = self.calls.get(op, 0)
        self.calls[op] = n + 1
        self.calls["*"] = self.calls.get("*", 0) + 1
        f = self.fault
        if f is None or f["op"] not in ("*", op) or self.calls[f["op"]] - 1 != f["call"]:
            return
        msg = f"injected fault ({f['kind']}) in {op} call {n} on rank {self.rank}"
        if f["kind"] in ("exit", "hang"):
            sys.stderr.write(f"#{self.rank}/{self.size}: {msg}\n")
            sys.stderr.flush()
            if f["kind"] == "exit":
                os._exit(7)
            threading.Event().wait()
        raise InjectedFault(msg)

    def _call(self, op, *a, **kw):
        self._enter(op)
        r = getattr(self.inner, op)(*a, **kw)
        HEARTBEAT.beat()
        return r

    def allreduce_(self, t, op="sum"):
        return self._call("allreduce_", t, op)

    def allgather(self, t):
        return self._call("allgather", t)

    def alltoallv(self, send, send_counts, recv_counts=None):
        return self._call("alltoallv", send, send_counts, recv_counts)

    def barrier(self):
        return self._call("barrier")

    def p2p(self, sends, recvs):
        return self._call("p2p", sends, recvs)

    def exchange_counts(self, counts):
        return self._call("exchange_counts", counts)

    def count_exchange(self, counts):
        return self._call("count_exchange", counts)

    def allgather_host(self, t):
        return self._call("allgather_host", t)


class Watchdog:
    """Per-rank daemon thread: peer-abort polling + progress timeout (see module doc)."""

    def __init__(self, rank: int, size: int, store=None, timeout: float | None = None, poll: float = 0.5,
                 comm_check=None, on_abort=None):
        """`comm_check()` -> error string or None: polled every interval (the native RCCL
        communicator's ncclCommGetAsyncError); `on_abort()` runs before the process exits
        on any watchdog abort (ncclCommAbort)."""
        self.rank, self.size = rank, size
        self.store = store
        self.comm_check = comm_check
        self.on_abort = on_abort
        self.timeout = timeout_s() if timeout is None else timeout
        self.poll = poll
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, name="lsknn-watchdog", daemon=True)

    def start(self) -> "Watchdog":
        HEARTBEAT.beat("start")
        self.thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _die(self, msg: str, code: int) -> None:
        if self.on_abort is not None:
            try:
                self.on_abort()
            except Exception:  # noqa: BLE001 - exiting anyway
                pass
        sys.stderr.write(f"#{self.rank}/{self.size}: {msg}\n")
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(code)

    def _run(self) -> None:
        while not self._stop.wait(self.poll):
            if self.store is not None:
                try:
                    if self.store.check([ABORT_KEY]):
                        who = self.store.get(ABORT_KEY).decode(errors="replace")
                        if not self._stop.is_set():
                            self._die(f"aborting: {who}", EXIT_PEER_ABORT)
                except Exception:  # noqa: BLE001 - store gone = rank 0 (the store host) died
                    if not self._stop.is_set():
                        self._die("aborting: lost the rendezvous store (a peer died)", EXIT_PEER_ABORT)
            if self.comm_check is not None:
                try:
                    err = self.comm_check()
                except Exception as e:  # noqa: BLE001
                    err = f"communicator check failed: {e}"
                if err and not self._stop.is_set():
                    if self.store is not None:
                        try:
                            self.store.set(ABORT_KEY, f"rank {self.rank}: {err}")
                        except Exception:  # noqa: BLE001
                            pass
                    self._die(f"aborting: {err}", EXIT_COMM_ERROR)
            idle = time.monotonic() - HEARTBEAT.t
            if HEARTBEAT.host > 0:
                continue
            if idle > self.timeout and not self._stop.is_set():
                if self.store is not None:
                    try:
                        self.store.set(ABORT_KEY, f"rank {self.rank} timed out in {HEARTBEAT.what}")
                    except Exception:  # noqa: BLE001
                        pass
                self._die(f"watchdog: timeout in {HEARTBEAT.what}: no progress for {idle:.0f}s, aborting",
                          EXIT_TIMEOUT)


def announce_failure(store, rank: int, size: int, exc: BaseException) -> None:
    """Publish this rank's failure so that every peer's watchdog aborts promptly."""
    if store is None:
        return
    try:
        store.set(ABORT_KEY, f"rank {rank}/{size} failed: {type(exc).__name__}: {exc}")
    except Exception:  # noqa: BLE001
        pass
