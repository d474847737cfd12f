"""roctx markers and ranges: visible in ``rocprofv3 --marker-trace``
timelines next to the kernels. The reference has no tracing at all.

* :func:`mark` — an instantaneous marker (``PhaseTimer.mark`` emits ``lsknn:<phase>``
  at the end of every pipeline phase);
* :func:`range` — a context manager pushing / popping a named range (one per
  benchmark or CLI step).

The roctx library is loaded lazily; when it is absent, or ``LSKNN_ROCTX=0``, both are
no-ops.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if not _tried:
        _tried = True
        if os.environ.get("LSKNN_ROCTX", "1") != "0":
            for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                         "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    _lib = lib
                    break
                except OSError:
                    continue
    return _lib


def available() -> bool:
    return _roctx() is not None


def mark(name: str) -> None:
    lib = _roctx()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
