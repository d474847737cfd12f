"""float3 point files, distance files and file lists (native pread/pwrite runtime).

File formats are those of the reference:

* input  : headerless little-endian packed float32 x,y,z records (12 B); trailing
           bytes < 12 are ignored;
* output : headerless float32 distances;
* list   : text file, one point-file path per line, line i = rank i.

``read_portion`` reproduces readFilePortion (unorderedDataVariant.cu:42-63): rank r of
P reads records [floor(N*r/P), floor(N*(r+1)/P)), with the arithmetic done in 128-bit
integers so any file size works (the reference's size_t math overflows N*r past
2^64/P; SURVEY D1-D3 list its 32-bit limits elsewhere).
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from .. import _native

REC = 12  # sizeof(float3)


def _nthreads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def _err(rc: int, what: str, path: str) -> None:
    if rc != 0:
        raise OSError(-rc, f"{what} failed for {path!r}: {os.strerror(-rc) if rc < 0 else rc}")


def portion(path: str, rank: int = 0, size: int = 1, recsize: int = REC) -> tuple[int, int, int]:
    """(begin, count, total) records of `path` owned by `rank` of `size`."""
    b, c, t = C.c_int64(), C.c_int64(), C.c_int64()
    rc = _native.host().lsk_io_portion(path.encode(), rank, size, recsize, C.byref(b), C.byref(c), C.byref(t))
    _err(rc, "portion", path)
    return b.value, c.value, t.value


def read_portion(path: str, rank: int = 0, size: int = 1, pin_memory: bool = False):
    """Read this rank's block of a float3 file -> ([n,3] float32 tensor, begin, total)."""
    begin, count, total = portion(path, rank, size)
    out = torch.empty((count, 3), dtype=torch.float32, pin_memory=pin_memory)
    if count:
        rc = _native.host().lsk_io_read(path.encode(), begin * REC, count * REC, out.data_ptr(), _nthreads())
        _err(rc, "read", path)
    return out, begin, total


def read_points(path: str, pin_memory: bool = False) -> torch.Tensor:
    return read_portion(path, 0, 1, pin_memory)[0]


def write_floats(path: str, data: torch.Tensor, offset_records: int = 0, truncate: bool = True,
                 total_records: int | None = None) -> None:
    """pwrite float32 values at record offset (4 B records). flags: truncate / ftruncate."""
    data = data.detach().contiguous()
    if data.device.type != "cpu":
        data = data.cpu()
    assert data.dtype == torch.float32
    flags = (1 if truncate else 0) | (2 if total_records is not None else 0)
    total = -1 if total_records is None else total_records * 4
    rc = _native.host().lsk_io_write(path.encode(), offset_records * 4, data.data_ptr(), data.numel() * 4, flags,
                                     total, _nthreads())
    _err(rc, "write", path)


def write_points(path: str, pts: torch.Tensor) -> None:
    pts = pts.detach().to(torch.float32).contiguous().cpu()
    rc = _native.host().lsk_io_write(path.encode(), 0, pts.data_ptr(), pts.numel() * 4, 1, -1, _nthreads())
    _err(rc, "write", path)


def read_floats(path: str) -> torch.Tensor:
    n = os.path.getsize(path) // 4
    out = torch.empty(n, dtype=torch.float32)
    if n:
        rc = _native.host().lsk_io_read(path.encode(), 0, n * 4, out.data_ptr(), _nthreads())
        _err(rc, "read", path)
    return out


def read_file_list(path: str) -> list[str]:
    """Reference readListOfFileNames, fixed: an unterminated last line is
    kept, CR is stripped, blank lines are skipped."""
    size = 1 << 16
    while True:
        buf = C.create_string_buffer(size)
        n = _native.host().lsk_io_read_filelist(path.encode(), buf, size)
        if n <= -1000000:
            size = -(n + 1000000) + 16
            continue
        if n < 0:
            raise OSError(-n, f"cannot read file list {path!r}")
        if n == 0:
            return []
        return buf.value.decode().split("\n")
