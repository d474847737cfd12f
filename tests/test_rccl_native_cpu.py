"""Native RCCL communicator, host side (no GPU): the library builds, RCCL loads by path
and reports its version, bad paths fail loudly, the piece planning of large messages."""
import ctypes as C
import os

import pytest
import torch

from mpi_cuda_largescaleknn_amd import _native
from mpi_cuda_largescaleknn_amd.parallel import rccl as R


def test_comm_library_loads_rccl_by_path():
    lib = _native.comm()
    assert lib.lsk_comm_id_bytes() == 128
    v = C.c_int(0)
    # before a successful load every call fails with a message
    path = R.rccl_path()
    assert os.path.exists(path)
    assert lib.lsk_comm_load(path.encode()) == 0
    assert lib.lsk_comm_version(C.byref(v)) == 0 and v.value >= 22600


def test_rccl_path_override(monkeypatch):
    monkeypatch.setenv("LSKNN_RCCL_LIB", "/x/librccl.so")
    assert R.rccl_path() == "/x/librccl.so"
    monkeypatch.delenv("LSKNN_RCCL_LIB")
    assert R.rccl_path().endswith(("librccl.so.1", "librccl.so"))


def test_bad_library_path_reports_dlopen_error():
    import subprocess
    import sys
    code = ("from mpi_cuda_largescaleknn_amd import _native; lib=_native.comm(); "
            "rc=lib.lsk_comm_load(b'/nonexistent/librccl.so'); "
            "print(rc, lib.lsk_comm_last_error().decode())")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("1 dlopen /nonexistent/librccl.so")


def test_piece_planning():
    assert R.plan_pieces([], 256) == 0
    assert R.plan_pieces([0, 0], 256) == 0
    assert R.plan_pieces([1, 256, 257], 256) == 2
    assert R.plan_pieces([3 << 30], 256 << 20) == 12


def test_rccl_comm_needs_gpu():
    with pytest.raises(ValueError):
        R.RcclComm(torch.device("cpu"), 0, 1, None)


def test_unknown_backend_rejected(monkeypatch):
    from mpi_cuda_largescaleknn_amd.parallel import launch as LA
    saved = dict(os.environ)  # init exports RANK / WORLD_SIZE / MASTER_* before it fails
    monkeypatch.setenv("LSKNN_DIST_BACKEND", "bogus")
    try:
        with pytest.raises(ValueError, match="nccl, rccl, gloo or mpi"):
            LA.init(device_pref="cpu", force_distributed=True)
    finally:
        for k in set(os.environ) - set(saved):
            del os.environ[k]
        os.environ.update(saved)


def test_default_gpu_backend(monkeypatch):
    """The native communicator is the GPU default when its library and an RCCL are on
    disk (the measured-faster path), torch's group otherwise; the choice depends only on
    files, so every rank of a job makes the same one."""
    from mpi_cuda_largescaleknn_amd import _build
    from mpi_cuda_largescaleknn_amd.parallel import launch as LA
    real, lib = os.path.exists, R.rccl_path()
    monkeypatch.setattr(os.path, "exists", lambda p: True if p in (_build.COMM_LIB, lib) else real(p))
    assert LA.default_gpu_backend() == "rccl"
    monkeypatch.setattr(os.path, "exists", lambda p: False if p == _build.COMM_LIB else real(p))
    assert LA.default_gpu_backend() == "nccl"
