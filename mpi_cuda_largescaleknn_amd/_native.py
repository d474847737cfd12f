"""ctypes bindings for the native libraries.

``host()`` returns the C++ host runtime (always available: pure CPU), ``hip()`` the
gfx950 kernel library. ``import torch`` happens first so that the kernel library binds
to the same HIP runtime instance as PyTorch (both carry the SONAME libamdhip64.so.7),
which lets every kernel run on torch's current stream and on torch-allocated memory.

On a machine with a GPU, a missing or unloadable kernel library is an error — there
is no silent fallback for CUDA tensors.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (must be loaded before the HIP library, see module doc)

from . import _build

_lock = threading.Lock()
_host_lib = None
_hip_lib = None

i64 = C.c_int64
i32 = C.c_int
u32p = C.POINTER(C.c_uint32)
vp = C.c_void_p
fp = C.c_void_p  # raw device / host pointers are passed as integers


class CliArgs(C.Structure):
    _fields_ = [
        ("input", C.c_char * 4096),
        ("output", C.c_char * 4096),
        ("k", C.c_int),
        ("max_radius", C.c_float),
        ("gpu_affinity", C.c_int),
        ("mode", C.c_char * 32),
        ("device", C.c_char * 16),
        ("stats", C.c_char * 4096),
        ("verbose", C.c_int),
        ("bootstrap", C.c_char * 16),
        ("nproc", C.c_int),
        ("device_map", C.c_char * 256),
        ("balance", C.c_char * 8),
    ]


class TreeView(C.Structure):
    _fields_ = [
        ("pts", vp),
        ("nodes", vp),
        ("qnodes", vp),
        ("n", i64),
        ("depth", C.c_int32),
        ("pad", C.c_int32),
    ]


HIP_ABI = 10  # lsk_hip_abi_version() of a library matching the structs below


class KnnArgs(C.Structure):
    _fields_ = [
        ("qpts", vp),
        ("nq", i64),
        ("groups", vp),
        ("ngroups", i64),
        ("tree", TreeView * 2),
        ("ntrees", C.c_int32),
        ("k", C.c_int32),
        ("cut2", C.c_float),
        ("r_hint2", C.c_float),
        ("out_d2", vp),
        ("stats", vp),
        ("qstatus", vp),
        ("seed", C.c_int32),
        ("wave_base", C.c_int32),
        ("init_d2", vp),
        ("out_perm", vp),
        ("out_final", vp),
        ("fail_list", vp),
        ("fail_count", vp),
        ("fail_cap", i64),
        ("debug_fail_mod", C.c_int32),
        ("wave_end", C.c_int32),
        ("gate", vp),
        ("gate_on", C.c_int32),
        ("pad2", C.c_int32),
        ("ngroups_dev", vp),
        ("wq", vp),
        ("qrot", vp),
    ]


class GridView(C.Structure):
    _fields_ = [
        ("slots", vp),
        ("pad_", vp),
        ("box", vp),
        ("inf4", vp),
        ("level", C.c_int32),
        ("pad", C.c_int32),
    ]


def _declare_host(lib: C.CDLL) -> None:
    lib.lsk_host_abi_version.restype = i32
    lib.lsk_cli_parse.argtypes = [i32, i32, C.POINTER(C.c_char_p), C.POINTER(CliArgs), C.c_char_p, i32]
    lib.lsk_cli_parse.restype = i32
    lib.lsk_io_portion.argtypes = [C.c_char_p, i64, i64, i64, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
    lib.lsk_io_portion.restype = i32
    lib.lsk_io_read.argtypes = [C.c_char_p, i64, i64, vp, i32]
    lib.lsk_io_read.restype = i32
    lib.lsk_io_write.argtypes = [C.c_char_p, i64, vp, i64, i32, i64, i32]
    lib.lsk_io_write.restype = i32
    lib.lsk_io_read_filelist.argtypes = [C.c_char_p, C.c_char_p, i64]
    lib.lsk_io_read_filelist.restype = i64
    lib.lsk_peer_permutation.argtypes = [i32, i32, vp]
    lib.lsk_peer_permutation.restype = None
    lib.lsk_peer_choose.argtypes = [vp, vp, i32, C.c_float, vp, vp]
    lib.lsk_peer_choose.restype = i32
    lib.lsk_box_distance.argtypes = [vp, vp]
    lib.lsk_box_distance.restype = C.c_float
    for name in ("lsk_cpu_kth_brute", "lsk_cpu_kth_kdtree"):
        f = getattr(lib, name)
        f.argtypes = [vp, i64, vp, i64, i32, C.c_float, vp, i32]
        f.restype = None
    lib.lsk_cpu_count_below.argtypes = [vp, i64, vp, vp, i32, vp, i32]
    lib.lsk_cpu_count_below.restype = None
    lib.lsk_cpu_bounds.argtypes = [vp, i64, vp, i32]
    lib.lsk_cpu_bounds.restype = None
    lib.lsk_cpu_morton.argtypes = [vp, i64, vp, C.c_float, vp, i32, i32]
    lib.lsk_cpu_morton.restype = None
    lib.lsk_cpu_halo_mask.argtypes = [vp, i64, vp, vp, i32, i32, vp, i32]
    lib.lsk_cpu_halo_mask.restype = None
    lib.lsk_cpu_lbt_build.argtypes = [vp, i64, vp, vp]
    lib.lsk_cpu_lbt_build.restype = None
    lib.lsk_cpu_refalgo_knn.argtypes = [vp, i64, vp, i64, vp, i32, C.c_float, i32, vp, C.c_uint32, i32]
    lib.lsk_cpu_refalgo_knn.restype = None
    lib.lsk_cpu_refalgo_extract.argtypes = [vp, i64, i32, vp]
    lib.lsk_cpu_refalgo_extract.restype = None


def _declare_hip(lib: C.CDLL) -> None:
    lib.lsk_hip_abi_version.restype = i32
    lib.lsk_hip_last_error.restype = C.c_char_p
    lib.lsk_hip_device_info.argtypes = [i32, C.c_char_p, i32]
    lib.lsk_hip_device_info.restype = i32
    sigs = {
        "lsk_hip_bounds_ws_bytes": ([i64], C.c_size_t),
        "lsk_hip_bounds": ([vp, i64, vp, vp, vp], i32),
        "lsk_hip_box_finalize": ([vp, vp], i32),
        "lsk_hip_radius_hint": ([vp, i64, i32, vp, vp], i32),
        "lsk_hip_morton": ([vp, i64, vp, vp, vp, i32, vp], i32),
        "lsk_hip_morton_ex": ([vp, i64, vp, vp, vp, i32, i64, vp, vp], i32),
        "lsk_hip_gather3": ([vp, vp, i64, vp, vp], i32),
        "lsk_hip_scatter1": ([vp, vp, i64, vp, i32, vp], i32),
        "lsk_hip_finalize": ([vp, i64, vp, vp], i32),
        "lsk_hip_dest_rank": ([vp, i64, vp, i32, i32, vp, vp, vp], i32),
        "lsk_hip_key_histogram": ([vp, i64, i32, i32, vp, vp], i32),
        "lsk_hip_count_dest": ([vp, i64, i32, vp, vp], i32),
        "lsk_hip_sort_ws_bytes": ([i64], C.c_size_t),
        "lsk_hip_sort_pairs": ([vp, vp, vp, vp, i64, i32, vp, C.POINTER(C.c_int), vp], i32),
        "lsk_hip_sort_keys_iota": ([vp, vp, vp, vp, i64, i32, vp, C.POINTER(C.c_int), vp], i32),
        "lsk_hip_sort_keys_iota_gather": ([vp, vp, vp, vp, i64, i32, vp, C.POINTER(C.c_int), vp, vp, vp], i32),
        "lsk_hip_key_census": ([vp, i64, vp, i64, vp, vp], i32),
        "lsk_hip_tree_depth": ([i64], i32),
        "lsk_hip_tree_nodes": ([i64], i64),
        "lsk_hip_build_tree": ([vp, i64, vp, vp, vp], i32),
        "lsk_hip_tree_set_radii": ([vp, i64, vp, vp], i32),
        "lsk_hip_tree_set_radii_ub": ([vp, vp, i64, i32, vp], i32),
        "lsk_hip_knn_exact": ([C.POINTER(KnnArgs), vp, vp, i64, vp], i32),
        "lsk_hip_knn_rows": ([C.POINTER(KnnArgs), vp], i32),
        "lsk_hip_knn_grid": ([C.POINTER(KnnArgs), C.POINTER(GridView), vp], i32),
        "lsk_hip_knn_grid2": ([C.POINTER(KnnArgs), C.POINTER(GridView), C.POINTER(GridView), vp], i32),
        "lsk_hip_grid_decide": ([vp, vp, i64, i32, C.c_float, i32, vp, vp], i32),
        "lsk_hip_boundary_groups": ([vp, i32, i64, vp, vp, vp, C.c_int, C.c_int, vp, vp], i32),
        "lsk_hip_grid_build": ([vp, vp, i64, vp, i32, vp, vp], i32),
        "lsk_hip_key_levels": ([vp, i64, vp, vp], i32),
        "lsk_hip_grid_sq": ([vp, i64, vp, vp], i32),
        "lsk_hip_halo_mask": ([vp, i64, vp, vp, vp, i32, i32, vp, vp], i32),
        "lsk_hip_flag_query_groups": ([vp, vp, i64, vp, C.c_int32, i64, vp, vp], i32),
        "lsk_hip_flag_groups_inverse": ([vp, i64, vp, C.c_int32, i64, vp, vp], i32),
        "lsk_hip_compact_flags": ([vp, i64, vp, vp, vp], i32),
        "lsk_hip_halo_pack": ([vp, vp, i64, i32, vp, vp, vp, vp], i32),
        "lsk_hip_mask_counts": ([vp, i64, i32, vp, vp], i32),
        "lsk_hip_lbt_keys": ([vp, i64, i32, vp, vp, vp], i32),
        "lsk_hip_lbt_retag": ([vp, i64, i32, vp], i32),
        "lsk_hip_gather_u32": ([vp, vp, i64, vp, vp], i32),
        "lsk_hip_refalgo_knn": ([vp, i64, vp, i64, vp, i32, C.c_float, i32, vp, C.c_uint32, vp], i32),
        "lsk_hip_refalgo_extract": ([vp, i64, i32, vp, vp], i32),
        "lsk_hip_count_below": ([vp, i64, vp, vp, i32, vp, vp], i32),
        "lsk_hip_segment_bounds": ([vp, vp, i64, i64, vp, vp, vp], i32),
    }
    for name, (args, res) in sigs.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res


def host() -> C.CDLL:
    global _host_lib
    if _host_lib is None:
        with _lock:
            if _host_lib is None:
                path = _build.build_host()
                lib = C.CDLL(path)
                _declare_host(lib)
                _host_lib = lib
    return _host_lib


def hip() -> C.CDLL:
    """The gfx950 kernel library; raises if it cannot be built or loaded."""
    global _hip_lib
    if _hip_lib is None:
        with _lock:
            if _hip_lib is None:
                path = _build.HIP_LIB
                override = os.environ.get("LSKNN_HIP_LIB")  # tuning experiments only
                if override:
                    path = override
                elif not os.path.exists(path) or os.environ.get("LSKNN_REBUILD"):
                    path = _build.build_hip()
                else:
                    # rebuild if sources changed (cheap mtime check; needs hipcc)
                    try:
                        path = _build.build_hip()
                    except RuntimeError:
                        if not os.path.exists(path):
                            raise
                lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
                _declare_hip(lib)
                ver = lib.lsk_hip_abi_version()
                if ver != HIP_ABI:  # the ctypes structs below must match lsk_hip.h
                    raise NativeError(f"{path}: ABI version {ver}, expected {HIP_ABI} (rebuild)")
                _hip_lib = lib
    return _hip_lib


_comm_lib = None


def comm() -> C.CDLL:
    """The native RCCL communicator library (csrc/comm/rccl_comm.cpp)."""
    global _comm_lib
    if _comm_lib is None:
        with _lock:
            if _comm_lib is None:
                path = _build.build_comm()
                lib = C.CDLL(path)
                lib.lsk_comm_last_error.restype = C.c_char_p
                lib.lsk_comm_load.argtypes = [C.c_char_p]
                lib.lsk_comm_version.argtypes = [C.POINTER(C.c_int)]
                lib.lsk_comm_unique_id.argtypes = [C.c_char_p, i32]
                lib.lsk_comm_init.argtypes = [C.c_char_p, i32, i32, i32, C.POINTER(vp)]
                lib.lsk_comm_destroy.argtypes = [vp, i32]
                lib.lsk_comm_async_error.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_char_p)]
                lib.lsk_comm_allreduce.argtypes = [vp, vp, i64, i32, i32, vp]
                lib.lsk_comm_allgather.argtypes = [vp, vp, vp, i64, vp]
                lib.lsk_comm_alltoallv.argtypes = [vp, i32, i32, vp, vp, vp, vp, vp, vp, i64, i32, vp]
                lib.lsk_comm_sendrecv.argtypes = [vp, i32, vp, vp, vp, i32, vp, vp, vp, i64, vp]
                _comm_lib = lib
    return _comm_lib


_mpi_lib = None


def mpi() -> C.CDLL:
    """The native MPI host communicator library (csrc/mpi/mpi_comm.cpp)."""
    global _mpi_lib
    if _mpi_lib is None:
        with _lock:
            if _mpi_lib is None:
                path = _build.build_mpi()
                if path is None:
                    raise NativeError("LSKNN_DIST_BACKEND=mpi: no MPI installation found "
                                      "(set LSKNN_MPI_HOME to a directory with include/mpi.h and lib/libmpi.so)")
                lib = C.CDLL(path)
                lib.lsk_mpi_last_error.restype = C.c_char_p
                lib.lsk_mpi_init.argtypes = [C.POINTER(C.c_int), C.POINTER(C.c_int)]
                lib.lsk_mpi_abort.argtypes = [i32]
                lib.lsk_mpi_abort.restype = None
                lib.lsk_mpi_bcast.argtypes = [vp, i64, i32]
                lib.lsk_mpi_allreduce.argtypes = [vp, i64, i32, i32]
                lib.lsk_mpi_allgather.argtypes = [vp, vp, i64, i64]
                lib.lsk_mpi_alltoallv.argtypes = [i32, vp, vp, vp, vp, vp, vp, i64, i32]
                lib.lsk_mpi_sendrecv.argtypes = [i32, vp, vp, vp, i32, vp, vp, vp, i64]
                _mpi_lib = lib
    return _mpi_lib


class NativeError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = hip().lsk_hip_last_error()
        raise NativeError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def loaded_libraries() -> list[str]:
    """Paths of the native libraries loaded into this process."""
    out = []
    if _host_lib is not None:
        out.append(_build.HOST_LIB)
    if _hip_lib is not None:
        out.append(_build.HIP_LIB)
    if _comm_lib is not None:
        out.append(_build.COMM_LIB)
    return out
