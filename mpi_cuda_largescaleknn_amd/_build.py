"""In-tree build of the native libraries.

* ``lib/liblsknn_host.so``  — C++17 host runtime (I/O, CLI, peer schedule, CPU oracle),
  built with g++.
* ``lib/liblsknn_hip.so``   — hand-written gfx950 HIP kernels, built with
  ``hipcc --offload-arch=gfx950`` (cross-compiles without a GPU).
* ``lib/liblsknn_comm.so``  — native RCCL communicator (host code, RCCL dlopen'ed).
* ``lib/liblsknn_mpi.so``   — native MPI host communicator (g++ against the image's
  MPICH; skipped when no MPI installation is found).

All are rebuilt only when a source or header is newer than the library. The
libraries are git-ignored but travel to the GPU box with the working tree.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "lib")
HOST_LIB = os.path.join(LIB_DIR, "liblsknn_host.so")
HIP_LIB = os.path.join(LIB_DIR, "liblsknn_hip.so")
GPU_ARCH = os.environ.get("LSKNN_GPU_ARCH", "gfx950")

# -ffp-contract=off everywhere: the canonical dist2 association must not be changed by
# FMA contraction; correctly-rounded sqrtf requires no fast-math.
COMMON_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math"]
HOST_FLAGS = COMMON_FLAGS + ["-mfma", "-mavx2", "-pthread", "-Wall", "-Wno-unused-function"]
HIP_FLAGS = COMMON_FLAGS + [f"--offload-arch={GPU_ARCH}", "-Wno-unused-result"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def _sources(sub: str, ext: str) -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, sub, f"*.{ext}")))


def _headers() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True) +
                  glob.glob(os.path.join(CSRC, "**", "*.inc"), recursive=True))


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + proc.stdout)


# The SLP vectorizer packs the per-candidate distance math into v_pk_* ops, which cannot
# take the DPP row broadcast as an operand: it adds a v_mov_dpp per operand and ~50 VGPRs.
FILE_FLAGS = {
    # the pass-1 log is a dynamically indexed private array: keep it in scratch memory
    # instead of promoting it to (dynamically indexed, hence many) VGPRs
    # iterative-maxocc scheduling (round 5, 2e7 k=100: clustered 595-600 vs 587-588 Mpts/s
    # with max-memory-clause, planar 1228-1246 vs 1207-1212, profiles/r5_kernel_ab/
    # rows_sched_nonuniform_2e7.txt; round 2: max-memory-clause 0.1255 vs default 0.1265 s
    # on 1e8, ilp 0.131, iterative-ilp 0.138, profiles/archive/r2_kernel/README.txt)
    # candidates arrive in SGPRs: packed-math pairs would need them moved into VGPRs;
    # iterative-minreg scheduling: 1e8 k=100 74.4 vs 76.8 ms (iterative-maxocc 75.1,
    # max-memory-clause 77.5, max-ilp 78.1, iterative-ilp 77.4; profiles/r5_kernel_ab/sched_1e8.txt)
    "knn_grid.hip": ["-fno-slp-vectorize", "-mllvm", "-amdgpu-sched-strategy=iterative-minreg"],
    "knn_rows.hip": ["-fno-slp-vectorize", "-mllvm", "-disable-promote-alloca-to-vector",
                     "-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"],
}


def build_host(force: bool = False, verbose: bool = False) -> str:
    srcs = _sources("host", "cpp")
    if force or _stale(HOST_LIB, srcs + _headers()):
        os.makedirs(LIB_DIR, exist_ok=True)
        tmp = HOST_LIB + ".tmp"
        cmd = ["g++", *HOST_FLAGS, "-shared", "-o", tmp, *srcs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_hip(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    srcs = _sources("hip", "hip")
    # (this file holds the compile flags: a flag change rebuilds every object)
    if not (force or _stale(HIP_LIB, srcs + _headers() + [__file__])):
        return HIP_LIB
    hipcc = _hipcc()
    obj_dir = os.path.join(LIB_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    hdrs = _headers() + [__file__]

    def compile_one(src: str) -> str:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if force or _stale(obj, [src] + hdrs):
            cmd = [hipcc, *HIP_FLAGS, *FILE_FLAGS.get(os.path.basename(src), []), "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            _run(cmd)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(srcs)))) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = HIP_LIB + ".tmp"
    _run([hipcc, f"--offload-arch={GPU_ARCH}", "-shared", "-fPIC", "-o", tmp, *objs])
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


COMM_LIB = os.path.join(LIB_DIR, "liblsknn_comm.so")


def build_comm(force: bool = False, verbose: bool = False) -> str:
    """Native RCCL communicator (csrc/comm): host C++ against the HIP runtime and the
    RCCL headers; RCCL itself is dlopen'ed at run time (no link-time dependency)."""
    srcs = _sources("comm", "cpp")
    if force or _stale(COMM_LIB, srcs + _headers()):
        os.makedirs(LIB_DIR, exist_ok=True)
        tmp = COMM_LIB + ".tmp"
        cmd = [_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", tmp, *srcs, "-ldl"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(tmp, COMM_LIB)
    return COMM_LIB


MPI_LIB = os.path.join(LIB_DIR, "liblsknn_mpi.so")


def mpi_home() -> str | None:
    """MPI installation with include/mpi.h and lib/libmpi.so: LSKNN_MPI_HOME, else the
    image's MPICH (/opt/conda); None when there is none (the MPI backend is optional)."""
    for home in (os.environ.get("LSKNN_MPI_HOME"), "/opt/conda"):
        if home and os.path.exists(os.path.join(home, "include", "mpi.h")) and \
                os.path.exists(os.path.join(home, "lib", "libmpi.so")):
            return home
    return None


def build_mpi(force: bool = False, verbose: bool = False) -> str | None:
    """Native MPI host communicator (csrc/mpi): plain C++ linked against the MPI library
    (rpath to it), loaded only when LSKNN_DIST_BACKEND=mpi."""
    home = mpi_home()
    if home is None:
        return None
    srcs = _sources("mpi", "cpp")
    if force or _stale(MPI_LIB, srcs):
        os.makedirs(LIB_DIR, exist_ok=True)
        tmp = MPI_LIB + ".tmp"
        lib = os.path.join(home, "lib")
        cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"-I{os.path.join(home, 'include')}",
               "-o", tmp, *srcs, f"-L{lib}", f"-Wl,-rpath,{lib}", "-lmpi"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(tmp, MPI_LIB)
    return MPI_LIB


# Measured-and-rejected experiments that a test still exercises (not part of the product
# library): scripts/micro/<name>.hip -> lib/exp/liblsknn_<name>.so
MICRO_DIR = os.path.join(os.path.dirname(PKG_DIR), "scripts", "micro")
MICRO_LIBS = ["screen_ab"]


def micro_lib(name: str) -> str:
    return os.path.join(LIB_DIR, "exp", f"liblsknn_{name}.so")


def build_micro(force: bool = False, verbose: bool = False) -> list[str]:
    out = []
    for name in MICRO_LIBS:
        src = os.path.join(MICRO_DIR, f"{name}.hip")
        lib = micro_lib(name)
        if os.path.exists(src) and (force or _stale(lib, [src] + _headers())):
            os.makedirs(os.path.dirname(lib), exist_ok=True)
            if verbose:
                print(f"[build] {os.path.basename(lib)}")
            tmp = lib + ".tmp"
            _run([_hipcc(), *HIP_FLAGS, "-I", os.path.join(CSRC, "hip"), "-I", CSRC, "-shared", src, "-o", tmp])
            os.replace(tmp, lib)
        out.append(lib)
    return out


def build_all(force: bool = False, verbose: bool = False) -> tuple[str, str]:
    build_comm(force, verbose)
    build_mpi(force, verbose)
    build_micro(force, verbose)
    return build_host(force, verbose), build_hip(force, verbose)


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(force=force, verbose=True):
        print(p)
    print(COMM_LIB)
