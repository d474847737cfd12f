"""The two build descriptions ship the same kernels: the per-file compile flags of
CMakeLists.txt must equal _build.py FILE_FLAGS (the in-tree build the benchmarks measure),
and both carry the exactness flags (-ffp-contract=off, no fast-math)."""
import os
import re

import pytest

from mpi_cuda_largescaleknn_amd import _build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cmake_file_flags() -> dict:
    text = open(os.path.join(ROOT, "CMakeLists.txt")).read()
    out = {}
    for m in re.finditer(r"set_source_files_properties\(\$\{CSRC\}/hip/(\S+)\s+PROPERTIES\s+COMPILE_OPTIONS\s+"
                         r"\"([^\"]*)\"\)", text):
        out[m.group(1)] = [f for f in m.group(2).split(";") if f]
    return out


def test_cmake_per_file_flags_match_build_py():
    assert _cmake_file_flags() == {k: list(v) for k, v in B.FILE_FLAGS.items()}


def test_every_flagged_file_exists():
    for name in B.FILE_FLAGS:
        assert os.path.exists(os.path.join(B.CSRC, "hip", name)), name


def test_exactness_flags_in_both():
    text = open(os.path.join(ROOT, "CMakeLists.txt")).read()
    assert "-ffp-contract=off" in text and "-fno-fast-math" in text
    assert "-ffp-contract=off" in B.COMMON_FLAGS and "-fno-fast-math" in B.COMMON_FLAGS
    assert re.search(r"CMAKE_HIP_ARCHITECTURES\s+gfx950", text) and B.GPU_ARCH == "gfx950"


def test_hip_library_builds():
    """The gfx950 kernel library compiles from the tree's sources (a no-op when the in-tree
    library is newer than every source; otherwise hipcc cross-compiles it here)."""
    import shutil
    if not (os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    path = B.build_hip()
    assert os.path.exists(path)


def test_flag_change_rebuilds_hip_objects(monkeypatch):
    """FILE_FLAGS live in _build.py: the library and every object depend on that file, so a
    changed compile flag cannot leave an object built with the old flags in the library."""
    seen = []

    def fake_stale(target, deps):
        seen.append((os.path.basename(target), list(deps)))
        return False  # nothing to rebuild: only the dependency lists are checked

    monkeypatch.setattr(B, "_stale", fake_stale)
    B.build_hip()
    assert seen and seen[0][0] == os.path.basename(B.HIP_LIB)
    assert os.path.abspath(B.__file__) in [os.path.abspath(d) for d in seen[0][1]]
