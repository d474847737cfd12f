"""T0 unit tests of the native host runtime: CLI grammar, file I/O partition math,
file lists and the prePartitioned peer schedule."""
import ctypes
import ctypes.util
import math
import os

import pytest
import torch

from mpi_cuda_largescaleknn_amd import _native
from mpi_cuda_largescaleknn_amd.utils import cli, io

SYN = "./mpiHugeQuery -k <k> [-r <maxRadius>] in.float3s -o out.dat\n"


# --------------------------------------------------------------------------- CLI
def test_cli_basic_unordered():
    a = cli.parse(cli.UNORDERED, ["prog", "pts.float3", "-o", "out.float", "-k", "100"])
    assert (a.input, a.output, a.k) == ("pts.float3", "out.float", 100)
    assert math.isinf(a.max_radius) and a.gpu_affinity == 0 and a.mode == "auto"


def test_cli_last_positional_wins_and_flags():
    a = cli.parse(cli.UNORDERED, ["p", "a.f3", "-k", "8", "b.f3", "-r", "0.5", "-g", "8", "-o", "o"])
    assert a.input == "b.f3" and a.max_radius == pytest.approx(0.5) and a.gpu_affinity == 8


@pytest.mark.parametrize("argv,msg", [
    (["p", "-o", "o", "-k", "3"], "no input file name specified"),
    (["p", "in", "-k", "3"], "no output file name specified"),
    (["p", "in", "-o", "o"], "no k specified, or invalid k value"),
    (["p", "in", "-o", "o", "-k", "0"], "no k specified, or invalid k value"),
    (["p", "in", "-o", "o", "-k", "2", "-x"], "unknown cmdline arg '-x'"),
    (["p", "in", "-o", "o", "-k", "2", "-h"], "unknown cmdline arg '-h'"),
])
def test_cli_errors_match_reference_text(argv, msg):
    with pytest.raises(cli.UsageError) as e:
        cli.parse(cli.UNORDERED, argv)
    assert e.value.code == 1
    assert e.value.text == f"Error: {msg}\n\n{SYN}"


def test_cli_prepartitioned_error_strings():
    with pytest.raises(cli.UsageError) as e:
        cli.parse(cli.PREPARTITIONED, ["p", "-o", "x", "-k", "1"])
    assert "should be a text file with list of input files" in e.value.text
    with pytest.raises(cli.UsageError) as e:
        cli.parse(cli.PREPARTITIONED, ["p", "list.txt", "-k", "1"])
    assert "no output file(s) prefix specified" in e.value.text


def test_cli_missing_value_is_an_error_not_ub():
    with pytest.raises(cli.UsageError) as e:
        cli.parse(cli.UNORDERED, ["p", "in", "-k", "3", "-o"])
    assert "missing value" in e.value.text


def test_cli_extensions():
    a = cli.parse(cli.UNORDERED, ["p", "in", "-o", "o", "-k", "1", "--mode", "ring", "--device", "cpu", "-v",
                                  "--stats", "s.json"])
    assert (a.mode, a.device, a.verbose, a.stats) == ("ring", "cpu", True, "s.json")
    with pytest.raises(cli.UsageError):
        cli.parse(cli.UNORDERED, ["p", "in", "-o", "o", "-k", "1", "--mode", "bogus"])


# --------------------------------------------------------------------------- I/O
def _write_bytes(path, nbytes):
    with open(path, "wb") as f:
        f.write(os.urandom(nbytes))


@pytest.mark.parametrize("nrec,extra", [(0, 0), (1, 0), (10, 5), (1000, 11), (12345, 1)])
@pytest.mark.parametrize("size", [1, 2, 3, 7, 8])
def test_portion_matches_reference_formula(tmp_path, nrec, extra, size):
    p = str(tmp_path / "x.float3")
    _write_bytes(p, nrec * 12 + extra)
    covered = 0
    for r in range(size):
        b, c, t = io.portion(p, r, size)
        assert t == nrec
        assert b == nrec * r // size and b + c == nrec * (r + 1) // size
        covered += c
    assert covered == nrec


def test_read_write_roundtrip_and_trailing_bytes(tmp_path):
    p = str(tmp_path / "pts.float3")
    pts = torch.rand(1001, 3)
    io.write_points(p, pts)
    with open(p, "ab") as f:
        f.write(b"\x01\x02\x03")  # trailing partial record is ignored
    got, begin, total = io.read_portion(p, 1, 3)
    assert total == 1001 and begin == 1001 // 3
    assert torch.equal(got, pts[begin:begin + got.shape[0]])
    assert torch.equal(io.read_points(p), pts)


def test_parallel_pwrite_equals_serial_append(tmp_path):
    vals = torch.rand(10007)
    p = str(tmp_path / "out.float")
    size = 5
    # rank 0 truncates & sizes the file, every rank writes its block at begin*4
    io.write_floats(p, vals[:0], 0, truncate=True, total_records=vals.numel())
    for r in reversed(range(size)):
        b, e = vals.numel() * r // size, vals.numel() * (r + 1) // size
        io.write_floats(p, vals[b:e], b, truncate=False)
    assert torch.equal(io.read_floats(p), vals)


@pytest.mark.parametrize("content,expected", [
    ("a\nb\nc\n", ["a", "b", "c"]),
    ("a\nb\nc", ["a", "b", "c"]),          # reference drops 'c' (SURVEY D11): fixed
    ("a\r\nb\r\n", ["a", "b"]),            # CRLF
    ("a\n\nb\n\n", ["a", "b"]),            # blank lines carry no rank
    ("", []),
])
def test_file_list(tmp_path, content, expected):
    p = tmp_path / "list.txt"
    p.write_text(content)
    assert io.read_file_list(str(p)) == expected


# --------------------------------------------------------------------------- peer schedule
def _ref_permutation(rank, size):
    libc = ctypes.CDLL(ctypes.util.find_library("c"))
    libc.srand(rank + 0x1234567)
    for _ in range(10):
        libc.rand()
    ret = list(range(size))
    for i in range(size - 1, 0, -1):
        other = libc.rand() % i
        ret[other], ret[i] = ret[i], ret[other]
    return ret


@pytest.mark.parametrize("size", [1, 2, 5, 8, 12])
def test_peer_permutation_matches_glibc_sattolo(size):
    lib = _native.host()
    for rank in range(size):
        out = (ctypes.c_int * size)()
        lib.lsk_peer_permutation(rank, size, out)
        assert list(out) == _ref_permutation(rank, size)
        # Sattolo's shuffle yields a single cycle
        if size > 1:
            seen, x = set(), 0
            while x not in seen:
                seen.add(x)
                x = out[x]
            assert len(seen) == size


def _box_dist(a, b):
    d = [max(0.0, a[i] - b[3 + i], b[i] - a[3 + i]) for i in range(3)]
    return math.sqrt(sum(x * x for x in d))


def test_peer_choose_matches_reference_rule():
    lib = _native.host()
    g = torch.Generator().manual_seed(0)
    for trial in range(50):
        size = 6
        lo = torch.rand((size, 3), generator=g) * 4
        boxes = torch.cat([lo, lo + torch.rand((size, 3), generator=g)], 1).contiguous()
        me = trial % size
        seen = (ctypes.c_uint8 * size)(*[1 if (j == me or (trial + j) % 4 == 0) else 0 for j in range(size)])
        perm = (ctypes.c_int * size)(*_ref_permutation(me, size))
        cutoff = float(torch.rand(1, generator=g)) * 3
        got = lib.lsk_peer_choose(boxes[me].contiguous().data_ptr(), boxes.data_ptr(), size,
                                  ctypes.c_float(cutoff), ctypes.addressof(seen), ctypes.addressof(perm))
        best, closest = -1, math.inf
        for peer in perm:
            if seen[peer]:
                continue
            d = _box_dist(boxes[me].tolist(), boxes[peer].tolist())
            if d >= cutoff or d >= closest:
                continue
            best, closest = peer, d
        assert got == best


def test_native_host_unit_tests(tmp_path):
    """The C++ host unit-test binary (CTest target host_tests) builds and passes."""
    import subprocess

    from mpi_cuda_largescaleknn_amd import _build
    lib = _build.build_host()
    src = os.path.join(_build.CSRC, "tests", "host_tests.cpp")
    exe = str(tmp_path / "host_tests")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(_build.CSRC, "host"),
                    src, "-o", exe, lib, f"-Wl,-rpath,{os.path.dirname(lib)}"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "host tests passed" in r.stdout


def test_roctx_trace_is_safe_without_profiler():
    from mpi_cuda_largescaleknn_amd.utils import trace
    assert isinstance(trace.available(), bool)
    trace.mark("lsknn:test")
    with trace.range("lsknn:test-range"):
        pass


# --------------------------------------------------------------------------- curve keys
def _cell_keys(coords, curve):
    """Curve keys of grid cells (integer coords in [0, 1024)^3) via the C++ encoder."""
    from mpi_cuda_largescaleknn_amd.ops import kernels as K
    pts = (coords.to(torch.float32) + 0.5) / 1024.0
    box = torch.tensor([0, 0, 0, 1, 1, 1, 1024.0, 1.0], dtype=torch.float32)
    keys, _ = K.morton(pts, box, with_iota=False, curve=curve)
    return keys.to(torch.int64) & 0xFFFFFFFF


@pytest.mark.parametrize("corner", [(0, 0, 0), (992, 0, 480), (512, 512, 512)])
def test_hilbert_cell_block_is_a_face_connected_path(corner):
    """A 32^3 octree cell maps to one aligned block of 32^3 consecutive Hilbert keys
    (what splitter snapping relies on), and consecutive keys are face neighbours."""
    r = torch.arange(32)
    g = torch.stack(torch.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3) + torch.tensor(corner)
    keys = _cell_keys(g, "hilbert")
    order = torch.argsort(keys)
    ks = keys[order]
    assert int(ks[0]) % (1 << 15) == 0
    assert torch.equal(ks - ks[0], torch.arange(1 << 15))
    steps = (g[order][1:] - g[order][:-1]).abs().sum(1)
    assert bool((steps == 1).all())


def test_morton_key_bit_interleave():
    c = torch.tensor([[1, 0, 0], [0, 1, 0], [0, 0, 1], [1023, 1023, 1023]])
    assert _cell_keys(c, "morton").tolist() == [4, 2, 1, (1 << 30) - 1]


def test_cmake_build_and_ctest(tmp_path):
    """B01: the CMake build (same flags as _build.py) configures, compiles the gfx950
    library and the host library, and its CTest host suite passes."""
    import shutil
    import subprocess

    if shutil.which("cmake") is None or shutil.which("ninja") is None:
        pytest.skip("cmake/ninja not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    b = str(tmp_path / "build")
    for cmd in (["cmake", "-S", root, "-B", b, "-G", "Ninja"],
                ["cmake", "--build", b, "-j8"],
                ["ctest", "--test-dir", b, "--output-on-failure"]):
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, f"{' '.join(cmd)} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    assert os.path.exists(os.path.join(b, "liblsknn_hip.so"))
    assert os.path.exists(os.path.join(b, "liblsknn_host.so"))


def test_cmake_sanitized_host_ctest(tmp_path):
    """the host runtime and its unit tests built with
    -DLSKNN_SANITIZE=address;undefined pass CTest (CPU code only)."""
    import shutil
    import subprocess

    if shutil.which("cmake") is None or shutil.which("ninja") is None:
        pytest.skip("cmake/ninja not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    b = str(tmp_path / "build_san")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    for cmd in (["cmake", "-S", root, "-B", b, "-G", "Ninja", "-DLSKNN_SANITIZE=address;undefined",
                 "-DCMAKE_BUILD_TYPE=RelWithDebInfo"],
                ["cmake", "--build", b, "-j8", "--target", "lsknn_host_tests"],
                ["ctest", "--test-dir", b, "--output-on-failure"]):
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, f"{' '.join(cmd)} failed:\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    flags = open(os.path.join(b, "build.ninja")).read()
    assert "-fsanitize=address,undefined" in flags
