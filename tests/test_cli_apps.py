"""End-to-end CLI tests (CPU, gloo): the two entrypoints with the reference grammar,
file formats, multi-process launch via torchrun, and the cross-variant identity of
SURVEY §2.7 C9 (prePartitioned on the P slices of a file, concatenated == unordered)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

from mpi_cuda_largescaleknn_amd.utils import io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT)


def port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run(args, nproc=1, cwd=None, check=True):
    if nproc == 1:
        cmd = [sys.executable, "-m"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={port()}", "-m"] + args
    p = subprocess.run(cmd, cwd=cwd, env=ENV, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=600)
    if check and p.returncode != 0:
        raise AssertionError(f"{cmd} failed rc={p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


UN = "mpi_cuda_largescaleknn_amd.apps.unordered"
PRE = "mpi_cuda_largescaleknn_amd.apps.prepartitioned"
TOOLS = "mpi_cuda_largescaleknn_amd.apps.tools"


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    run([TOOLS, "gen", str(d / "pts.float3"), "-n", "12000", "--dist", "clustered", "--seed", "3"])
    run([UN, str(d / "pts.float3"), "-o", str(d / "ref.float"), "-k", "20", "--device", "cpu"])
    return d


def test_single_process_output_matches_oracle(data):
    p = run([TOOLS, "check", str(data / "pts.float3"), str(data / "ref.float"), "-k", "20", "--samples", "3000"])
    assert "0 mismatches" in p.stdout
    assert io.read_floats(str(data / "ref.float")).shape[0] == 12000


def test_usage_errors_exit_1(data):
    p = run([UN, str(data / "pts.float3"), "-k", "3"], check=False)
    assert p.returncode == 1 and p.stderr.startswith("Error: no output file name specified")
    p = run([PRE, "-o", "x", "-k", "3"], check=False)
    assert p.returncode == 1 and "list of input files" in p.stderr


@pytest.mark.parametrize("mode", ["auto", "ring"])
def test_unordered_three_ranks(data, mode):
    out = data / f"u3_{mode}.float"
    p = run([UN, str(data / "pts.float3"), "-o", str(out), "-k", "20", "--device", "cpu", "--mode", mode], nproc=3)
    assert p.stdout.count("done all queries...") == 3
    assert torch.equal(io.read_floats(str(out)), io.read_floats(str(data / "ref.float")))


@pytest.mark.parametrize("mode", ["auto", "peer"])
def test_prepartitioned_cross_variant_identity(data, mode):
    pre = data / f"part_{mode}"
    run([TOOLS, "split", str(data / "pts.float3"), "-p", "3", "-o", str(pre)])  # contiguous slices
    out = data / f"o_{mode}"
    p = run([PRE, str(pre) + ".list", "-o", str(out), "-k", "20", "--device", "cpu", "--mode", mode], nproc=3)
    assert "bounds is" in p.stdout
    if mode == "peer":
        assert "round 0" in p.stdout
    cat = data / f"cat_{mode}.float"
    run([TOOLS, "cat", str(out), "3", str(cat)])
    r = run([TOOLS, "cmp", str(cat), str(data / "ref.float")])
    assert "identical" in r.stdout


def test_rank_count_must_match_file_list(data):
    lst = data / "two.list"
    lst.write_text(f"{data / 'pts.float3'}\n{data / 'pts.float3'}")  # 2 files, no trailing newline
    p = run([PRE, str(lst), "-o", str(data / "x"), "-k", "5", "--device", "cpu"], nproc=3, check=False)
    assert p.returncode != 0
    assert "number of input files does not match MPI size" in p.stderr


def test_bootstrap_spawn_matches_single(data):
    """--bootstrap spawn --nproc 3: the launcher starts its own 3 local ranks (no torchrun)."""
    out = data / "spawn.float"
    p = run([UN, str(data / "pts.float3"), "-o", str(out), "-k", "20", "--device", "cpu",
             "--bootstrap", "spawn", "--nproc", "3"])
    assert "#2/3: got" in p.stdout
    assert out.read_bytes() == (data / "ref.float").read_bytes()


def test_prepartitioned_spawn_balance_on(data, tmp_path):
    pts = io.read_points(str(data / "pts.float3"))
    names = []
    for r, (b, e) in enumerate([(0, 9000), (9000, 10000), (10000, 12000)]):  # skewed files
        f = tmp_path / f"part{r}.float3"
        io.write_points(str(f), pts[b:e])
        names.append(str(f))
    (tmp_path / "list.txt").write_text("\n".join(names) + "\n")
    run([PRE, str(tmp_path / "list.txt"), "-o", str(tmp_path / "out"), "-k", "20", "--device", "cpu",
         "--bootstrap", "spawn", "--nproc", "3", "--balance", "on"])
    got = b"".join((tmp_path / f"out_{r:06d}.float").read_bytes() for r in range(3))
    assert got == (data / "ref.float").read_bytes()


@pytest.mark.parametrize("bad,msg", [(["--bootstrap", "slurm"], "invalid --bootstrap"),
                                     (["--nproc", "2"], "go together"),
                                     (["--device-map", "0,,1"], "invalid --device-map"),
                                     (["--balance", "yes"], "invalid --balance")])
def test_extension_flag_errors(data, bad, msg):
    p = run([UN, str(data / "pts.float3"), "-o", "x.float", "-k", "4"] + bad, check=False)
    assert p.returncode == 1 and msg in p.stderr


def test_device_map_and_bootstrap_env():
    from mpi_cuda_largescaleknn_amd.parallel import launch as L

    assert L.pick_device(5, 1, 8, 0, [3, 2]) == 2
    assert L.pick_device(5, 1, 8, 4, None) == 1       # reference -g: rank % G
    assert L.pick_device(5, 1, 8, 0, None) == 1       # local rank
    env = {"PMI_RANK": "2", "PMI_SIZE": "4", "RANK": "0", "WORLD_SIZE": "1"}
    old = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update(env)
        assert L.rank_info("mpi")[:2] == (2, 4)
        assert L.rank_info("env")[:2] == (0, 1)
        assert L.rank_info("auto")[:2] == (0, 1)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["nccl", "rccl"])
def test_gpu_app_forced_rccl_matches_cpu(data, backend):
    """The unordered app on the GPU through its multi-rank path on a forced 1-rank RCCL
    group (torch.distributed "nccl" or the native communicator "rccl"): same output file
    as the CPU single-process run."""
    out = data / f"gpu_{backend}.float"
    env = dict(ENV, LSKNN_FORCE_DIST="1", LSKNN_DIST_BACKEND=backend, MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port()))
    p = subprocess.run([sys.executable, "-m", UN, str(data / "pts.float3"), "-o", str(out), "-k", "20",
                        "--device", "cuda"], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    assert out.read_bytes() == (data / "ref.float").read_bytes()


STREAM = "mpi_cuda_largescaleknn_amd.apps.stream"


@pytest.mark.parametrize("nproc", [1, 3])
def test_stream_app_matches_unordered_per_file(data, tmp_path, nproc):
    """hipKNN_stream over three files (one repeated): each output file has the same bytes as
    hipKNN_unorderedData run on that file alone."""
    run([TOOLS, "gen", str(tmp_path / "b.float3"), "-n", "5000", "--seed", "9"])
    run([UN, str(tmp_path / "b.float3"), "-o", str(tmp_path / "b_ref.float"), "-k", "20", "--device", "cpu"])
    files = [str(data / "pts.float3"), str(tmp_path / "b.float3"), str(data / "pts.float3")]
    p = run([STREAM, *files, "-o", str(tmp_path / "s"), "-k", "20", "--device", "cpu"], nproc=nproc)
    assert p.stdout.count("done all queries...") == nproc
    refs = [data / "ref.float", tmp_path / "b_ref.float", data / "ref.float"]
    for i, ref in enumerate(refs):
        assert (tmp_path / f"s_{i:06d}.float").read_bytes() == ref.read_bytes(), i


def test_stream_app_errors(data, tmp_path):
    p = run([STREAM, str(data / "pts.float3"), "-o", str(tmp_path / "x"), "-k", "0"], check=False)
    assert p.returncode != 0
    p = run([STREAM, str(tmp_path / "missing.float3"), "-o", str(tmp_path / "x"), "-k", "4", "--device", "cpu"],
            check=False)
    assert p.returncode == 1


@pytest.mark.gpu
def test_stream_app_gpu_matches_cpu(data, tmp_path):
    files = [str(data / "pts.float3"), str(data / "pts.float3")]
    run([STREAM, *files, "-o", str(tmp_path / "g"), "-k", "20", "--device", "cuda"])
    for i in range(2):
        assert (tmp_path / f"g_{i:06d}.float").read_bytes() == (data / "ref.float").read_bytes()
