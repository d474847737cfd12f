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
