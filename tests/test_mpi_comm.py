"""MPI host communicator (parallel/mpi.py + csrc/mpi/mpi_comm.cpp, SURVEY §5.8 HostComm):
the reference's own launcher and transport — `mpirun -n P` with LSKNN_DIST_BACKEND=mpi —
on the CPU: every collective, the two apps in every mode bit-identical to one process,
and a failing rank ending the whole job (the reference's CUKD_MPI_CALL behaviour)."""
import os
import shutil
import subprocess
import sys

import pytest

from mpi_cuda_largescaleknn_amd import _build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIRUN = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
HAVE_MPI = os.path.exists(MPIRUN) and _build.mpi_home() is not None
pytestmark = pytest.mark.skipif(not HAVE_MPI, reason="no MPI installation (mpirun + mpi.h + libmpi)")

UN = "mpi_cuda_largescaleknn_amd.apps.unordered"
PRE = "mpi_cuda_largescaleknn_amd.apps.prepartitioned"
TOOLS = "mpi_cuda_largescaleknn_amd.apps.tools"


def mpirun(nproc, args, extra_env=None, check=True, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, LSKNN_DIST_BACKEND="mpi", **(extra_env or {}))
    env.pop("MASTER_PORT", None)
    p = subprocess.run([MPIRUN, "-n", str(nproc), sys.executable, *args], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=timeout)
    if check and p.returncode != 0:
        raise AssertionError(f"mpirun -n {nproc} {args} rc={p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


def plain(args):
    env = dict(os.environ, PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, "-m", *args], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    return p


@pytest.fixture(scope="module")
def data(tmp_path_factory):
    d = tmp_path_factory.mktemp("mpi")
    plain([TOOLS, "gen", str(d / "pts.float3"), "-n", "12000", "--dist", "clustered", "--seed", "5"])
    plain([UN, str(d / "pts.float3"), "-o", str(d / "ref.float"), "-k", "20", "--device", "cpu"])
    return d


@pytest.mark.parametrize("nproc,force", [(3, "0"), (1, "1")])
def test_collectives(nproc, force):
    """allreduce (sum/min/max), allgather, all-to-all-v with uneven and empty blocks in
    40-byte pieces, ring send/recv; on 1 rank forced: own-rank traffic through MPI."""
    p = mpirun(nproc, [os.path.join(ROOT, "tests", "workers", "mpi_collectives.py"), "cpu"],
               {"LSKNN_FORCE_DIST": force})
    assert sorted(p.stdout.split("\n")[:-1]) == [f"ok {r}" for r in range(nproc)]


@pytest.mark.parametrize("mode", ["auto", "ring"])
def test_unordered_over_mpi(data, mode):
    out = data / f"u_{mode}.float"
    p = mpirun(3, ["-m", UN, str(data / "pts.float3"), "-o", str(out), "-k", "20", "--device", "cpu",
                   "--mode", mode])
    assert p.stdout.count("done all queries...") == 3
    assert out.read_bytes() == (data / "ref.float").read_bytes()


@pytest.mark.parametrize("mode", ["auto", "peer"])
def test_prepartitioned_over_mpi(data, mode):
    pre = data / f"part_{mode}"
    plain([TOOLS, "split", str(data / "pts.float3"), "-p", "3", "-o", str(pre)])
    out = data / f"o_{mode}"
    p = mpirun(3, ["-m", PRE, str(pre) + ".list", "-o", str(out), "-k", "20", "--device", "cpu", "--mode", mode])
    assert "bounds is" in p.stdout
    got = b"".join((data / f"o_{mode}_{r:06d}.float").read_bytes() for r in range(3))
    assert got == (data / "ref.float").read_bytes()


def test_rank_failure_ends_the_job(data):
    """An exception on rank 1 inside the first all-to-all-v: that rank reports and exits 1,
    mpirun ends the job with a non-zero status (no hang of the ranks blocked in MPI)."""
    p = mpirun(3, ["-m", UN, str(data / "pts.float3"), "-o", str(data / "f.float"), "-k", "20", "--device", "cpu"],
               {"LSKNN_FAULT": "rank=1,op=alltoallv,call=0,kind=raise", "LSKNN_TIMEOUT": "60"}, check=False,
               timeout=200)
    assert p.returncode != 0
    assert "#1/3: error" in p.stderr


@pytest.mark.gpu
def test_gpu_two_ranks_one_gpu_over_mpi(data):
    """Two GPU ranks sharing one MI355X (RCCL refuses that; MPI host staging does not):
    the halo pipeline's device buffers go through MPI, output equals the CPU file."""
    out = data / "gpu2.float"
    p = mpirun(2, ["-m", UN, str(data / "pts.float3"), "-o", str(out), "-k", "20", "--device", "cuda"],
               timeout=240)
    assert p.stdout.count("done all queries...") == 2
    assert out.read_bytes() == (data / "ref.float").read_bytes()
