"""Failure detection and fault injection (SURVEY §5.3, §4.2 "Fault injection"): a rank
that fails, crashes or hangs must end the whole job with a non-zero exit status and a
message, and no rank may stay blocked. CPU, gloo, 2-3 processes via torchrun."""
import os
import socket
import subprocess
import sys
import time

import pytest

from mpi_cuda_largescaleknn_amd.parallel import faults as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UN = "mpi_cuda_largescaleknn_amd.apps.unordered"
PRE = "mpi_cuda_largescaleknn_amd.apps.prepartitioned"
TOOLS = "mpi_cuda_largescaleknn_amd.apps.tools"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, nproc, env_extra=None, timeout=240):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m"] + args
    t = time.monotonic()
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    return p, time.monotonic() - t


@pytest.fixture(scope="module")
def pts(tmp_path_factory):
    d = tmp_path_factory.mktemp("faults")
    f = d / "pts.float3"
    subprocess.run([sys.executable, "-m", TOOLS, "gen", str(f), "-n", "6000", "--seed", "1"],
                   env=dict(os.environ, PYTHONPATH=ROOT), check=True)
    return f


def test_parse_fault_spec():
    assert F.parse_fault(None) is None
    f = F.parse_fault("rank=1,op=alltoallv,call=2,kind=hang")
    assert f == {"rank": 1, "op": "alltoallv", "call": 2, "kind": "hang"}
    assert F.parse_fault("rank=0")["op"] == "*"
    with pytest.raises(ValueError):
        F.parse_fault("op=barrier")
    with pytest.raises(ValueError):
        F.parse_fault("rank=0,kind=explode")


@pytest.mark.parametrize("kind,code", [("raise", 1), ("exit", 7)])
def test_injected_failure_ends_job(pts, tmp_path, kind, code):
    p, dt = _run([UN, str(pts), "-o", str(tmp_path / "o.float"), "-k", "8", "--device", "cpu"], 2,
                 {"LSKNN_FAULT": f"rank=1,op=alltoallv,call=0,kind={kind}"})
    assert p.returncode != 0
    assert "injected fault" in p.stderr
    assert "#1/2" in p.stderr
    assert dt < 200


def test_hang_is_caught_by_watchdog(pts, tmp_path):
    p, dt = _run([UN, str(pts), "-o", str(tmp_path / "o.float"), "-k", "8", "--device", "cpu"], 2,
                 {"LSKNN_FAULT": "rank=0,op=alltoallv,kind=hang", "LSKNN_TIMEOUT": "6"})
    assert p.returncode != 0
    assert "injected fault (hang)" in p.stderr
    # whichever fires first: this rank's watchdog, or the peer's collective timeout
    # (which then broadcasts its failure)
    assert any(m in p.stderr for m in ("watchdog: no progress", "aborting", "#1/2: error"))
    assert dt < 200


def test_missing_input_file_on_one_rank(pts, tmp_path):
    lst = tmp_path / "files.txt"
    lst.write_text(f"{pts}\n{tmp_path / 'does_not_exist.float3'}\n")
    p, dt = _run([PRE, str(lst), "-o", str(tmp_path / "out"), "-k", "8", "--device", "cpu"], 2)
    assert p.returncode != 0
    assert "#1/2: error:" in p.stderr
    assert dt < 200


def test_rank_count_mismatch_message(pts, tmp_path):
    lst = tmp_path / "files.txt"
    lst.write_text(f"{pts}\n")
    p, _ = _run([PRE, str(lst), "-o", str(tmp_path / "out"), "-k", "8", "--device", "cpu"], 2)
    assert p.returncode != 0
    assert "number of input files does not match MPI size" in p.stderr


def test_watchdog_aborts_on_communicator_error(tmp_path):
    """The watchdog polls the communicator's asynchronous error state (native RCCL:
    ncclCommGetAsyncError); on an error it runs the abort hook (ncclCommAbort) and the
    rank exits with EXIT_COMM_ERROR."""
    import subprocess
    import sys

    flag = tmp_path / "aborted"
    code = (
        "import time\n"
        "from mpi_cuda_largescaleknn_amd.parallel import faults as F\n"
        "n = [0]\n"
        "def check():\n"
        "    n[0] += 1\n"
        "    return 'RCCL async error 6: remote process exited' if n[0] >= 3 else None\n"
        f"F.Watchdog(0, 2, None, timeout=60, poll=0.05, comm_check=check,\n"
        f"           on_abort=lambda: open({str(flag)!r}, 'w').write('x')).start()\n"
        "time.sleep(30)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=root)
    assert out.returncode == 5, (out.returncode, out.stderr)
    assert "remote process exited" in out.stderr
    assert flag.exists()


def test_watchdog_skips_long_host_phase():
    """a long local host phase (data generation, a library build) is not a hang:
    inside HEARTBEAT.host_phase the progress timeout does not run; after it, idle time
    counts again and the rank exits with EXIT_TIMEOUT naming the last op."""
    import subprocess
    import sys

    code = (
        "import time\n"
        "from mpi_cuda_largescaleknn_amd.parallel import faults as F\n"
        "F.Watchdog(0, 2, None, timeout=0.5, poll=0.05).start()\n"
        "with F.HEARTBEAT.host_phase('make_points'):\n"
        "    time.sleep(2.0)\n"
        "print('phase done', flush=True)\n"
        "F.HEARTBEAT.beat('alltoallv')\n"
        "time.sleep(30)\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=root)
    assert "phase done" in out.stdout, out.stderr
    assert out.returncode == F.EXIT_TIMEOUT, (out.returncode, out.stderr)
    assert "timeout in alltoallv" in out.stderr


def test_bench_hang_names_the_collective():
    """bench.py's own progress timeout (bench.BENCH_TIMEOUT_S = 150 s, well under the
    driver's 600 s; shortened here through LSKNN_TIMEOUT): a rank hung in a collective
    ends the self-launched job non-zero, and the kept tail names the rank and the op."""
    import bench

    assert bench.BENCH_TIMEOUT_S <= 200
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2",
               LSKNN_FAULT="rank=1,op=alltoallv,kind=hang", LSKNN_TIMEOUT="8")
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    t = time.monotonic()
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--device", "cpu", "--points", "2e4", "--k", "8",
                        "--steps", "1", "--warmup", "0", "--verify", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    dt = time.monotonic() - t
    assert p.returncode != 0
    assert "#1/2: injected fault (hang) in alltoallv" in p.stderr
    assert "timeout in alltoallv" in p.stderr or "timed out in alltoallv" in p.stderr, p.stderr[-2000:]
    assert dt < 150
