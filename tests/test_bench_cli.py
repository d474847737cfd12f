"""bench.py contract rehearsal on the CPU: the multi-rank launch path the driver uses
(torch.distributed.run, one process per rank, barrier + max-over-ranks timing, one JSON
line from rank 0), with the gloo backend and CPU tensors instead of RCCL and GPUs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{\"metric\"")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_single_rank_cpu():
    out = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--points", "20000", "--k", "8",
                          "--steps", "2", "--warmup", "1"], cwd=ROOT, env=_env(), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 1 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    assert rec["config"]["all_finite"] is True
    assert rec["config"]["sampled_exact"] == "256/256"
    assert "(k=8) on 0.02M float3" in rec["metric"]
    assert rec["detail"]["phase_ms_max_over_ranks"]["knn_local"] > 0
    assert rec["config"]["knn_kernels"] == ["cpu"]


@pytest.mark.gpu
@pytest.mark.parametrize("graph", ["1", "0"])
def test_bench_single_gpu_graph_and_eager(graph):
    """The driver's default single-GPU bench path: the step captured as a HIP graph (or
    eager), distances finite, the graph flag reported."""
    out = subprocess.run([sys.executable, "bench.py", "--points", "300000", "--steps", "3", "--warmup", "1",
                          "--graph", graph, "--pipeline", "0"], cwd=ROOT, env=_env(), capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 1 and rec["value"] > 0
    assert rec["config"]["all_finite"] is True
    assert rec["config"]["hip_graph"] is (graph == "1")
    assert rec["config"]["sampled_exact"] == "256/256"
    # the kernels that ran are reported in graph mode too (captured launches)
    assert rec["config"]["knn_kernels"], rec["config"]
    assert rec["config"]["hw_queues"] >= 8


@pytest.mark.gpu
def test_bench_single_gpu_pipelined():
    """The single-GPU bench as a stream of two alternating point sets, step i+1's
    upload under step i's k-NN; both sets' outputs of the last two steps are checked."""
    out = subprocess.run([sys.executable, "bench.py", "--points", "300000", "--steps", "3", "--warmup", "1",
                          "--pipeline", "1"],  # (the default turns the stream on from 1e7 points)
                         cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["config"]["pipelined"] is True and rec["config"]["hip_graph"] is False
    assert rec["config"]["all_finite"] is True
    assert rec["config"]["sampled_exact"] == "512/512"
    assert "two different point sets" in rec["data"]
    assert "grid" in rec["config"]["knn_kernels"]  # uniform points: the cell-grid kernel


@pytest.mark.gpu
def test_bench_pipelined_forced_rccl_single_gpu():
    """--pipeline 1 on the multi-rank path (1-rank RCCL group): device-resident input per
    step, plain (non-streamed) redistribution beside the previous set's k-NN, both sets
    exact."""
    out = subprocess.run([sys.executable, "bench.py", "--points", "300000", "--steps", "2", "--warmup", "1",
                          "--force-dist", "--pipeline", "1"],
                         cwd=ROOT, env=dict(_env(), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port())),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["config"]["pipelined"] is True
    assert rec["config"]["sampled_exact"] == "512/512"


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["nccl", "rccl"])
def test_bench_forced_rccl_single_gpu(backend):
    """One rank through the multi-rank pipeline on a real 1-rank RCCL group: every
    collective of the step (all-reduce, all-gather, all-to-all-v) runs on RCCL — through
    torch.distributed ("nccl") or the native communicator ("rccl", parallel/rccl.py)."""
    out = subprocess.run([sys.executable, "bench.py", "--points", "300000", "--steps", "2", "--warmup", "1",
                          "--force-dist", "--pipeline", "0"], cwd=ROOT, env=dict(_env(), MASTER_ADDR="127.0.0.1",
                                                               MASTER_PORT=str(_free_port()),
                                                               LSKNN_DIST_BACKEND=backend),
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["config"]["hip_graph"] is False
    assert rec["config"]["sampled_exact"] == "256/256"
    assert "alltoallv_points" in rec["detail"]["phase_ms_max_over_ranks"]
    assert rec["config"]["comm"] == backend
    # which RCCL library moved the data: torch's bundled one or ROCm's (native communicator)
    v = rec["config"]["comm_info"]["rccl_version"]
    assert v and v.split(".")[0] == "2", rec["config"]["comm_info"]


@pytest.mark.gpu
@pytest.mark.parametrize("lib", ["default", "broken"])
def test_bench_default_backend_single_gpu(lib):
    """No LSKNN_DIST_BACKEND: the native communicator is the GPU data path; if it cannot
    come up (here: LSKNN_RCCL_LIB names a file that is no RCCL library) every rank agrees
    over gloo to fall back to torch's RCCL group, and the run still completes."""
    env = dict(_env(), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.pop("LSKNN_DIST_BACKEND", None)
    if lib == "broken":
        env["LSKNN_RCCL_LIB"] = os.path.join(ROOT, "bench.py")
    out = subprocess.run([sys.executable, "bench.py", "--points", "300000", "--steps", "2", "--warmup", "1",
                          "--force-dist", "--pipeline", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["config"]["sampled_exact"] == "256/256"
    want = "rccl" if lib == "default" else "nccl"
    assert rec["config"]["comm_info"]["backend"] == want, rec["config"]["comm_info"]
    if lib == "broken":
        assert "native RCCL communicator unavailable" in out.stdout + out.stderr


@pytest.mark.parametrize("variant", ["unordered", "prepartitioned"])
def test_bench_two_ranks_torchrun_gloo(variant):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--device", "cpu", "--points", "30000", "--k", "16", "--steps", "2", "--warmup", "1",
           "--variant", variant]
    out = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 2
    assert rec["config"]["global_batch"] == 30000
    assert rec["config"]["all_finite"] is True
    assert rec["ms_per_step"] > 0
    d = rec["detail"]
    assert len(d["knn_local_ms_per_rank"]) == 2
    assert sum(d["owned_points_per_rank"]) == 30000
    if variant == "unordered":
        assert rec["config"]["sampled_exact"] == "256/256"
        assert d["redistributed_bytes"] > 0


def test_bench_global_set_independent_of_rank_count():
    import torch
    sys.path.insert(0, ROOT)
    import bench
    cpu = torch.device("cpu")
    bench.GEN_CHUNK = 7000  # several chunk boundaries inside every block
    one = bench.make_points(50000, 0, 1, cpu, "unordered")
    parts = [bench.make_points(50000, r, 3, cpu, "unordered") for r in range(3)]
    assert torch.equal(torch.cat(parts), one)


def test_bench_four_ranks_streamed_uneven_chunks():
    """4 gloo ranks, 30001 points, forced streaming with 7500-point chunks: ranks hold
    7500 or 7501 points, i.e. one or two chunks — the agreed chunk count keeps their
    collective sequences equal; all sampled outputs exact."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "4",
           "--device", "cpu", "--points", "30001", "--k", "12", "--steps", "1", "--warmup", "1"]
    env = dict(_env(), LSKNN_FORCE_STREAM="1", LSKNN_STREAM_CHUNK="7500")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 4 and rec["config"]["global_batch"] == 30001
    assert rec["config"]["sampled_exact"] == "256/256"
    assert sum(rec["detail"]["owned_points_per_rank"]) == 30001


@pytest.mark.gpu
def test_bench_two_gpu_ranks_pipelined_gloo():
    """The driver's multi-rank launch (torchrun, 2 ranks) with the default pipelined
    stream, both ranks on the one GPU of the box over a host-staged gloo group (RCCL
    refuses two ranks on one device): both sets' sampled outputs exact."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--points", "400000", "--steps", "3", "--warmup", "1", "--pipeline", "1"]
    out = subprocess.run(cmd, cwd=ROOT, env=dict(_env(), LSKNN_DIST_BACKEND="gloo"), capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["pipelined"] is True
    assert rec["config"]["all_finite"] is True
    assert rec["config"]["sampled_exact"] == "512/512"
    assert sum(rec["detail"]["owned_points_per_rank"]) == 400000


def test_bench_self_launches_gpus_ranks_on_cpu():
    """`bench.py --gpus 4` with no launcher environment starts 4 local ranks itself (the
    reference's `mpirun -n P`, README.md:31,39) and reports them; no torchrun involved."""
    env = _env()
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--device", "cpu", "--points", "3e4",
                          "--steps", "2", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 4 and rec["config"]["ranks"] == 4
    assert rec["config"]["comm"] == "gloo"
    assert rec["config"]["comm_info"]["backend"] == "gloo"
    assert rec["config"]["sampled_exact"] == "256/256"
    assert rec["config"]["collectives_per_step"] > 0
    assert len(rec["detail"]["owned_points_per_rank"]) == 4


def test_bench_launcher_world_size_must_match_gpus():
    env = _env()
    env.update(RANK="0", WORLD_SIZE="2", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--device", "cpu", "--points", "3e4"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "started 2 ranks but --gpus is 4" in out.stderr


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_one_gpu_gloo():
    """Two self-launched ranks sharing the one GPU (gloo: RCCL refuses two ranks on one
    device): the full multi-rank GPU pipeline, outputs sampled exact."""
    env = _env()
    env["LSKNN_DIST_BACKEND"] = "gloo"
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(v, None)
    out = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--points", "4e5", "--steps", "2",
                          "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    rec = _json_line(out.stdout)
    assert rec["n_gpus"] == 2 and rec["config"]["ranks"] == 2
    assert rec["config"]["sampled_exact"] == "256/256"


def test_bench_ring_refuses_when_heaps_do_not_fit():
    """--mode ring at 1B on one rank needs 800 GB of the reference's k-heaps (N*k*8 B,
    unorderedDataVariant.cu:168): refused up front with the arithmetic, before any point
    is generated; 1e5 points fit."""
    out = subprocess.run([sys.executable, "bench.py", "--device", "cpu", "--mode", "ring", "--points", "1e9",
                          "--k", "100", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=_env(),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 3, out.stderr[-2000:]
    assert "800.0 GB of k-heaps" in out.stderr and "does not fit" in out.stderr
    assert "{\"metric\"" not in out.stdout


def test_ref_memory_arithmetic():
    from mpi_cuda_largescaleknn_amd.parallel import refalgo as RA

    # the 1B / 8-rank shape fits one MI355X (100 GB of heaps per rank), 1B on one does not
    RA.check_ref_fits(125_000_000, 100, 288 * 10**9, 8)
    with pytest.raises(ValueError, match="at least 3 ranks"):
        RA.check_ref_fits(1_000_000_000, 100, 288 * 10**9, 1)


@pytest.mark.parametrize("env,want", [(None, "8"), ("4", "4"), ("16", "16"), ("abc", "abc")])
def test_hardware_queue_default(env, want):
    """Importing the package fills in the HIP hardware-queue count (8: the box's default 4
    made unrelated streams share in-order queues) only when it is unset: an explicit value
    is kept (a lower one with a notice), a malformed one does not break the import
    (ADVICE r4)."""
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "LSKNN_HW_QUEUES")}
    if env is not None:
        e["GPU_MAX_HW_QUEUES"] = env
    out = subprocess.run([sys.executable, "-c", "import os, mpi_cuda_largescaleknn_amd; "
                          "print(os.environ['GPU_MAX_HW_QUEUES'])"], cwd=ROOT, env=e,
                         capture_output=True, text=True, check=True)
    assert out.stdout.strip() == want
    assert ("kept" in out.stderr) == (env == "4")


@pytest.mark.parametrize("env,want", [(None, 8), ("4", 8), ("16", 16), ("64", 32), ("abc", 8)])
def test_bench_hardware_queue_floor(env, want):
    """bench.py's own configuration: at least 8 queues (the measured best) even over the
    box's exported 4, at most 32, recorded in the JSON (config.hw_queues)."""
    e = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "LSKNN_HW_QUEUES")}
    if env is not None:
        e["GPU_MAX_HW_QUEUES"] = env
    out = subprocess.run([sys.executable, "-c", "import os, bench; print(bench.HW_QUEUES, "
                          "os.environ['GPU_MAX_HW_QUEUES'])"], cwd=ROOT, env=e,
                         capture_output=True, text=True, check=True)
    assert out.stdout.split() == [str(want), str(want)]


def test_bench_eight_ranks_driver_shape_on_cpu():
    """The driver's N=8 scaling command, rehearsed on the CPU: `bench.py --gpus 8` under
    torchrun (8 gloo ranks, 127.0.0.1 rendezvous) and self-launched with no launcher
    environment. Both report 8 ranks, 8 owned-point entries summing to the global count,
    and every sampled output exact."""
    pts = 40000
    torchrun = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "8",
                "--device", "cpu", "--points", str(pts), "--k", "16", "--steps", "2", "--warmup", "1"]
    self_env = _env()
    for v in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        self_env.pop(v, None)
    selfl = [sys.executable, "bench.py", "--gpus", "8", "--device", "cpu", "--points", str(pts), "--k", "16",
             "--steps", "2", "--warmup", "1"]
    for cmd, env in ((torchrun, dict(_env(), OMP_NUM_THREADS="1")), (selfl, dict(self_env, OMP_NUM_THREADS="1"))):
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-3000:]
        rec = _json_line(out.stdout)
        assert rec["n_gpus"] == 8 and rec["config"]["ranks"] == 8
        assert rec["steps"] == 2 and rec["warmup"] == 1
        s = rec["config"]["sampled_exact"]
        a, b = s.split("/")
        assert a == b and int(b) > 0, s
        own = rec["detail"]["owned_points_per_rank"]
        assert len(own) == 8 and sum(own) == pts
        assert rec["config"]["all_finite"] is True
