"""Multi-PROCESS GPU pipelines on one MI355X: separate processes (own HIP contexts, own
kernel libraries) share cuda:0 over a gloo process group whose collectives TorchComm
stages through host memory (RCCL refuses two ranks on one device). Together with the
LoopbackComm tests (threads, one process) this covers the one-process-per-GPU path the
8-GPU runs take, minus RCCL itself. Results must equal the single-rank GPU run bit for
bit (which the other GPU tests check against the CPU oracle)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from datasets import clustered, uniform

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _points(dist_name):
    return (uniform if dist_name == "uniform" else clustered)(60000, seed=5)


def _worker(rank, size, port, variant, dist_name, out_dir):
    import torch.distributed as dist

    from mpi_cuda_largescaleknn_amd.models import knn_engine as E
    from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
    from mpi_cuda_largescaleknn_amd.parallel.comm import TorchComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    p = _points(dist_name)
    cfg = E.KnnConfig(k=32)
    comm = TorchComm(dev)
    assert comm.staged
    if variant == "unordered":
        b, e = p.shape[0] * rank // size, p.shape[0] * (rank + 1) // size
        out = PL.unordered_knn(p[b:e].to(dev), comm, cfg)
    else:
        owner = torch.clamp((p[:, 0] * size).long(), max=size - 1)
        out = PL.prepartitioned_knn(p[owner == rank].to(dev), comm, cfg)
    torch.save(out.cpu(), os.path.join(out_dir, f"{rank}.pt"))
    comm.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant,dist_name,size", [("unordered", "uniform", 2),
                                                    ("unordered", "clustered", 3),
                                                    ("prepartitioned", "uniform", 2)])
def test_multiprocess_gpu_matches_single_rank(tmp_path, variant, dist_name, size):
    from mpi_cuda_largescaleknn_amd.models import knn_engine as E

    mp.spawn(_worker, args=(size, _port(), variant, dist_name, str(tmp_path)), nprocs=size, join=True)
    p = _points(dist_name)
    ref = E.knn_distances(p.to("cuda:0"), 32).cpu()
    outs = [torch.load(tmp_path / f"{r}.pt", weights_only=True) for r in range(size)]
    if variant == "unordered":
        assert torch.equal(torch.cat(outs), ref)
    else:
        owner = torch.clamp((p[:, 0] * size).long(), max=size - 1)
        for r in range(size):
            assert torch.equal(outs[r], ref[owner == r])


def test_cli_two_gpu_processes_match_one(tmp_path):
    """hipKNN_unorderedData under torchrun, 2 ranks on cuda:0 (-g 1), gloo staging:
    output file byte-identical to the single-process GPU run."""
    env = dict(os.environ, PYTHONPATH=ROOT, LSKNN_DIST_BACKEND="gloo")
    pts = tmp_path / "pts.float3"
    gen = [sys.executable, "-m", "mpi_cuda_largescaleknn_amd.apps.tools", "gen", str(pts), "-n", "200000",
           "--seed", "9"]
    subprocess.run(gen, env=env, check=True, timeout=120, capture_output=True)
    app = ["-m", "mpi_cuda_largescaleknn_amd.apps.unordered", str(pts), "-k", "100"]
    one = subprocess.run([sys.executable] + app + ["-o", str(tmp_path / "one.float")], env=env,
                         timeout=120, capture_output=True, text=True)
    assert one.returncode == 0, one.stderr
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node=2",
                          "--master-addr=127.0.0.1", f"--master-port={_port()}"] + app +
                         ["-o", str(tmp_path / "two.float"), "-g", "1"], env=env, timeout=120,
                         capture_output=True, text=True)
    assert two.returncode == 0, two.stderr[-3000:]
    assert "#1/2setting active GPU #0" in two.stdout
    a = (tmp_path / "one.float").read_bytes()
    b = (tmp_path / "two.float").read_bytes()
    assert len(a) == 4 * 200000 and a == b
