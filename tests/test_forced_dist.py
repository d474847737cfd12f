"""Forced multi-rank path on a 1-rank gloo group (CPU): every pipeline goes through its
collectives (TorchComm(force=True)) and equals the single-rank result bit for bit. The
GPU twin on a real 1-rank RCCL group is tests/test_gpu_rccl.py."""
import os
import socket

import torch
import torch.multiprocessing as mp

from datasets import clustered


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out_dir):
    import torch.distributed as dist

    from mpi_cuda_largescaleknn_amd.models import knn_engine as E
    from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
    from mpi_cuda_largescaleknn_amd.parallel import refalgo as RA
    from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm, TorchComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = TorchComm("cpu", force=True)
    PL.HALO_ONE_RANK = True  # exercise the (empty) halo exchange too
    p = clustered(6000, seed=2)
    cfg = E.KnnConfig(k=12)
    res = {}
    for name, fn in (("unordered", PL.unordered_knn), ("prepartitioned", PL.prepartitioned_knn),
                     ("ring", RA.ring_knn), ("peer", RA.peer_knn)):
        info = PL.RunInfo(PL.PhaseTimer(True, torch.device("cpu")))
        res[name] = fn(p, comm, cfg, info)
        res[name + "_single"] = fn(p, SingleComm("cpu"), cfg)
        res[name + "_phases"] = sorted(info.timer.times)
    PL.HALO_ONE_RANK = False  # default: a 1-rank group skips the halo
    info = PL.RunInfo(PL.PhaseTimer(True, torch.device("cpu")))
    res["nohalo"] = PL.prepartitioned_knn(p, comm, cfg, info)
    res["nohalo_phases"] = sorted(info.timer.times)
    torch.save(res, os.path.join(out_dir, "res.pt"))
    dist.destroy_process_group()


def test_forced_one_rank_gloo_equals_single(tmp_path):
    mp.spawn(_worker, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    res = torch.load(tmp_path / "res.pt", weights_only=True)
    for name in ("unordered", "prepartitioned", "ring", "peer"):
        assert torch.equal(res[name], res[name + "_single"]), name
    assert "alltoallv_points" in res["unordered_phases"]
    assert "knn_local+halo_exchange" in res["prepartitioned_phases"]  # overlapped halo
    assert torch.equal(res["nohalo"], res["prepartitioned_single"])
    assert "knn_local" in res["nohalo_phases"] and "knn_local+halo_exchange" not in res["nohalo_phases"]


def _chunk_worker(rank, size, port, out_dir):
    import torch.distributed as dist

    from mpi_cuda_largescaleknn_amd.parallel.comm import TorchComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    comm = TorchComm("cpu")
    comm.max_msg_bytes = 100  # force many rounds of pieces (uneven last pieces)
    g = torch.Generator().manual_seed(rank)
    counts = [(rank * 7 + 3 * j) % 11 + (40 if j == (rank + 1) % size else 0) for j in range(size)]
    send = torch.rand((sum(counts), 3), generator=g)
    recv, rc = comm.alltoallv(send, counts)
    # ring p2p of a payload much larger than one piece
    nxt, prv = (rank + 1) % size, (rank - 1) % size
    big = torch.arange(1000, dtype=torch.float32) + 1000 * rank
    (got,) = comm.p2p([(nxt, big)], [(prv, (1000,), torch.float32)])
    torch.save({"send": send, "counts": counts, "recv": recv, "rc": rc, "got": got},
               os.path.join(out_dir, f"{rank}.pt"))
    dist.destroy_process_group()


def test_alltoallv_and_p2p_in_pieces_gloo(tmp_path):
    size = 3
    mp.spawn(_chunk_worker, args=(size, _port(), str(tmp_path)), nprocs=size, join=True)
    r = [torch.load(tmp_path / f"{i}.pt", weights_only=True) for i in range(size)]
    for me in range(size):
        parts = []
        for src in range(size):
            c = r[src]["counts"]
            o = sum(c[:me])
            parts.append(r[src]["send"][o:o + c[me]])
        assert torch.equal(r[me]["recv"], torch.cat(parts))
        assert r[me]["rc"] == [r[src]["counts"][me] for src in range(size)]
        prv = (me - 1) % size
        assert torch.equal(r[me]["got"], torch.arange(1000, dtype=torch.float32) + 1000 * prv)


def _mixed_worker(rank, size, port, out_dir):
    import torch.distributed as dist

    from mpi_cuda_largescaleknn_amd.parallel.comm import TorchComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    comm = TorchComm("cpu")
    comm.max_msg_bytes = 4000  # 1000 float32 rows of 1 value
    # rank 0 sends one big message (3000 rows) to rank 1; every other message is small, so
    # only ranks 0 and 1 see a message above the cap: all ranks must still pick the same form
    counts = [[5, 3000, 2], [4, 6, 1], [7, 8, 9]][rank]
    send = torch.arange(sum(counts), dtype=torch.float32) + 1000 * rank
    recv, rc = comm.alltoallv(send, counts, recv_counts=[[5, 4, 7], [3000, 6, 8], [2, 1, 9]][rank])
    torch.save({"recv": recv, "rc": rc}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_alltoallv_form_agreed_across_ranks(tmp_path):
    """Known receive counts and one message above the cap on a single pair: every rank
    takes the piece-round form (agreed maximum), no rank waits in all_to_all_single."""
    mp.spawn(_mixed_worker, args=(3, _port(), str(tmp_path)), nprocs=3, join=True)
    sends = {r: torch.arange(sum(c), dtype=torch.float32) + 1000 * r
             for r, c in enumerate([[5, 3000, 2], [4, 6, 1], [7, 8, 9]])}
    offs = {r: [0, c[0], c[0] + c[1], sum(c)] for r, c in enumerate([[5, 3000, 2], [4, 6, 1], [7, 8, 9]])}
    for r in range(3):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        want = torch.cat([sends[j][offs[j][r]:offs[j][r + 1]] for j in range(3)])
        assert torch.equal(got["recv"], want)
