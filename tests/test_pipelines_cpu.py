"""T3: distributed pipelines without GPUs — P virtual ranks (LoopbackComm threads) and
real multi-process gloo groups — must reproduce the single-rank oracle exactly
(the result is independent of P and of the partitioning)."""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from datasets import GENERATORS, clustered, uniform
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.ops import kernels as K
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
from mpi_cuda_largescaleknn_amd.parallel.comm import run_loopback


def oracle(p, k, r=math.inf):
    return K.finalize_distances(K.kth_cpu(p, p, k, E.cut2_of(r)))


def block(n, r, size):
    return n * r // size, n * (r + 1) // size


@pytest.mark.parametrize("size", [1, 2, 3, 4, 7])
@pytest.mark.parametrize("dist", ["uniform", "clustered", "duplicates"])
def test_unordered_loopback(size, dist):
    p = GENERATORS[dist](6000, seed=size)
    k = 12
    cfg = E.KnnConfig(k=k, publish_levels=4)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e], comm, cfg)

    out = torch.cat(run_loopback(size, fn))
    assert torch.equal(out, oracle(p, k))


@pytest.mark.parametrize("size", [2, 4])
def test_prepartitioned_loopback_spatial_and_random(size):
    p = uniform(5000, seed=9)
    k = 20
    cfg = E.KnnConfig(k=k, publish_levels=3)
    # spatial slabs in x (the intended use) and a random split (worst case: total overlap)
    slab = torch.clamp((p[:, 0] * size).long(), max=size - 1)
    rnd = torch.randint(0, size, (p.shape[0],), generator=torch.Generator().manual_seed(1))
    ref = oracle(p, k)
    for owner in (slab, rnd):
        parts = [p[owner == r] for r in range(size)]
        outs = run_loopback(size, lambda comm: PL.prepartitioned_knn(parts[comm.rank], comm, cfg))
        for r in range(size):
            assert torch.equal(outs[r], ref[owner == r])


def test_cutoff_and_large_k_distributed():
    p = clustered(3000, seed=4)
    for k, r in [(50, 0.01), (3001, math.inf), (7, 0.0)]:
        cfg = E.KnnConfig(k=k, max_radius=r, publish_levels=3)

        def fn(comm):
            b, e = block(p.shape[0], comm.rank, comm.size)
            return PL.unordered_knn(p[b:e], comm, cfg)

        out = torch.cat(run_loopback(3, fn))
        assert torch.equal(out, oracle(p, k, r)), (k, r)


def test_empty_rank():
    p = uniform(100, seed=2)
    cfg = E.KnnConfig(k=5, publish_levels=2)
    parts = [p[:60], p[:0], p[60:]]
    outs = run_loopback(3, lambda comm: PL.prepartitioned_knn(parts[comm.rank], comm, cfg))
    ref = oracle(p, 5)
    assert torch.equal(torch.cat(outs), ref)


# --------------------------------------------------------------------------- gloo
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, size, port, variant, result_dir):
    import torch.distributed as dist
    from mpi_cuda_largescaleknn_amd.parallel.comm import TorchComm

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    p = uniform(4000, seed=21)
    cfg = E.KnnConfig(k=10, publish_levels=4)
    comm = TorchComm("cpu")
    if variant == "unordered":
        b, e = block(p.shape[0], rank, size)
        out = PL.unordered_knn(p[b:e], comm, cfg)
    else:
        owner = torch.clamp((p[:, 1] * size).long(), max=size - 1)
        out = PL.prepartitioned_knn(p[owner == rank], comm, cfg)
    torch.save(out, os.path.join(result_dir, f"{variant}_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["unordered", "prepartitioned"])
def test_gloo_two_processes(tmp_path, variant):
    size = 2
    mp.spawn(_gloo_worker, args=(size, _free_port(), variant, str(tmp_path)), nprocs=size, join=True)
    p = uniform(4000, seed=21)
    ref = oracle(p, 10)
    outs = [torch.load(tmp_path / f"{variant}_{r}.pt", weights_only=True) for r in range(size)]
    if variant == "unordered":
        assert torch.equal(torch.cat(outs), ref)
    else:
        owner = torch.clamp((p[:, 1] * size).long(), max=size - 1)
        for r in range(size):
            assert torch.equal(outs[r], ref[owner == r])


# --------------------------------------------------------------------------- ref-algo schedules
from mpi_cuda_largescaleknn_amd.ops import refalgo as R  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import refalgo as RA  # noqa: E402


def _check_lbt(tree, n):
    # left-balanced invariant: left subtree coords <= split <= right subtree coords
    def sub(t):
        out, st = [], [t]
        while st:
            x = st.pop()
            if x < n:
                out.append(x)
                st += [2 * x + 1, 2 * x + 2]
        return out

    for t in range(min(n, 200)):
        level = (t + 1).bit_length() - 1
        dim = level % 3
        split = tree[t, dim]
        for c in sub(2 * t + 1):
            assert tree[c, dim] <= split
        for c in sub(2 * t + 2):
            assert tree[c, dim] >= split


def test_lbt_cpu_invariant_and_ids():
    p = uniform(777, seed=5)
    tree, ids = R.build_lbt(p)
    _check_lbt(tree, 777)
    assert torch.equal(tree, p[ids.long()])


@pytest.mark.parametrize("size", [1, 2, 3])
def test_ring_mode_loopback(size):
    p = clustered(3000, seed=size)
    k = 9
    cfg = E.KnnConfig(k=k)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return RA.ring_knn(p[b:e], comm, cfg)

    assert torch.equal(torch.cat(run_loopback(size, fn)), oracle(p, k))


@pytest.mark.parametrize("split", ["slab", "random"])
def test_peer_mode_loopback(split):
    size = 4
    p = uniform(4000, seed=12)
    k = 15
    if split == "slab":
        owner = torch.clamp((p[:, 0] * size).long(), max=size - 1)
    else:
        owner = torch.randint(0, size, (p.shape[0],), generator=torch.Generator().manual_seed(3))
    parts = [p[owner == r] for r in range(size)]
    rounds = {}

    def fn(comm):
        info = PL.RunInfo(PL.PhaseTimer(False))
        out = RA.peer_knn(parts[comm.rank], comm, E.KnnConfig(k=k), info)
        rounds[comm.rank] = info.counts["peer_rounds"]
        return out

    outs = run_loopback(size, fn)
    ref = oracle(p, k)
    for r in range(size):
        assert torch.equal(outs[r], ref[owner == r])
    if split == "slab":  # culling: not every rank pulls every shard
        assert max(rounds.values()) <= size


@pytest.mark.parametrize("size", [2, 3])
def test_unordered_loopback_sub_cell_core(size):
    """A 1e-3 core in a 1000^3 box: every rank's owned share of the core exceeds
    knn_engine.HEAVY_RUN points of one key, so the per-rank index build re-keys it
    (second-level curve keys); results stay identical to the oracle."""
    p = GENERATORS["mixed_scale"](24000, seed=size)
    k = 10
    cfg = E.KnnConfig(k=k, publish_levels=4)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e], comm, cfg)

    out = torch.cat(run_loopback(size, fn))
    assert torch.equal(out, oracle(p, k))


@pytest.mark.parametrize("balance", ["auto", "off", "on"])
def test_prepartitioned_skewed_files_rebalance(balance):
    """8 spatial files, one holding half of the points: the balanced run
    gives every rank ~N/8 points to query, the results stay exact and in file order."""
    size = 8
    p = uniform(16000, seed=12)
    k = 10
    cfg = E.KnnConfig(k=k, publish_levels=4)
    # x < 0.5 -> rank 0 (half the points), the rest in 7 slabs
    owner = torch.where(p[:, 0] < 0.5, torch.zeros_like(p[:, 0]).long(),
                        1 + torch.clamp(((p[:, 0] - 0.5) * 14).long(), max=6))
    parts = [p[owner == r] for r in range(size)]
    infos = [PL.RunInfo(PL.PhaseTimer(False, torch.device("cpu"))) for _ in range(size)]
    outs = run_loopback(size, lambda c: PL.prepartitioned_knn(parts[c.rank], c, cfg, infos[c.rank],
                                                              balance=balance))
    ref = oracle(p, k)
    for r in range(size):
        assert torch.equal(outs[r], ref[owner == r])
    owned = [i.counts["owned_points"] for i in infos]
    assert sum(owned) == 16000
    if balance == "off":
        assert max(owned) == parts[0].shape[0] and all("rebalanced" not in i.counts for i in infos)
    else:
        assert all(i.counts.get("rebalanced") == 1 for i in infos)
        assert max(owned) < 1.1 * 16000 / size, owned


@pytest.mark.parametrize("size", [1, 2, 3, 5])
def test_unordered_streamed_redistribution(size, monkeypatch):
    """Chunked (streamed) redistribution: ownership from the first chunks, return through
    the chunk permutations; results equal the oracle in input order."""
    monkeypatch.setattr(PL, "FORCE_STREAM", True)
    monkeypatch.setattr(PL, "STREAM_CHUNK", 700)
    p = clustered(7000, seed=size + 20)
    k = 9
    cfg = E.KnnConfig(k=k, publish_levels=4)
    infos = [PL.RunInfo(PL.PhaseTimer(False, torch.device("cpu"))) for _ in range(size)]

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e], comm, cfg, infos[comm.rank])

    out = torch.cat(run_loopback(size, fn))
    assert torch.equal(out, oracle(p, k))
    if size > 1:
        assert all(i.counts["stream_chunks"] >= 2 for i in infos)
        assert sum(i.counts["owned_points"] for i in infos) == 7000


def test_streamed_redistribution_unrepresentative_first_chunk(monkeypatch):
    """Input sorted along x: the first chunk's cube misses most points (clamped keys) —
    only the balance suffers, the result stays exact."""
    monkeypatch.setattr(PL, "FORCE_STREAM", True)
    monkeypatch.setattr(PL, "STREAM_CHUNK", 500)
    p = uniform(4000, seed=3)
    p = p[torch.argsort(p[:, 0])].contiguous()
    cfg = E.KnnConfig(k=6, publish_levels=4)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e], comm, cfg)

    assert torch.equal(torch.cat(run_loopback(3, fn)), oracle(p, 6))


@pytest.mark.parametrize("k", [5, 100, 300])
def test_overlapped_halo_subset_and_exact(k, monkeypatch):
    """knn_with_halo's overlapped form classifies the query groups with a-priori radius
    bounds (tree_set_radii_ub) against the other ranks' published trees, queries the
    boundary groups first and publishes their exact radii (interior groups: 0): its halo
    is a subset of the sequential form's (exact radii on every leaf), the re-query flags
    from the final radii, and the results are identical (and exact). k = 300 > 64: the
    bound window spans several buckets; 4 ranks, clustered data."""
    p = clustered(8000, seed=k)
    cfg = E.KnnConfig(k=k, publish_levels=4)
    res = {}
    for mode in (False, True):
        monkeypatch.setattr(PL, "OVERLAP_HALO", mode)
        infos = [PL.RunInfo(PL.PhaseTimer(False, torch.device("cpu"))) for _ in range(4)]

        def fn(comm):
            b, e = block(p.shape[0], comm.rank, comm.size)
            return PL.unordered_knn(p[b:e], comm, cfg, infos[comm.rank])

        res[mode] = (torch.cat(run_loopback(4, fn)), sum(i.counts.get("halo_recv", 0) for i in infos))
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][0], oracle(p, k))
    assert res[False][1] >= res[True][1] > 0


def test_radius_upper_bound_covers_kth():
    """Every leaf's a-priori bound >= the largest k-th squared distance of its queries."""
    for n, k in ((5000, 1), (5000, 64), (5000, 65), (3000, 200), (100, 100), (50, 100), (6000, 500)):
        p = uniform(n, seed=n + k)
        idx = E.build_index(p)
        nodes = K.tree_set_radii_ub(idx.nodes.clone(), idx.pts, idx.n, k)
        d2 = K.kth_cpu(idx.pts[:n], idx.pts[:n], k, math.inf)
        slots = 1 << idx.depth
        nb = (n + 63) // 64
        leaf_max = torch.zeros(slots * 64)
        leaf_max[:n] = d2
        leaf_max = leaf_max.view(slots, 64).amax(dim=1)
        ub = nodes[slots:slots + nb, 3]
        assert bool((ub >= leaf_max[:nb]).all()), (n, k)
        assert float(nodes[1, 3]) >= float(d2.max())


def test_overlapped_halo_cutoff_caps_bounds(monkeypatch):
    """With -r the a-priori bounds are capped at the cutoff: a small radius sends a much
    smaller halo than no radius, results stay exact."""
    p = uniform(12000, seed=3)
    k = 20
    res = {}
    for r in (math.inf, 0.02):
        cfg = E.KnnConfig(k=k, max_radius=r, publish_levels=4)
        infos = [PL.RunInfo(PL.PhaseTimer(False, torch.device("cpu"))) for _ in range(4)]

        def fn(comm):
            b, e = block(p.shape[0], comm.rank, comm.size)
            return PL.unordered_knn(p[b:e], comm, cfg, infos[comm.rank])

        out = torch.cat(run_loopback(4, fn))
        assert torch.equal(out, oracle(p, k, r))
        res[r] = sum(i.counts.get("halo_recv", 0) for i in infos)
    assert res[0.02] < res[math.inf] / 2, res


@pytest.mark.timeout(120)
@pytest.mark.parametrize("sizes", [(10, 2500, 6000), (0, 4000, 900), (3000, 3000, 2999)])
def test_streamed_redistribution_uneven_ranks(sizes, monkeypatch):
    """Ranks with different point counts (and an empty rank) stream different numbers of
    non-empty chunks: the chunk count is agreed over ranks (trailing empty chunks), so
    every rank runs the same all-to-all-v sequence; exact results."""
    monkeypatch.setattr(PL, "FORCE_STREAM", True)
    monkeypatch.setattr(PL, "STREAM_CHUNK", 1000)
    n = sum(sizes)
    p = clustered(n, seed=n)
    offs = [0, sizes[0], sizes[0] + sizes[1], n]
    cfg = E.KnnConfig(k=7, publish_levels=4)

    def fn(comm):
        return PL.unordered_knn(p[offs[comm.rank]:offs[comm.rank + 1]], comm, cfg)

    assert torch.equal(torch.cat(run_loopback(3, fn)), oracle(p, 7))
