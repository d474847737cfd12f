"""Multi-rank pipelines on one GPU: P virtual ranks (LoopbackComm threads) share the
device and exercise the GPU halo path (publish, halo_mask filter, pack, halo tree,
group flagging, 2-tree re-query) and the spatial redistribution. Results must equal
the single-rank GPU result (itself checked against the CPU oracle) bit for bit."""
import math

import pytest
import torch

from datasets import clustered, duplicates, uniform
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.ops import kernels as K
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
from mpi_cuda_largescaleknn_amd.parallel.comm import run_loopback

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def block(n, r, size):
    return n * r // size, n * (r + 1) // size


def single(p, k, r=math.inf):
    return E.knn_distances(p.to(DEV), k, max_radius=r).cpu()


@pytest.mark.parametrize("size", [2, 3, 4, 8])
@pytest.mark.parametrize("gen", [uniform, clustered])
def test_unordered_multirank_gpu(size, gen):
    p = gen(200_000, seed=size)
    k = 100
    cfg = E.KnnConfig(k=k, collect_stats=True)
    ref = single(p, k)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        info = PL.RunInfo(PL.PhaseTimer(False, DEV))
        out = PL.unordered_knn(p[b:e].to(DEV), comm, cfg, info)
        return out.cpu(), info

    res = run_loopback(size, fn, DEV)
    out = torch.cat([r[0] for r in res])
    assert torch.equal(out, ref)
    for _, info in res:
        assert info.stats.counters.get("mismatch_lanes", 0) == 0
        assert info.counts["halo_recv"] < p.shape[0]  # halo, not whole shards


def test_unordered_matches_cpu_oracle_small():
    p = duplicates(30_000, seed=3)
    ref = K.finalize_distances(K.kth_cpu(p, p, 16, math.inf))

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e].to(DEV), comm, E.KnnConfig(k=16)).cpu()

    assert torch.equal(torch.cat(run_loopback(4, fn, DEV)), ref)


@pytest.mark.parametrize("split", ["slab", "random"])
def test_prepartitioned_multirank_gpu(split):
    size = 4
    p = uniform(150_000, seed=7)
    k = 50
    ref = single(p, k)
    if split == "slab":
        owner = torch.clamp((p[:, 2] * size).long(), max=size - 1)
    else:
        owner = torch.randint(0, size, (p.shape[0],), generator=torch.Generator().manual_seed(0))
    parts = [p[owner == r] for r in range(size)]

    def fn(comm):
        return PL.prepartitioned_knn(parts[comm.rank].to(DEV), comm, E.KnnConfig(k=k)).cpu()

    outs = run_loopback(size, fn, DEV)
    for r in range(size):
        assert torch.equal(outs[r], ref[owner == r])


def test_cutoff_multirank_gpu():
    p = clustered(60_000, seed=1)
    for k, r in [(100, 0.002), (10, 0.05)]:
        ref = single(p, k, r)

        def fn(comm):
            b, e = block(p.shape[0], comm.rank, comm.size)
            return PL.unordered_knn(p[b:e].to(DEV), comm, E.KnnConfig(k=k, max_radius=r)).cpu()

        assert torch.equal(torch.cat(run_loopback(3, fn, DEV)), ref)


def test_single_rank_direct_host_output():
    """One rank: the k-NN kernel writes into a pinned host buffer over PCIe (bench
    default); same bits as the device buffer + copy, for both entrypoints."""
    from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm
    p = clustered(120_000, seed=4)
    cfg = E.KnnConfig(k=40)
    comm = SingleComm(DEV)
    for fn in (PL.unordered_knn, PL.prepartitioned_knn):
        ref = fn(p.to(DEV), comm, cfg).cpu()
        host = torch.full((p.shape[0],), -1.0).pin_memory()
        got = fn(p.to(DEV), comm, cfg, out=host)
        torch.cuda.synchronize()
        assert got.data_ptr() == host.data_ptr()
        assert torch.equal(host, ref)
    with pytest.raises(ValueError):
        PL.unordered_knn(p.to(DEV), comm, cfg, out=torch.empty(p.shape[0]))  # not pinned


@pytest.mark.parametrize("size", [2, 4])
def test_unordered_multirank_gpu_sub_cell_core(size):
    """1e-3 core in a 1000^3 box (second-level keys in the per-rank index build and in
    the single-rank reference) through the GPU halo pipeline; checked against the CPU
    oracle directly."""
    from datasets import mixed_scale

    p = mixed_scale(60_000, seed=size)
    k = 16
    cfg = E.KnnConfig(k=k)
    ref = K.finalize_distances(K.kth_cpu(p, p, k, math.inf))
    assert torch.equal(single(p, k), ref)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        return PL.unordered_knn(p[b:e].to(DEV), comm, cfg).cpu()

    out = torch.cat(run_loopback(size, fn, DEV))
    assert torch.equal(out, ref)


@pytest.mark.parametrize("size", [2, 4])
def test_unordered_streamed_from_pinned_host(size, monkeypatch):
    """Host-resident (pinned) input: the redistribution streams it to the device in chunks
    on a copy stream, overlapped with the exchange; bit-identical to one rank."""
    monkeypatch.setattr(PL, "STREAM_CHUNK", 40_000)
    p = uniform(300_000, seed=21)
    k = 100
    ref = single(p, k)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        host = torch.empty((e - b, 3), dtype=torch.float32, pin_memory=True)
        host.copy_(p[b:e])
        info = PL.RunInfo(PL.PhaseTimer(False, DEV))
        out = PL.unordered_knn(host, comm, E.KnnConfig(k=k), info)
        return out.cpu(), info

    res = run_loopback(size, fn, DEV)
    assert torch.equal(torch.cat([r[0] for r in res]), ref)
    assert all(r[1].counts["stream_chunks"] >= 2 for r in res)


@pytest.mark.parametrize("k", [16, 100])
def test_overlapped_halo_gpu_equals_sequential(k, monkeypatch):
    """The side-stream halo exchange (boundary groups from a-priori radius bounds queried
    first, their exact radii published, filter/pack/exchange while the interior groups'
    k-NN runs) gives the sequential form's bits; its halo is a subset of the sequential
    one; the overlapped path really ran."""
    p = clustered(300_000, seed=k)
    ref = single(p, k)
    cfg = E.KnnConfig(k=k)
    res = {}
    for mode in (False, True):
        monkeypatch.setattr(PL, "OVERLAP_HALO", mode)

        def fn(comm):
            b, e = block(p.shape[0], comm.rank, comm.size)
            info = PL.RunInfo(PL.PhaseTimer(False, DEV))
            out = PL.unordered_knn(p[b:e].to(DEV), comm, cfg, info)
            return out.cpu(), info

        r = run_loopback(4, fn, DEV)
        res[mode] = (torch.cat([x[0] for x in r]), sum(x[1].counts["halo_recv"] for x in r),
                     [x[1].counts.get("halo_overlap", 0) for x in r])
    assert torch.equal(res[True][0], ref) and torch.equal(res[False][0], ref)
    assert res[False][1] >= res[True][1] > 0
    assert res[True][2] == [1, 1, 1, 1] and res[False][2] == [0, 0, 0, 0]


@pytest.mark.parametrize("k", [1, 100, 448, 600])
def test_radius_upper_bound_gpu(k):
    """tree.hip leaf_radius_ub_kernel: every leaf's a-priori bound covers the k-th squared
    distance of all its queries (GPU k-NN), and matches the CPU formula closely
    (k = 600: the box-pair fallback beyond 8 window buckets)."""
    p = clustered(100_000, seed=k).to(DEV)
    idx = E.build_index(p)
    n = idx.n
    ub = K.tree_set_radii_ub(idx.nodes.clone(), idx.pts, n, k)
    d2 = E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, n, k))
    slots = 1 << idx.depth
    nb = (n + 63) // 64
    leaf_max = torch.zeros(slots * 64, device=DEV)
    leaf_max[:n] = d2
    leaf_max = leaf_max.view(slots, 64).amax(dim=1)
    assert bool((ub[slots:slots + nb, 3] >= leaf_max[:nb]).all())
    cpu = K.tree_set_radii_ub(idx.nodes.cpu().clone(), idx.pts.cpu(), n, k)
    assert torch.allclose(cpu[slots:slots + nb, 3], ub[slots:slots + nb, 3].cpu(), rtol=1e-5)


@pytest.mark.parametrize("groups", [1, 3, 4])
def test_grouped_return_into_pinned_host(groups, monkeypatch):
    """Streamed input and a pinned host output: the result return runs in groups of stream
    chunks, each group's rows copied to the host on a copy stream while the next group is
    exchanged (groups=1: the single return + copy); bit-identical to one rank."""
    monkeypatch.setattr(PL, "STREAM_CHUNK", 30_000)
    monkeypatch.setattr(PL, "RETURN_GROUPS", groups)
    p = clustered(250_000, seed=groups)
    k = 50
    ref = single(p, k)

    def fn(comm):
        b, e = block(p.shape[0], comm.rank, comm.size)
        host = torch.empty((e - b, 3), dtype=torch.float32, pin_memory=True)
        host.copy_(p[b:e])
        out = torch.full((e - b,), -1.0, dtype=torch.float32, pin_memory=True)
        got = PL.unordered_knn(host, comm, E.KnnConfig(k=k), PL.RunInfo(PL.PhaseTimer(False, DEV)), out=out)
        torch.cuda.synchronize()
        assert got.data_ptr() == out.data_ptr()
        return out.clone()

    res = run_loopback(3, fn, DEV)
    assert torch.equal(torch.cat(res), ref)


@pytest.mark.parametrize("sizes", [(5, 70_000, 150_000), (0, 90_000, 30_000)])
def test_streamed_uneven_ranks_gpu(sizes, monkeypatch):
    """Pinned host inputs of different sizes (one empty): the agreed chunk count gives
    every rank the same all-to-all-v sequence (empty trailing chunks), grouped return
    into pinned output included; bit-identical to one rank."""
    monkeypatch.setattr(PL, "STREAM_CHUNK", 25_000)
    n = sum(sizes)
    p = clustered(n, seed=n)
    offs = [0, sizes[0], sizes[0] + sizes[1], n]
    ref = single(p, 30)

    def fn(comm):
        b, e = offs[comm.rank], offs[comm.rank + 1]
        host = torch.empty((e - b, 3), dtype=torch.float32, pin_memory=True)
        host.copy_(p[b:e])
        out = torch.empty(e - b, dtype=torch.float32, pin_memory=True)
        PL.unordered_knn(host, comm, E.KnnConfig(k=30), out=out)
        torch.cuda.synchronize()
        return out.clone()

    assert torch.equal(torch.cat(run_loopback(3, fn, DEV)), ref)
