"""The single-rank pipeline captured in one HIP graph (bench.py's default on one GPU):
host->device copy, bounds, device-side radius hint, Hilbert sort, tree, k-NN with the
distances written to pinned host memory (or copied back). Every decision baked into the
graph at capture time is data independent, so replaying it on NEW contents of the same
pinned input buffer must give exactly the eager result for that data."""
import pytest
import torch

from datasets import clustered, uniform
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.mark.parametrize("variant", ["unordered", "prepartitioned"])
@pytest.mark.parametrize("k", [100, 16])
def test_graph_replay_matches_eager_on_new_data(variant, k):
    n = 150_000
    host_pts = torch.empty((n, 3), dtype=torch.float32, pin_memory=True)
    host_out = torch.empty(n, dtype=torch.float32, pin_memory=True)
    host_pts.copy_(uniform(n, seed=1))
    cfg = E.KnnConfig(k=k)
    comm = SingleComm(DEV)
    direct = PL.direct_host_out_pays(k)

    def body():
        pts = host_pts.to(DEV, non_blocking=True)
        o = host_out if direct else None
        if variant == "unordered":
            out = PL.unordered_knn(pts, comm, cfg, n_total=n, out=o)
        else:
            out = PL.prepartitioned_knn(pts, comm, cfg, out=o)
        if out.data_ptr() != host_out.data_ptr():
            host_out.copy_(out, non_blocking=True)

    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        body()
    torch.cuda.current_stream(DEV).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    E.reset_kernels_used()
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()
    # the captured build decides grid vs rows on the device (knn_engine.build_grid)
    assert len(E.GATES_SEEN) == 1
    gate = E.GATES_SEEN[0]

    for i, (data, grid) in enumerate(((uniform(n, seed=1), True), (clustered(n, seed=2), None),
                                      (uniform(n, seed=3) * 7.0 - 2.0, True))):
        host_pts.copy_(data)
        host_out.fill_(-1.0)
        g.replay()
        torch.cuda.synchronize()
        if grid:  # (replay 2 after a clustered one: the grid's slot table is cleared by a
            # kernel node — a captured hipMemsetAsync did not re-run, dev.h lsk_fill32)
            assert int(gate.item()) == 1, f"replay {i}"  # uniform data: the captured grid kernel ran
        ref = E.knn_distances(data.to(DEV), k).cpu()
        assert torch.equal(host_out, ref)


def _capture(fn):
    side = torch.cuda.Stream(DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream(DEV).wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    torch.cuda.synchronize()
    return g


def test_graph_with_heavy_cell_refinement(monkeypatch):
    """mixed_scale (a sub-cell core): the eager warmup refines, the capture then records
    the fixed-size refinement; replay == eager bit for bit and about as fast."""
    import time

    from datasets import mixed_scale

    n, k = 2_000_000, 100
    data = mixed_scale(n, seed=4)
    host_pts = torch.empty((n, 3), dtype=torch.float32, pin_memory=True)
    host_pts.copy_(data)
    out = torch.empty(n, dtype=torch.float32, device=DEV)

    def body():
        out.copy_(E.knn_distances(host_pts.to(DEV, non_blocking=True), k))

    monkeypatch.setattr(E, "LAST_REFINED", False)
    body()
    torch.cuda.synchronize()
    assert E.LAST_REFINED
    t = time.perf_counter()
    body()
    torch.cuda.synchronize()
    eager_s = time.perf_counter() - t
    eager = out.cpu()
    monkeypatch.setattr(E, "REFINE_CAPTURE", True)
    g = _capture(body)
    out.fill_(-1)
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    graph_s = time.perf_counter() - t
    assert not E.captured_heavy_cells(clear=True)
    E.verify_captured_failures(clear=True)
    assert torch.equal(out.cpu(), eager)
    print(f"mixed_scale 2e6 k=100: eager {eager_s * 1e3:.1f} ms, graph {graph_s * 1e3:.1f} ms")
    assert graph_s < 1.5 * eager_s + 0.02


def test_graph_without_refinement_flags_heavy_cells(monkeypatch):
    from datasets import mixed_scale

    n, k = 40_000, 16
    data = mixed_scale(n, seed=6).to(DEV)
    out = torch.empty(n, dtype=torch.float32, device=DEV)
    monkeypatch.setattr(E, "REFINE_CAPTURE", False)
    E.CAPTURED_HEAVY.clear()
    g = _capture(lambda: out.copy_(E.knn_distances(data, k)))
    g.replay()
    torch.cuda.synchronize()
    assert E.captured_heavy_cells(clear=True)
    E.verify_captured_failures(clear=True)
    assert torch.equal(out.cpu(), E.knn_distances(data, k).cpu())  # exact, only unrefined
