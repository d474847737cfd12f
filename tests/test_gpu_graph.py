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
    with torch.cuda.graph(g):
        body()
    torch.cuda.synchronize()

    for data in (uniform(n, seed=1), clustered(n, seed=2), uniform(n, seed=3) * 7.0 - 2.0):
        host_pts.copy_(data)
        host_out.fill_(-1.0)
        g.replay()
        torch.cuda.synchronize()
        ref = E.knn_distances(data.to(DEV), k).cpu()
        assert torch.equal(host_out, ref)
