"""Flat data in a rotated index frame (knn_engine.flat_frame / _build_rotated): keys, tree
boxes and box tests in the principal-axes frame, canonical distances in the points' own —
bit for bit against the CPU oracle, and the frame is only taken for flat, non-axis-aligned
sets."""
import math

import pytest
import torch

from datasets import GENERATORS, uniform
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.ops import kernels as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def oracle(points, k, max_radius=math.inf):
    return K.finalize_distances(K.kth_cpu(points, points, k, E.cut2_of(max_radius)))


def _random_plane(n, seed):
    g = torch.Generator().manual_seed(seed)
    uv = torch.rand((n, 2), generator=g) * 2 - 1
    a, b = torch.tensor([0.6, -0.3, 0.74]), torch.tensor([0.2, 0.9, 0.1])
    a = a / a.norm()
    b = b - (b @ a) * a
    b = b / b.norm()
    return (uv[:, :1] * a + uv[:, 1:] * b + torch.tensor([3.0, -1.0, 0.5])).contiguous()


@pytest.mark.parametrize("keys", ["3d", "2d"])
@pytest.mark.parametrize("gen", ["tilted_plane", "random_plane"])
@pytest.mark.parametrize("k", [1, 8, 100])
def test_flat_sets_rotated_frame_exact(gen, k, keys, monkeypatch):
    """3d: the curve keys of the rotated points; 2d: 2-D Morton keys of the in-plane axes
    (the default above PLANE_2D_MIN points)."""
    monkeypatch.setattr(E, "PLANE_KEYS", keys)
    p = _random_plane(120_000, 3) if gen == "random_plane" else GENERATORS[gen](120_000, seed=2)
    assert E.flat_frame(p.to(DEV)) is not None
    old = E.FRAME_MIN_K
    E.FRAME_MIN_K = 1  # (the rotated path for every k here)
    try:
        _check(p, k, gen)
    finally:
        E.FRAME_MIN_K = old


def _check(p, k, gen):
    for r in (math.inf, 0.01):
        st = E.KnnStats()
        got = E.knn_distances(p.to(DEV), k, max_radius=r, stats=st).cpu()
        assert torch.equal(got.view(torch.int32), oracle(p, k, r).view(torch.int32)), (gen, k, r)


def test_flat_frame_only_for_unaligned_planes():
    assert E.flat_frame(uniform(50_000, seed=1).to(DEV)) is None  # 3-D
    assert E.flat_frame(GENERATORS["planar"](50_000, seed=1).to(DEV)) is None  # axis-aligned plane
    assert isinstance(E.flat_frame(GENERATORS["line"](50_000, seed=1).to(DEV)), E.LineAxis)  # not rotated
    assert E.flat_frame(GENERATORS["tilted_plane"](50_000, seed=1).to(DEV)) is not None


@pytest.mark.parametrize("k", [1, 16, 100])
def test_rotated_frame_on_a_line_stays_exact(k):
    """An index built in a line's principal frame (not chosen by flat_frame, which keeps
    lines in their own frame for speed) still gives the oracle's bits."""
    import numpy as np
    p = GENERATORS["line"](60_000, seed=4)
    c = (p - p.mean(0)).double()
    w, v = np.linalg.eigh((c.T @ c).numpy())
    R = torch.tensor(v[:, ::-1].T.copy(), dtype=torch.float32, device=DEV)
    idx = E.build_index(p.to(DEV), frame=R)
    out = torch.empty(idx.n, dtype=torch.float32, device=DEV)
    E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, idx.n, k), final_out=out)
    assert torch.equal(out.cpu().view(torch.int32), oracle(p, k).view(torch.int32))


def test_rotated_index_boxes_contain_rotated_points():
    """Every bucket box (widened by the rotation margin) holds its points' rotated
    coordinates; the index's points are the input points in sorted order."""
    p = GENERATORS["tilted_plane"](70_000, seed=5).to(DEV)
    R = E.flat_frame(p)
    idx = E.build_index(p, frame=R)
    n, d = idx.n, idx.depth
    assert idx.qrot is not None and idx.grid is None
    assert torch.equal(idx.pts[:n], p[idx.perm.long()])
    leaves = idx.nodes[1 << d:(1 << d) + (n + 63) // 64]
    q = idx.qrot[:n]
    b = torch.arange(n, device=DEV) // 64
    assert bool((q >= leaves[b, 0:3]).all()) and bool((q <= leaves[b, 4:7]).all())


def test_dense_planes_keep_their_own_frame(monkeypatch):
    """The frame is refused once the plane's k-NN radius nears the boxes' rotation margin
    (FRAME_RADIUS_X: measured loss at 2e8 points, k = 100)."""
    p = GENERATORS["tilted_plane"](50_000, seed=1).to(DEV)
    assert E.flat_frame(p) is not None
    monkeypatch.setattr(E, "FRAME_RADIUS_X", 1e4)
    assert E.flat_frame(p) is None


def test_axis_aligned_plane_takes_the_frame_with_2d_keys(monkeypatch):
    """Above PLANE_2D_MIN an axis-aligned plane is indexed in its frame too (for the 2-D
    keys); still bit-exact."""
    p = GENERATORS["planar"](100_000, seed=3)
    assert E.flat_frame(p.to(DEV)) is None
    monkeypatch.setattr(E, "PLANE_2D_MIN", 50_000)
    monkeypatch.setattr(E, "FRAME_MIN_K", 1)
    assert E.flat_frame(p.to(DEV)) is not None
    _check(p, 16, "planar")


def _random_line(n, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand(n, generator=g) * 2 - 1
    a = torch.tensor([-0.35, 0.8, 0.49])
    return (t[:, None] * (a / a.norm()) + torch.tensor([1.5, 0.25, -2.0])).contiguous()


def _axis_line(n, seed):
    g = torch.Generator().manual_seed(seed)
    p = torch.full((n, 3), 0.5)
    p[:, 1] = torch.rand(n, generator=g)
    return p


@pytest.mark.parametrize("gen", ["line", "random_line", "axis_line"])
@pytest.mark.parametrize("k", [1, 16, 100])
def test_lines_sorted_along_their_axis_exact(gen, k):
    """A line keeps its own frame and is sorted by its position along the axis (line_keys):
    bit-exact against the oracle; the index's points are in axis order."""
    p = {"random_line": _random_line, "axis_line": _axis_line}.get(gen, lambda n, s: GENERATORS["line"](n, seed=s))(
        90_000, 7)
    f = E.flat_frame(p.to(DEV))
    assert isinstance(f, E.LineAxis)
    idx = E.build_index(p.to(DEV), frame=f)
    assert idx.qrot is None and idx.grid is None
    t = (idx.pts[:idx.n] @ f.a).cpu()
    assert bool((t[1:] >= t[:-1] - 1e-5).all())
    _check(p, k, gen)
