"""T1: the CPU oracle and the CPU path of the engine (exact k-th-distance semantics)."""
import math

import pytest
import torch

from datasets import GENERATORS, lattice, uniform
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.ops import kernels as K


def brute_reference(points, queries, k, max_radius=math.inf):
    """Plain PyTorch fp32 reference: same canonical dist² association as the kernels."""
    cut2 = E.cut2_of(max_radius)
    out = []
    for q in queries:
        dx = (q[0] - points[:, 0])
        dy = (q[1] - points[:, 1])
        dz = (q[2] - points[:, 2])
        d2 = torch.addcmul(torch.addcmul(dx * dx, dy, dy), dz, dz)  # unfused on CPU = fma order?
        d2 = d2[d2 < cut2]
        if d2.numel() < k:
            out.append(cut2)
        else:
            out.append(torch.kthvalue(d2, k).values.item())
    return torch.tensor(out, dtype=torch.float32)


@pytest.mark.parametrize("dist", list(GENERATORS))
@pytest.mark.parametrize("k", [1, 4, 33, 100])
def test_kdtree_equals_brute(dist, k):
    p = GENERATORS[dist](3000, seed=k)
    a = K.kth_cpu(p, p, k, math.inf, "kdtree")
    b = K.kth_cpu(p, p, k, math.inf, "brute")
    assert torch.equal(a, b)


def test_brute_close_to_torch_reference():
    # torch's own fp32 arithmetic may associate differently: compare to within 1 ulp-ish
    p = uniform(500, seed=3)
    a = K.kth_cpu(p, p, 10, math.inf, "brute")
    b = brute_reference(p, p, 10)
    assert torch.allclose(a, b, rtol=1e-6, atol=0)


@pytest.mark.parametrize("r", [0.0, 0.01, 0.05, 0.2, math.inf])
def test_cutoff_semantics(r):
    p = uniform(2000, seed=5)
    k = 20
    got = K.kth_cpu(p, p, k, E.cut2_of(r), "kdtree")
    cut2 = E.cut2_of(r)
    d2 = ((p[:, None, :] - p[None, :, :]) ** 2).sum(-1)
    for i in range(0, 2000, 97):
        row = d2[i][d2[i] < cut2]
        # exact count semantics: fewer than k below cut2 -> cut2
        if row.numel() < k:
            assert got[i].item() == cut2
        else:
            assert got[i].item() < cut2


def test_k_larger_than_n_is_inf():
    p = uniform(10, seed=1)
    assert torch.isinf(K.kth_cpu(p, p, 11, math.inf)).all()
    assert torch.all(K.kth_cpu(p, p, 10, math.inf) < math.inf)


def test_self_counts_and_duplicates():
    p = torch.tensor([[0.0, 0, 0], [0.0, 0, 0], [1.0, 0, 0]])
    d2 = K.kth_cpu(p, p, 2, math.inf)
    assert d2.tolist() == [0.0, 0.0, 1.0]


def test_engine_cpu_path_matches_brute():
    for dist in GENERATORS:
        p = GENERATORS[dist](4000, seed=11)
        got = E.knn_distances(p, 16)
        ref = K.finalize_distances(K.kth_cpu(p, p, 16, math.inf, "brute"))
        assert torch.equal(got, ref), dist


def test_lattice_ties_cpu():
    p = lattice(10)
    for k in [1, 7, 27]:
        a = K.kth_cpu(p, p, k, math.inf, "kdtree")
        b = K.kth_cpu(p, p, k, math.inf, "brute")
        assert torch.equal(a, b)


def test_bucket_tree_cpu_invariants():
    p = uniform(5000, seed=2)
    idx = E.build_index(p)
    n, d = idx.n, idx.depth
    assert (1 << d) * 64 >= n
    leaves = idx.nodes[(1 << d):]
    for b in range(0, (n + 63) // 64, 7):
        pts = idx.pts[b * 64:min(n, b * 64 + 64)]
        assert torch.equal(leaves[b, 0:3], pts.min(0).values)
        assert torch.equal(leaves[b, 4:7], pts.max(0).values)
    # parents contain children
    for node in range(1, 1 << d):
        par, l, r = idx.nodes[node], idx.nodes[2 * node], idx.nodes[2 * node + 1]
        assert torch.all(par[0:3] <= torch.minimum(l[0:3], r[0:3]))
    # perm is a permutation and pts are the permuted input
    assert torch.equal(torch.sort(idx.perm.long()).values, torch.arange(n))
    assert torch.equal(idx.pts[:n], p[idx.perm.long()])


def _fp64_kth(p, k, r=math.inf, chunk=512):
    """Independent float64 brute force (PyTorch): k-th smallest true squared distance
    among points with d2 < r^2 (self counted), r^2 if fewer than k qualify."""
    pd = p.double()
    r2 = r * r
    out = torch.empty(p.shape[0], dtype=torch.float64)
    for s in range(0, p.shape[0], chunk):
        q = pd[s:s + chunk]
        d2 = ((q[:, None, :] - pd[None, :, :]) ** 2).sum(-1)
        d2 = torch.where(d2 < r2, d2, torch.full_like(d2, math.inf))
        kth = torch.kthvalue(d2, min(k, d2.shape[1]), dim=1).values
        out[s:s + chunk] = torch.where(torch.isinf(kth), torch.full_like(kth, r2), kth)
    return out


@pytest.mark.parametrize("k", [1, 10, 100])
def test_oracle_against_fp64_brute_force_20k(k):
    """The C++ oracle (fp32 canonical d2) agrees with an fp64 PyTorch brute force on 20K
    points to within the rounding of fp32 d2 (a few ulp)."""
    p = uniform(20000, seed=21)
    got = K.kth_cpu(p, p, k, math.inf, "kdtree").double()
    ref = _fp64_kth(p, k)
    rel = ((got - ref).abs() / ref.clamp_min(1e-30))
    assert float(rel.max()) < 5e-7, float(rel.max())


@pytest.mark.parametrize("k,r", [(7, math.inf), (27, math.inf), (30, 0.13), (200, 0.1)])
def test_oracle_against_fp64_lattice_ties_and_cutoff(k, r):
    """Lattice points (coordinates j/16, every d2 exact in fp32): massive ties; the fp32
    oracle must equal the fp64 brute force exactly, also with a -r cutoff."""
    p = lattice(16)
    got = K.kth_cpu(p, p, k, E.cut2_of(r), "kdtree").double()
    ref = _fp64_kth(p, k, r)
    if math.isinf(r):
        assert torch.equal(got, ref)
    else:
        # cutoff: same set of outputs; the "fewer than k" value is fp32(r)^2 in fp32
        short = ref == r * r
        assert torch.equal(got[~short], ref[~short])
        assert torch.all(got[short] == float(E.cut2_of(r)))
