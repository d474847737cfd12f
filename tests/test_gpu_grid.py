"""Cell-grid k-NN pass (knn_grid.hip): grid tables against a torch reference, and the
k-th distances bit for bit against the C++ CPU oracle on every data distribution."""
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


def grid_knn(p, k, max_radius=math.inf, mode="on"):
    old = E.GRID
    E.GRID = mode
    try:
        cfg = E.KnnConfig(k=k, max_radius=max_radius)
        idx = E.build_index(p.to(DEV), grid=True)
        st = E.KnnStats()
        out = torch.empty(idx.n, dtype=torch.float32, device=DEV)
        E.query(idx, cfg, E.radius_hint(idx.box, idx.n, k), stats=st, final_out=out)
        return out.cpu(), idx, st
    finally:
        E.GRID = old


@pytest.mark.parametrize("n", [1, 100, 5000, 200_003])
def test_grid_slots_match_torch(n):
    """Every level-`lc` cell's 64 slots hold its grandchildren's runs of the sorted array
    in curve order: (start, end, packed coordinates) — checked against a torch rebuild."""
    p = uniform(n, seed=n).to(DEV)
    idx = E.build_index(p)
    box = idx.box.cpu()
    keys, _ = K.morton(idx.pts[:n].cpu(), box)  # curve keys of the sorted points
    for lc in (0, 2, 4):
        g = lc + 2
        slots = K.grid_build(idx.pts, keys.to(DEV), n, idx.box, lc).cpu().to(torch.int64)
        q = ((idx.pts[:n].cpu() - box[0:3]) * box[6]).clamp(0, 1023).to(torch.int64) >> (10 - g)
        kg = (keys.to(torch.int64) & 0x3FFFFFFF) >> (3 * (10 - g))
        assert bool((kg[1:] >= kg[:-1]).all())  # sorted by the grandchild prefix
        cm = torch.zeros(n, dtype=torch.int64)
        c = q >> 2
        for b in range(lc):  # Morton index of the level-lc cell: x bit 2, y bit 1, z bit 0
            for a, sh in ((0, 2), (1, 1), (2, 0)):
                cm |= ((c[:, a] >> b) & 1) << (3 * b + sh)
        ref = torch.zeros((64 << (3 * lc), 4), dtype=torch.int64)
        uniq, cnt = torch.unique_consecutive(kg, return_counts=True)
        starts = torch.cumsum(cnt, 0) - cnt
        row = cm[starts] * 64 + (uniq & 63)
        ref[row, 0] = starts
        ref[row, 1] = starts + cnt
        ref[row, 2] = q[starts, 0] | (q[starts, 1] << 10) | (q[starts, 2] << 20)
        assert torch.equal(slots[:, :3], ref[:, :3]), lc


@pytest.mark.parametrize("dist", list(GENERATORS))
@pytest.mark.parametrize("k", [1, 8, 16, 100])
def test_grid_knn_matches_oracle(dist, k):
    p = GENERATORS[dist](30000, seed=k + 7)
    ref = oracle(p, k)
    got, idx, st = grid_knn(p, k)
    assert idx.grid is not None
    bad = (got != ref) & ~(torch.isnan(got) & torch.isnan(ref))
    assert int(bad.sum()) == 0, f"{int(bad.sum())} mismatches; stats={st.counters}"
    assert torch.isfinite(got).all()


@pytest.mark.parametrize("k", [1, 5, 64, 100])
def test_grid_knn_cutoff(k):
    p = uniform(20000, seed=3)
    r = 0.02
    ref = oracle(p, k, r)
    got, _, _ = grid_knn(p, k, r)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("k", [1, 2, 16, 100])
def test_grid_knn_cutoff_below_first_range(k):
    """A cutoff at or below the start of the first range (round 6: with the clamped
    histogram add, an empty range left the query's own zero uncounted at k = 1 and the
    cutoff came back instead): the range then starts at 0; 0, tiny and large cutoffs."""
    p = uniform(20000, seed=3)
    for r in (0.0, 1e-4, 1e-3, 0.05, 1.0):
        got, _, _ = grid_knn(p, k, r)
        assert torch.equal(got, oracle(p, k, r)), (k, r)


def test_grid_knn_k_larger_than_n_and_tiny_sets():
    for n in (1, 2, 63, 64, 65, 130):
        p = uniform(n, seed=n)
        for k in (1, 3, 64, 200):
            got, _, _ = grid_knn(p, k)
            assert torch.equal(got, oracle(p, k)), (n, k)


def test_grid_uniform_large_equals_rows_bitwise():
    p = uniform(2_000_000, seed=11).to(DEV)
    for k in (16, 100):
        got, idx, st = grid_knn(p, k)
        old = E.KNN_IMPL
        idx.grid = None
        out = torch.empty(idx.n, dtype=torch.float32, device=DEV)
        E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, idx.n, k), final_out=out)
        assert E.KNN_IMPL == old
        assert torch.equal(got, out.cpu())
        assert st.counters.get("failed_lanes", 0) == 0


def test_grid_auto_skips_crowded_data():
    # mixed-scale data: a dense core far below one sub-cell of the global cube
    p = GENERATORS["mixed_scale"](200_000, seed=2).to(DEV)
    old = E.GRID
    E.GRID = "auto"
    try:
        idx = E.build_index(p, grid=True)
        assert idx.grid is not None and not idx.grid.applies()  # the device said no
        got = torch.empty(idx.n, dtype=torch.float32, device=DEV)
        E.reset_kernels_used()
        E.query(idx, E.KnnConfig(k=16), E.radius_hint(idx.box, idx.n, 16), final_out=got)
        assert E.kernels_used() == ["rows"]
        assert torch.equal(got.cpu(), oracle(p.cpu(), 16))
        idx = E.build_index(uniform(200_000, seed=2).to(DEV), grid=True)
        assert idx.grid is not None and idx.grid.applies()
    finally:
        E.GRID = old


def test_grid_level_from_counts():
    """The host picks the level from the point counts (no census read): the census's
    choice for uniform data, capped by the local table size."""
    assert [E.grid_level_for(n, n) for n in (10_000_000, 100_000_000, 1_000_000_000)] == [7, 8, 9]
    # a rank's share of a 3.2B-point global cube: level 10 would be a 16 GiB table
    assert E.grid_level_for(3_200_000_000, 100_000_000) == 9
    assert E.grid_level_for(1_000_000_000, 125_000_000) == 9


def _rows_output(idx, k):
    grid, idx.grid = idx.grid, None
    try:
        out = torch.empty(idx.n, dtype=torch.float32, device=DEV)
        E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, idx.n, k), final_out=out)
        return out
    finally:
        idx.grid = grid


def _sampled(p, out, k, nsamp):
    from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm
    from mpi_cuda_largescaleknn_amd.utils import verify as V

    r = V.sampled_exact(SingleComm(torch.device(DEV)), p, out, 0, p.shape[0], k, nsamp=nsamp)
    assert r["exact"] == r["samples"] >= min(nsamp, p.shape[0]) * 0.99, r


@pytest.mark.parametrize("k", [16, 100])
def test_grid_production_level_1e8(k):
    """1e8 uniform points: the level the 1e8 bench runs at (grandchildren at level 8). The
    grid kernel's whole output equals the bucket-tree kernel's bit for bit, and 131072
    sampled outputs are exact against all 1e8 points (brute-force counts)."""
    n = 100_000_000
    g = torch.Generator(device=DEV).manual_seed(123 + k)
    p = torch.rand((n, 3), generator=g, device=DEV)
    idx = E.build_index(p, grid=True)
    assert idx.grid is not None and idx.grid.level + 2 == 8 and idx.grid.applies()
    out = torch.empty(n, dtype=torch.float32, device=DEV)
    st = E.KnnStats()
    E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, n, k), stats=st, final_out=out)
    assert st.counters.get("failed_lanes", 0) == 0 and st.counters.get("fallback_queries", 0) == 0
    assert torch.equal(out, _rows_output(idx, k))
    del idx
    _sampled(p, out, k, 1 << 17)


@pytest.mark.parametrize("k", [16, 100])
def test_grid_forced_level9_subcube(k):
    """Grandchildren at level 9 (the 1B bench's level) on 2e7 points in a 1/64 sub-cube of
    the key cube (eight far corner points span the cube): same density per cell as 1B
    uniform points. Whole output grid == rows bitwise, plus exact samples."""
    n = 20_000_000
    g = torch.Generator(device=DEV).manual_seed(77 + k)
    p = torch.rand((n, 3), generator=g, device=DEV) * 0.25
    corners = torch.tensor([[x, y, z] for x in (0.0, 1.0) for y in (0.0, 1.0) for z in (0.0, 1.0)],
                           device=DEV)
    p[:8] = corners
    idx = E.build_index(p, grid=True, grid_level=9)
    assert idx.grid.level + 2 == 9 and idx.grid.applies()
    out = torch.empty(n, dtype=torch.float32, device=DEV)
    E.query(idx, E.KnnConfig(k=k), E.radius_hint(idx.box, n, k), final_out=out)
    assert torch.equal(out, _rows_output(idx, k))
    del idx
    _sampled(p, out, k, 1 << 14)


def test_grid_knn_large_k_counter_wraps():
    """k in the thousands: a histogram pass makes tens of thousands of adds per lane, so
    16-bit bin counters (two lanes per dword in the paired-lane layout) can wrap; every
    wrap must be caught (checksum -> exact backstop) and the output stay exact."""
    p = uniform(120_000, seed=5)
    for k in (2000, 6000):
        got, _, st = grid_knn(p, k)
        assert torch.equal(got, oracle(p, k)), (k, st.counters)


@pytest.mark.parametrize("expect", [True, False])
def test_gate_misprediction_runs_the_persistent_form(expect, monkeypatch):
    """The kernel the gate is not expected to pick gets a small persistent (strided)
    launch: a wrong expectation still gives exact results — uniform data with the rows
    kernel expected (the grid kernel strides), mixed-scale data with the grid expected
    (the rows kernel strides)."""
    monkeypatch.setattr(E, "GRID", "auto")
    for gen in ("uniform", "mixed_scale"):
        p = GENERATORS[gen](120_000, seed=4)
        monkeypatch.setattr(E, "GRID_EXPECT", [expect])
        idx = E.build_index(p.to(DEV), grid=True)
        out = torch.empty(idx.n, dtype=torch.float32, device=DEV)
        E.query(idx, E.KnnConfig(k=32), E.radius_hint(idx.box, idx.n, 32), final_out=out)
        assert torch.equal(out.cpu(), oracle(p, 32)), gen
        assert E.GRID_EXPECT[0] == (gen == "uniform")  # updated from the decision


@pytest.mark.parametrize("gen", ["uniform", "mixed_scale"])
def test_short_group_list_strided_launch(gen, monkeypatch):
    """A device-counted group list far shorter than its bound (a rank's boundary groups)
    runs in the persistent strided form at full occupancy (short_list): the listed groups
    get exactly the whole-set result, the others stay untouched — grid (uniform) and rows
    (mixed-scale: the gate picks knn_rows) kernels, with the count below the bound."""
    monkeypatch.setattr(E, "GRID", "auto")
    p = GENERATORS[gen](200_000, seed=6)
    idx = E.build_index(p.to(DEV), grid=True)
    cfg = E.KnnConfig(k=100)
    hint2 = E.radius_hint(idx.box, idx.n, 100)
    full = E.query(idx, cfg, hint2)
    ng = (idx.n + 63) // 64
    g = torch.Generator().manual_seed(1)
    sel = torch.randperm(ng, generator=g)[:ng // 20].sort().values.to(torch.int32)
    lst = torch.full((ng,), -1, dtype=torch.int32)
    lst[:sel.numel()] = sel
    cnt = torch.tensor([sel.numel()], dtype=torch.int32)
    d2 = torch.full((idx.n,), -7.0, device=DEV)
    E.query(idx, cfg, hint2, out=d2, groups=lst.to(DEV), ngroups=ng, ngroups_dev=cnt.to(DEV),
            short_list=True)
    rows = (sel.long()[:, None] * 64 + torch.arange(64)[None, :]).reshape(-1)
    rows = rows[rows < idx.n]
    assert torch.equal(d2.cpu()[rows], full.cpu()[rows])
    mask = torch.ones(idx.n, dtype=torch.bool)
    mask[rows] = False
    assert bool((d2.cpu()[mask] == -7.0).all())


@pytest.mark.parametrize("gen", ["uniform", "mixed_scale"])
def test_chunked_pass_equals_one_launch(gen, monkeypatch):
    """A pass sent as several launches over consecutive wave ranges (chunks: kernel
    boundaries for the high-priority streams) gives exactly the one-launch result — the
    whole set, and a device-counted group list — on the grid (uniform) and rows (mixed-
    scale: the gate picks knn_rows) kernels."""
    monkeypatch.setattr(E, "GRID", "auto")
    p = GENERATORS[gen](150_001, seed=8)
    idx = E.build_index(p.to(DEV), grid=True)
    cfg = E.KnnConfig(k=32)
    hint2 = E.radius_hint(idx.box, idx.n, 32)
    one = E.query(idx, cfg, hint2)
    for c in (2, 3, 7):
        assert torch.equal(E.query(idx, cfg, hint2, chunks=c), one), c
    ng = (idx.n + 63) // 64
    lst = torch.arange(0, ng, 3, dtype=torch.int32)
    cnt = torch.tensor([lst.numel() - 5], dtype=torch.int32)
    full = torch.full((ng,), -1, dtype=torch.int32)
    full[:lst.numel()] = lst
    outs = []
    # (short_list: the persistent form, whose waves take groups from one work-queue
    # counter per launch — four chunks, four counters)
    for c, sl in ((1, False), (4, False), (1, True), (4, True)):
        d2 = torch.zeros(idx.n, device=DEV)
        E.query(idx, cfg, hint2, out=d2, groups=full.to(DEV), ngroups=ng, ngroups_dev=cnt.to(DEV), chunks=c,
                short_list=sl)
        outs.append(d2)
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    rows = (lst[:cnt.item()].long()[:, None] * 64 + torch.arange(64)[None, :]).reshape(-1)
    rows = rows[rows < idx.n]
    assert torch.equal(outs[1].cpu()[rows], one.cpu()[rows])


def _two_source(p, h, k, r=math.inf, groups=None, grid_halo=True, init=True):
    """Local index over p, halo index over h (with a grid at the local level unless
    grid_halo=False), a local pass, then the re-query of `groups` (all: None) against both
    sources with the local k-th as the upper bound — the distributed halo re-query."""
    old = E.GRID
    E.GRID = "on"
    try:
        cfg = E.KnnConfig(k=k, max_radius=r)
        idx = E.build_index(p.to(DEV), grid=True)
        hidx = E.build_index(h.to(DEV), grid=grid_halo, grid_level=idx.grid.level + 2 if grid_halo else None,
                             grid_gated=False)
        hint = E.radius_hint(idx.box, idx.n, k)
        d2 = E.query(idx, cfg, hint)
        ng = (idx.n + 63) // 64
        if groups is None:
            groups = torch.arange(ng, dtype=torch.int32, device=DEV)
        cnt = torch.tensor([groups.numel()], dtype=torch.int32, device=DEV)
        st = E.KnnStats()
        out = d2.clone()
        E.query(idx, cfg, hint, extra=hidx, groups=groups, ngroups=ng, ngroups_dev=cnt, short_list=True,
                out=out, init_d2=d2.clone() if init else None, stats=st)
        return out, d2, idx, st
    finally:
        E.GRID = old


@pytest.mark.parametrize("k", [1, 16, 100])
def test_grid_two_sources_match_oracle(k):
    """knn_grid2 (the halo re-query on the grid: local grid + the halo's own grid, the
    local k-th as the first range's top): bitwise equal to the CPU oracle over the union,
    with a cutoff, and equal to the bucket-tree kernel's two-tree re-query."""
    p = uniform(60_000, seed=11)
    h = uniform(8_000, seed=12) * 0.3 + torch.tensor([1.0, 0.2, 0.4])  # a slab beside p's cube
    allp = torch.cat([p, h])
    for r in (math.inf, 0.03):
        out, _, idx, st = _two_source(p, h, k, r)
        ref = K.kth_cpu(allp, idx.pts[:idx.n].cpu(), k, E.cut2_of(r))
        assert torch.equal(out.cpu().view(torch.int32), ref.view(torch.int32)), (k, r)
        assert st.counters.get("fallback_queries", 0) == 0
        rows, _, _, _ = _two_source(p, h, k, r, grid_halo=False)
        assert torch.equal(out.cpu().view(torch.int32), rows.cpu().view(torch.int32)), (k, r)


def test_grid_two_sources_listed_groups_and_no_bound():
    """Only listed groups change; without the upper bound (init_d2) the two-source pass
    starts from the density estimate and gives the same bits."""
    k = 24
    p = uniform(40_000, seed=21)
    h = uniform(5_000, seed=22) * torch.tensor([0.2, 1.0, 1.0]) + torch.tensor([-0.2, 0.0, 0.0])
    groups = torch.arange(0, (40_000 + 63) // 64, 3, dtype=torch.int32, device=DEV)
    out, d2, idx, _ = _two_source(p, h, k, groups=groups)
    nob, _, _, _ = _two_source(p, h, k, groups=groups, init=False)
    assert torch.equal(out.view(torch.int32), nob.view(torch.int32))
    rows = (groups.to(torch.int64)[:, None] * 64 + torch.arange(64, device=DEV)[None, :]).reshape(-1)
    rows = rows[rows < idx.n].cpu()
    ref = K.kth_cpu(torch.cat([p, h]), idx.pts[:idx.n].cpu()[rows], k, math.inf)
    assert torch.equal(out.cpu()[rows].view(torch.int32), ref.view(torch.int32))
    keep = torch.ones(idx.n, dtype=torch.bool)
    keep[rows] = False
    assert torch.equal(out.cpu()[keep], d2.cpu()[keep])  # unlisted groups untouched
