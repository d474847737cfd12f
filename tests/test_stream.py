"""SetStream (parallel/stream.py): a stream of point sets through the unordered pipeline,
the next set's upload (and on several ranks the previous set's result download)
overlapped with the current set's k-NN. Every set's output equals the one-set-at-a-time
oracle bit for bit — on the CPU (loopback ranks, sequential) and on the GPU (streams)."""
import pytest
import torch

from datasets import GENERATORS
from mpi_cuda_largescaleknn_amd.models import knn_engine as E
from mpi_cuda_largescaleknn_amd.ops import kernels as K
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm, run_loopback
from mpi_cuda_largescaleknn_amd.parallel.stream import SetStream


def oracle(p, k):
    return K.finalize_distances(K.kth_cpu(p, p, k, E.cut2_of(float("inf"))))


def sets():
    # different sizes and distributions, one set repeated (buffer reuse)
    a = GENERATORS["uniform"](5000, seed=1)
    b = GENERATORS["clustered"](7000, seed=2)
    c = GENERATORS["duplicates"](3000, seed=3)
    return [a, b, c, a]


@pytest.mark.parametrize("size", [1, 2, 3])
def test_stream_loopback_cpu(size):
    k = 10
    cfg = E.KnnConfig(k=k, publish_levels=4)
    S = sets()

    def fn(comm):
        ins, outs = [], []
        for p in S:
            b, e = p.shape[0] * comm.rank // comm.size, p.shape[0] * (comm.rank + 1) // comm.size
            ins.append(p[b:e].contiguous())
            outs.append(torch.empty(e - b, dtype=torch.float32))
        SetStream(comm, cfg).run(ins, outs, n_totals=[p.shape[0] for p in S])
        return outs

    per_rank = run_loopback(size, fn)
    for i, p in enumerate(S):
        got = torch.cat([per_rank[r][i] for r in range(size)])
        assert torch.equal(got, oracle(p, k)), i


@pytest.mark.parametrize("size", [1, 2, 3])
def test_stream_prepartitioned_loopback_cpu(size):
    """variant="prepartitioned": every rank's set is its own spatial slab (a file per
    rank); the concatenated outputs equal the oracle of the union, set by set."""
    k = 9
    cfg = E.KnnConfig(k=k, publish_levels=4)
    S = [GENERATORS["uniform"](4000, seed=4), GENERATORS["clustered"](5000, seed=8)]
    slabs = []
    for p in S:
        order = torch.argsort(p[:, 0], stable=True)  # x slabs: one "file" per rank
        slabs.append(p[order].contiguous())

    def fn(comm):
        ins, outs = [], []
        for p in slabs:
            b, e = p.shape[0] * comm.rank // comm.size, p.shape[0] * (comm.rank + 1) // comm.size
            ins.append(p[b:e].contiguous())
            outs.append(torch.empty(e - b, dtype=torch.float32))
        SetStream(comm, cfg, variant="prepartitioned").run(ins, outs)
        return outs

    per_rank = run_loopback(size, fn)
    for i, p in enumerate(slabs):
        assert torch.equal(torch.cat([per_rank[r][i] for r in range(size)]), oracle(p, k)), i


def test_stream_length_mismatch():
    with pytest.raises(ValueError):
        SetStream(SingleComm("cpu"), E.KnnConfig(k=4)).run([torch.zeros(10, 3)], [])


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
@pytest.mark.parametrize("pre", [True, False])
def test_stream_single_gpu(direct, pre):
    """One rank on the GPU: pinned host sets of different sizes (the device buffers are
    reallocated), the kernel writing the pinned outputs directly (or device results copied
    back), the next set's box and curve keys computed on the side stream beside the
    current k-NN (PRE_KEYS) or at the head of its build, equal to the CPU oracle."""
    k = 16
    cfg = E.KnnConfig(k=k)
    dev = torch.device("cuda", torch.cuda.current_device())
    S = sets() + [GENERATORS["uniform"](30_000, seed=5)]
    ins = [p.pin_memory() for p in S]
    outs = [torch.full((p.shape[0],), -1.0).pin_memory() for p in S]
    runner = SetStream(SingleComm(dev), cfg, direct_out=direct, pre_keys=pre)
    runner.run(ins, outs)
    for i, p in enumerate(S):
        assert torch.equal(outs[i], oracle(p, k)), i
    assert runner.last_info is not None


@pytest.mark.parametrize("size", [1, 3])
def test_compute_set_hook_redistributes_next_set_cpu(size):
    """The multi-rank two-phase API with the overlap hook (SetStream's GPU path): set B is
    redistributed from inside set A's compute phase; both results equal the oracle."""
    k = 8
    cfg = E.KnnConfig(k=k, publish_levels=4)
    A = GENERATORS["uniform"](4000, seed=5)
    B = GENERATORS["clustered"](5000, seed=6)

    def part(p, comm):
        b, e = p.shape[0] * comm.rank // comm.size, p.shape[0] * (comm.rank + 1) // comm.size
        return p[b:e].contiguous()

    def fn(comm):
        comm.force = True  # the multi-rank path even on one rank
        PA = PL.redistribute_set(part(A, comm), comm, cfg, A.shape[0])
        nxt = {}

        def hook(after):
            nxt["P"] = PL.redistribute_set(part(B, comm), comm, cfg, B.shape[0])
            return None

        ra = PL.compute_set(PA, comm, cfg, hook=hook)
        rb = PL.compute_set(nxt["P"], comm, cfg)
        return ra, rb

    outs = run_loopback(size, fn)
    assert torch.equal(torch.cat([o[0] for o in outs]), oracle(A, k))
    assert torch.equal(torch.cat([o[1] for o in outs]), oracle(B, k))


class _Lazy:
    """A lazily materialised sequence that records accesses and what is alive."""

    def __init__(self, make, n):
        self.make, self.n, self.alive, self.log = make, n, {}, []

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        if i not in self.alive:
            self.alive[i] = self.make(i)
            self.log.append(i)
        return self.alive[i]


def _check_lazy_stream(dev, pin, direct):
    k = 12
    S = sets() * 2
    ins = _Lazy(lambda i: S[i].pin_memory() if pin else S[i].clone(), len(S))
    outs = _Lazy(lambda i: torch.full((S[i].shape[0],), -1.0).pin_memory() if pin
                 else torch.full((S[i].shape[0],), -1.0), len(S))
    done, peak = [], [0]

    def on_done(i):
        assert torch.equal(outs[i], oracle(S[i], k)), i
        done.append(i)
        ins.alive.pop(i)
        outs.alive.pop(i)

    def track(i):
        peak[0] = max(peak[0], len(ins.alive))

    ins_get = ins.__getitem__
    ins.__class__ = type("_LazyTracked", (_Lazy,), {"__getitem__": lambda self, i: (ins_get(i), track(i))[0]})
    SetStream(SingleComm(dev), E.KnnConfig(k=k), direct_out=direct).run(ins, outs, on_done=on_done)
    assert done == list(range(len(S)))
    assert not ins.alive and not outs.alive
    assert peak[0] <= 3  # only the sets in flight are materialised


def test_stream_lazy_sets_and_on_done_cpu():
    """Sets are read when reached and released in on_done (apps/stream.py's bounded host
    memory): callbacks in order, every output complete when its callback runs."""
    _check_lazy_stream(torch.device("cpu"), False, False)


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [True, False])
def test_stream_lazy_sets_and_on_done_gpu(direct):
    _check_lazy_stream(torch.device("cuda", torch.cuda.current_device()), True, direct)


@pytest.mark.gpu
@pytest.mark.parametrize("ahead", [False, True])
def test_stream_failure_overflow_rerun_gpu(ahead, monkeypatch):
    """every k-NN launch hands every 7th query to the backstop and the failure
    list holds only 16, so every set's failure word overflows and the host reruns the
    whole set on the exact kernel while the next set is already queued — set i's output
    copy must follow that rerun (SetStream._release), with and without the pre-computed keys (PRE_KEYS)
    modes, with lazy inputs / outputs released in on_done."""
    from mpi_cuda_largescaleknn_amd.ops import kernels as KK

    monkeypatch.setattr(E, "DEBUG_FAIL_MOD", 7)
    monkeypatch.setattr(KK, "FAIL_CAP_OVERRIDE", 16)
    dev = torch.device("cuda", torch.cuda.current_device())
    k = 12
    S = sets() + [GENERATORS["uniform"](40_000, seed=9)]
    ins = _Lazy(lambda i: S[i].pin_memory(), len(S))
    outs = _Lazy(lambda i: torch.full((S[i].shape[0],), -1.0).pin_memory(), len(S))
    done = []

    def on_done(i):
        assert torch.equal(outs[i], oracle(S[i], k)), i
        done.append(i)
        ins.alive.pop(i)
        outs.alive.pop(i)

    SetStream(SingleComm(dev), E.KnnConfig(k=k), direct_out=False, pre_keys=ahead).run(ins, outs, on_done=on_done)
    assert done == list(range(len(S)))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["unordered", "prepartitioned"])
@pytest.mark.parametrize("size", [2, 3])
def test_stream_distributed_loopback_gpu(variant, size):
    """The multi-rank stream on the GPU (loopback ranks as threads sharing cuda:0): next
    set's redistribution under the current k-NN, result copies under the next set, no
    host sync between sets; every set equals the oracle and on_done runs in order."""
    dev = torch.device("cuda", torch.cuda.current_device())
    k = 10
    cfg = E.KnnConfig(k=k, publish_levels=6)
    S = [GENERATORS["uniform"](20_000, seed=1), GENERATORS["clustered"](15_000, seed=2),
         GENERATORS["uniform"](25_000, seed=3)]
    if variant == "prepartitioned":
        S = [p[torch.argsort(p[:, 0], stable=True)].contiguous() for p in S]

    def fn(comm):
        ins, outs, order = [], [], []
        for p in S:
            b, e = p.shape[0] * comm.rank // comm.size, p.shape[0] * (comm.rank + 1) // comm.size
            ins.append(p[b:e].contiguous().pin_memory())
            outs.append(torch.full((e - b,), -1.0).pin_memory())
        SetStream(comm, cfg, variant=variant).run(ins, outs, on_done=order.append)
        assert order == list(range(len(S)))
        return outs

    per_rank = run_loopback(size, fn, dev)
    for i, p in enumerate(S):
        assert torch.equal(torch.cat([per_rank[r][i] for r in range(size)]), oracle(p, k)), i


@pytest.mark.gpu
def test_stream_learns_heavy_cells_gpu():
    """A stream of sets with over-full key cells (a dense core inside a large box): the
    first set's build checks eagerly and refines, and so does every later one (the data
    is known to have over-full cells); nothing is left unrefined; every output exact."""
    dev = torch.device("cuda", 0)
    p = GENERATORS["mixed_scale"](60_000, seed=4)
    q = GENERATORS["mixed_scale"](60_000, seed=5)
    S = [p, q, p, q]
    k = 20
    ins = [s.pin_memory() for s in S]
    outs = [torch.empty(s.shape[0], dtype=torch.float32).pin_memory() for s in S]
    E.deferred_heavy_cells(clear=True)
    E.LAST_REFINED = False
    old = E.HEAVY_RUN
    E.HEAVY_RUN = 512  # (the core's points share one key; a small set still has over-full runs)
    try:
        SetStream(SingleComm(dev), E.KnnConfig(k=k)).run(ins, outs)
    finally:
        E.HEAVY_RUN = old
    assert E.LAST_REFINED
    assert not E.deferred_heavy_cells(clear=True)
    for s, o in zip(S, outs):
        assert torch.equal(o, oracle(s, k))


@pytest.mark.gpu
def test_stream_clean_sets_stay_sync_free_gpu():
    """Uniform sets: the first build checks eagerly (clean), later builds defer their flag
    (no host read) and nothing is reported unrefined."""
    dev = torch.device("cuda", 0)
    S = [GENERATORS["uniform"](50_000, seed=s) for s in (1, 2, 3)]
    k = 16
    ins = [s.pin_memory() for s in S]
    outs = [torch.empty(s.shape[0], dtype=torch.float32).pin_memory() for s in S]
    E.deferred_heavy_cells(clear=True)
    SetStream(SingleComm(dev), E.KnnConfig(k=k)).run(ins, outs)
    assert E._HEAVY_KNOWN[0] is False or E._HEAVY_PENDING
    assert not E.deferred_heavy_cells(clear=True)
    for s, o in zip(S, outs):
        assert torch.equal(o, oracle(s, k))


@pytest.mark.gpu
def test_stream_after_clean_stream_checks_heavy_again_gpu():
    """a clean stream, then a stream with over-full cells in the same process.
    The second stream must not inherit the first one's clean verdict: its first set takes
    the eager check and refines, nothing is left unrefined, outputs exact."""
    dev = torch.device("cuda", 0)
    k = 16
    clean = [GENERATORS["uniform"](50_000, seed=s) for s in (1, 2)]
    E.deferred_heavy_cells(clear=True)
    SetStream(SingleComm(dev), E.KnnConfig(k=k)).run([s.pin_memory() for s in clean],
                                                     [torch.empty(s.shape[0]).pin_memory() for s in clean])
    assert E._HEAVY_KNOWN[0] is False or E._HEAVY_PENDING  # the clean verdict is known / pending
    heavy = [GENERATORS["mixed_scale"](60_000, seed=s) for s in (4, 5)]
    outs = [torch.empty(s.shape[0], dtype=torch.float32).pin_memory() for s in heavy]
    E.LAST_REFINED = False
    old = E.HEAVY_RUN
    E.HEAVY_RUN = 512
    try:
        SetStream(SingleComm(dev), E.KnnConfig(k=k)).run([s.pin_memory() for s in heavy], outs)
    finally:
        E.HEAVY_RUN = old
    assert E.LAST_REFINED
    assert not E.deferred_heavy_cells(clear=True)
    for s, o in zip(heavy, outs):
        assert torch.equal(o, oracle(s, k))


def test_new_stream_forgets_heavy_verdict_cpu():
    """SetStream.run resets what an earlier stream learned about over-full cells (but not
    the DEFERRED_HEAVY report)."""
    E.deferred_heavy_cells(clear=True)
    E._HEAVY_KNOWN[0] = False
    E._HEAVY_PENDING.append(("flag", "event"))
    E.DEFERRED_HEAVY.append(torch.tensor(False))
    E.new_heavy_stream()
    assert E._HEAVY_KNOWN[0] is None and not E._HEAVY_PENDING
    assert len(E.DEFERRED_HEAVY) == 1
    E.deferred_heavy_cells(clear=True)
