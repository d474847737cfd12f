"""Host timeline of the forced 1-rank stream of sets: where does the host wait?
(host timestamps around the k-NN launch, the failure-word staging and the next set's
redistribution; `busy` = the compute stream still has work queued)."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import launch as LA  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import pipelines as PL  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.stream import SetStream  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
os.environ.setdefault("LSKNN_TIMEOUT", "600")
launch = LA.init(force_distributed=True)
comm, dev = launch.comm, launch.device
T0 = time.perf_counter()
LOG = []


def log(tag):
    LOG.append((time.perf_counter() - T0, tag, torch.cuda.current_stream(dev).query()))


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **kw):
        log(f"> {name}")
        r = f(*a, **kw)
        log(f"< {name}")
        return r
    setattr(mod, name, g)


wrap(E, "query")
POLL = []


def poll_events(tagged):
    """Background thread: host time at which each (tag, event) completes."""
    import threading

    def run():
        pending = list(tagged)
        while pending:
            for item in list(pending):
                if item[1].query():
                    LOG.append((time.perf_counter() - T0, f"   done {item[0]}", None))
                    pending.remove(item)
            time.sleep(0.0002)
    th = threading.Thread(target=run, daemon=True)
    th.start()
    POLL.append(th)


_rs = PL.redistribute_set


def redistribute_set(*a, **kw):
    # events at entry: the redistribution stream (after its waits), the copy stream, and the
    # compute stream (after the k-NN just queued)
    st = {}
    for nm, s_ in (("redist(entry)", torch.cuda.current_stream(dev)), ("copy", RUNNER[0].copy_stream),
                   ("compute", torch.cuda.default_stream(dev))):
        e = torch.cuda.Event()
        e.record(s_)
        st[nm] = e
    poll_events(list(st.items()))
    return _rs(*a, **kw)


PL.redistribute_set = redistribute_set
RUNNER = []
wrap(PL, "redistribute_set")
wrap(K.FailWord, "stage")
wrap(K.FailWord, "value")
wrap(E, "build_index")
wrap(PL, "global_box")
wrap(PL, "redistribute")
sets = []
for s in range(2):
    g = torch.Generator().manual_seed(s)
    sets.append(torch.rand((n, 3), generator=g).pin_memory())
outs = [torch.empty(n, dtype=torch.float32).pin_memory() for _ in range(2)]
runner = SetStream(comm, E.KnnConfig(k=100), direct_out=False)
RUNNER.append(runner)
runner.run([sets[i % 2] for i in range(3)], [outs[i % 2] for i in range(3)], n_totals=[n] * 3)
torch.cuda.synchronize()
LOG.clear()
T0 = time.perf_counter()
runner.run([sets[i % 2] for i in range(5)], [outs[i % 2] for i in range(5)], n_totals=[n] * 5)
torch.cuda.synchronize()
for t, tag, idle in sorted(LOG, key=lambda x: x[0]):
    print(f"{t * 1e3:9.2f} ms  {'' if idle is None else ('idle' if idle else 'busy')}  {tag}")
LA.finalize(launch)
