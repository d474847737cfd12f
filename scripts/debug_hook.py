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
runner.run([sets[i % 2] for i in range(3)], [outs[i % 2] for i in range(3)], n_totals=[n] * 3)
torch.cuda.synchronize()
LOG.clear()
T0 = time.perf_counter()
runner.run([sets[i % 2] for i in range(5)], [outs[i % 2] for i in range(5)], n_totals=[n] * 5)
torch.cuda.synchronize()
for t, tag, idle in LOG:
    print(f"{t * 1e3:9.2f} ms  {'idle' if idle else 'busy'}  {tag}")
LA.finalize(launch)
