"""What does the result copy cost a stream of 1B-point sets? (tuning probe)

    python scripts/stream_d2h_probe.py [n] [sets] [mode ...]

Runs SetStream over `sets` alternating sets of n uniform points (pinned host memory, as
bench.py) per mode and prints ms per set (after the first two sets):
  copy     production: the result goes to pinned host memory on the output stream
  nocopy   the result stays on the device (wrong for users: measures the copy's share)
Measured (profiles/r5_stream/): copy 885-896 ms per set in the steady state; a result
copy by a narrow-grid kernel of our own (8-32 workgroups, tried in round 5 and removed)
937-991 ms — the runtime's blit stays.
"""
import sys
import time

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel import stream as S  # noqa: E402
from mpi_cuda_largescaleknn_amd.parallel.comm import SingleComm  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
nsets = int(sys.argv[2]) if len(sys.argv) > 2 else 6
modes = sys.argv[3:] or ["copy", "nocopy", "copy"]
dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(3)
hosts = []
for s in range(2):
    h = torch.empty((n, 3), dtype=torch.float32, pin_memory=True)
    h.copy_(torch.rand((n, 3), generator=g))
    hosts.append(h)
outs = [torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(2)]


class NoCopy(S.SetStream):
    def _release(self, rec, outputs, after=None):
        j, res, ev, pend = rec
        E.settle(pend)
        return j, ev


for mode in modes:
    cls = NoCopy if mode == "nocopy" else S.SetStream
    runner = cls(SingleComm(dev), E.KnnConfig(k=100), direct_out=False)
    for rep in range(2):  # rep 0: first use of the runner (allocations); rep 1: as bench.py's timed run
        stamps = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        runner.run([hosts[i % 2] for i in range(nsets)], [outs[i % 2] for i in range(nsets)],
                   on_done=lambda i: stamps.append(time.perf_counter()))
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t0) * 1e3
        per = (stamps[-1] - stamps[1]) / (len(stamps) - 2) * 1e3 if len(stamps) > 2 else float("nan")
        print(f"{mode} run {rep}: {per:.1f} ms per set (steady state over {len(stamps) - 2} sets), "
              f"total {tot:.0f} ms = {tot / nsets:.1f} ms per set; first set done at "
              f"{(stamps[0] - t0) * 1e3:.0f} ms", flush=True)
