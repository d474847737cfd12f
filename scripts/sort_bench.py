"""Index-build pieces alone on N uniform points: curve keys, 4-pass key sort (iota values),
key census, gather, tree, grid; best of 3 each (events); checks the sort's output
(non-decreasing keys, a permutation, keys[perm] == sorted keys).

    python scripts/sort_bench.py [N]"""
import sys

import torch

sys.path.insert(0, ".")
from mpi_cuda_largescaleknn_amd.models import knn_engine as E  # noqa: E402
from mpi_cuda_largescaleknn_amd.ops import kernels as K  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
g = torch.Generator(device="cuda").manual_seed(1)
p = torch.rand((n, 3), generator=g, device="cuda")
box = K.bounds(p)


def t(fn, reps=3, setup=None):
    """Best of `reps` event-timed calls; `setup()` (untimed) makes each call's fresh input."""
    best, out = 1e9, None
    for _ in range(reps):
        arg = setup() if setup is not None else None
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        out = fn(arg) if setup is not None else fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return out, best


(keys,), t_keys = t(lambda: (K.morton(p, box, with_iota=False)[0],))
# the sort ping-pongs through its input buffer (an even pass count leaves the sorted keys
# there): every rep sorts a fresh copy of the unsorted keys, or reps 2-3 would sort sorted
# keys and the gather below would read an identity permutation
(sk, perm), t_sort = t(lambda kk: K.sort_keys_iota(kk, 30), setup=lambda: keys.clone())
ok = bool((sk[1:n] >= sk[:n - 1]).all()) and bool((keys[perm[:n].long()] == sk[:n]).all()) \
    and bool((torch.bincount(perm[:n].long(), minlength=n) == 1).all())
print(f"sort check: {'ok' if ok else 'WRONG'}", flush=True)
_, t_census = t(lambda: K.key_census(sk[:n], E.HEAVY_RUN))
pts, t_gather = t(lambda: K.gather3(p, perm, pad=K.PAD_POINTS))
_, t_build = t(lambda: E.build_index(p, box, grid=True))
print(f"n={n}: keys {t_keys:.2f} ms, sort {t_sort:.2f} ms, census {t_census:.2f} ms, gather {t_gather:.2f} ms, "
      f"whole build_index {t_build:.2f} ms", flush=True)
