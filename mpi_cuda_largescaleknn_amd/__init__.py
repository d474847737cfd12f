"""lsknn — MI355X-native large-scale k-NN distance engine.

Capabilities of ingowald/MPI-CUDA-LargeScaleKNN (both entrypoints, same CLI and file
formats), redesigned for AMD Instinct MI355X (gfx950): hand-written HIP kernels for the
Morton sort, bucket k-d tree and radix-select k-NN, RCCL (torch.distributed "nccl")
over xGMI for the spatial redistribution and halo exchange.
"""
__version__ = "0.1.0"

import os as _os

# Hardware queues per process (read by the HIP runtime when it is loaded, i.e. at
# `import torch`: import this package first, or set it in the environment — bench.py does).
# HIP's default of 4 is fewer than the streams a stream of point sets keeps busy (compute,
# copy, output, redistribution, halo, RCCL's): unrelated streams then share an in-order
# queue and wait for each other — the forced 1-rank RCCL 1e8 stream ran at 844.8 Mpts/s
# with 4 queues, 977.4 with 8, 973.5 with 16 (profiles/r4_s1/fd_q*.log). Filled in with
# LSKNN_HW_QUEUES (default 8; never above 32) only when unset: an explicit value is kept
# (a lower one with a one-line notice), a malformed one is ignored.
def _hw_queues() -> None:
    want = 8
    try:
        want = max(1, min(int(_os.environ.get("LSKNN_HW_QUEUES", "8")), 32))
    except ValueError:
        pass
    have = _os.environ.get("GPU_MAX_HW_QUEUES")
    if not have:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(want)
        return
    try:
        if int(have) < want:
            import sys as _sys
            _sys.stderr.write(f"lsknn: GPU_MAX_HW_QUEUES={have} kept (streams of point sets measured "
                              f"fastest with {want}; set LSKNN_HW_QUEUES or unset it)\n")
    except ValueError:
        pass


_hw_queues()

from .models.knn_engine import KnnConfig, build_index, knn_distances, query  # noqa: F401
