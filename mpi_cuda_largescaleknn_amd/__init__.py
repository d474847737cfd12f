"""lsknn — MI355X-native large-scale k-NN distance engine.

Capabilities of ingowald/MPI-CUDA-LargeScaleKNN (both entrypoints, same CLI and file
formats), redesigned for AMD Instinct MI355X (gfx950): hand-written HIP kernels for the
Morton sort, bucket k-d tree and radix-select k-NN, RCCL (torch.distributed "nccl")
over xGMI for the spatial redistribution and halo exchange.
"""
__version__ = "0.1.0"

from .models.knn_engine import KnnConfig, build_index, knn_distances, query  # noqa: F401
