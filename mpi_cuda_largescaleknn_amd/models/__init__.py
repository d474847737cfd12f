"""The k-th-NN distance "model": single-rank engine (bounds, sort, tree, select)."""
from .knn_engine import KnnConfig, LocalIndex, build_index, knn_distances, query  # noqa: F401
