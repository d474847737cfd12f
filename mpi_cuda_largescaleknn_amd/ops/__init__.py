"""Tensor-level wrappers of the gfx950 kernels (csrc/hip) and CPU counterparts."""
from . import kernels  # noqa: F401
