"""Optimizers (multi-tensor HIP kernels)."""
from .sgd import SGD  # noqa: F401
