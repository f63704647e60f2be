"""Precision policy ("autocast") for the native ops.

Torch's autocast is a dispatcher-level per-op cast table; here the policy is
explicit: every native op asks :func:`compute_dtype` for the dtype its
activations are stored and multiplied in.  Weights stay fp32 masters and are
cast inside the kernels (the LDS/register staging does the fp32 -> bf16/fp16
conversion, so there is no separate cast launch as with torch's autocast
weight cache).  Normalisation statistics, softmax / loss and all reductions
accumulate in fp32, matching torch's CUDA autocast policy for
conv2d/linear (low precision) vs. softmax/nll (fp32)
(torch/testing/_internal/autocast_test_lists.py:94,146-147,210-214).

The context manager also enters ``torch.autocast`` for the same device type so
that any non-native op in a user model sees the same policy.

reference: /root/reference/ddp_main.py:31 — ``torch.cuda.amp.autocast()``
(fp16).  The reference default dtype is float16; this framework accepts
float16 or bfloat16 (bf16 is the default for the benchmark: same speed on
MFMA, no overflow-driven step skipping).
"""
from __future__ import annotations

import contextlib
import threading

import torch

_state = threading.local()


def _stack():
    s = getattr(_state, "stack", None)
    if s is None:
        s = _state.stack = []
    return s


def is_enabled() -> bool:
    s = _stack()
    return bool(s) and s[-1] is not None


def current_dtype():
    s = _stack()
    return s[-1] if s else None


def compute_dtype(t: torch.Tensor | None = None) -> torch.dtype:
    """dtype a native op should compute/store activations in."""
    d = current_dtype()
    if d is not None:
        return d
    if t is not None and t.dtype in (torch.float32, torch.bfloat16, torch.float16):
        return t.dtype
    return torch.float32


@contextlib.contextmanager
def autocast(enabled: bool = True, dtype: torch.dtype = torch.bfloat16, device_type: str | None = None):
    """Enable the low-precision policy (``dtype`` in {bfloat16, float16})."""
    if enabled and dtype not in (torch.bfloat16, torch.float16):
        raise ValueError(f"autocast dtype must be bfloat16 or float16, got {dtype}")
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    cpu_ok = device_type != "cpu" or dtype == torch.bfloat16
    s = _stack()
    s.append(dtype if enabled else None)
    try:
        if cpu_ok:
            with torch.autocast(device_type, dtype=dtype, enabled=enabled):
                yield
        else:
            yield
    finally:
        s.pop()
