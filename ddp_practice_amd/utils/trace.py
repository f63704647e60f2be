"""roctx ranges around the phases of a run (data / fwd / bwd / comm / step /
eval / checkpoint).  Visible on the timeline of
``rocprofv3 --marker-trace --kernel-trace -- python ...``.  The reference has
no tracing at all (only a wall-clock ``time.time()``).

Enabled by ``DPA_TRACE=1`` or ``set_tracing(True)`` (the CLIs' ``--profile``);
when disabled a range costs one attribute check.
"""
from __future__ import annotations

import contextlib
import os

_ENABLED = os.environ.get("DPA_TRACE", "0") == "1"
_RT = None


def set_tracing(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def tracing_enabled() -> bool:
    return _ENABLED


def _rt():
    global _RT
    if _RT is None:
        from .._ext import load

        _RT = load().runtime
    return _RT


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    rt = _rt()
    rt.range_push(name)
    try:
        yield
    finally:
        rt.range_pop()


def mark(name: str) -> None:
    if _ENABLED:
        _rt().mark(name)
