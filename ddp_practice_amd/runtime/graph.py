"""hipGraph capture of a whole training step (or K unrolled steps).

The ConvNet step is ~25 tiny kernels (tens of microseconds of GPU work), so
eager execution is bound by Python + launch overhead (~3.5 us host cost per
launch, MI355X_MICROARCH.md 'graph-replay-floor').  Every op on the native
path is capture-safe (no host syncs: GradScaler's found_inf, SyncBN counts
and the data position all stay on the device), so the step — data gather,
forward, loss, backward, DDP all-reduce, unscale/inf-check, SGD, scale
update — is captured once and replayed.  ``steps_per_graph`` unrolls K steps
into one graph to amortise the ~10-16 us replay floor.

This plays the role a tracing compiler would on other stacks; there is no
compiler here, just stream capture of the exact eager kernel sequence.
"""
from __future__ import annotations

import contextlib
import gc
import os
from typing import Callable

import torch


def _upload(g: "torch.cuda.CUDAGraph") -> None:
    """hipGraphUpload of a freshly captured graph: its first replay then runs as fast as the
    later ones (measured by bench.py's short timed region, which would otherwise hold every
    graph's first launch).  A no-op when the handle or the native runtime is unavailable."""
    if os.environ.get("DPA_NO_GRAPH_UPLOAD") == "1":  # A/B runs
        return
    try:
        exec_ = int(g.raw_cuda_graph_exec())
    except (AttributeError, RuntimeError, TypeError):
        return
    from .._ext import load as _load_ext

    _load_ext().runtime.graph_upload(exec_)
    torch.cuda.synchronize()


@contextlib.contextmanager
def gc_paused():
    """No automatic garbage collection while a stream is being captured.  A collection that
    runs inside the capture -- in any thread, the autograd engine's included -- and frees an
    unreachable earlier graph destroys its executable then, which HIP refuses during a
    capture (hipErrorStreamCaptureUnsupported from ~CUDAGraph: a terminate in the 8-rank
    shared-GPU rehearsal, profiles/r6d_rehearse8_gc_in_capture.txt).  Collected before,
    paused during, restored after."""
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


class CapturedStep:
    def __init__(self, fn: Callable[[], None], warmup: int = 3, steps_per_graph: int = 1, enabled: bool = True,
                 pre_capture: Callable[[], None] | None = None):
        self.fn = fn
        self.steps_per_graph = max(1, int(steps_per_graph))
        self.enabled = enabled and torch.cuda.is_available()
        self.graph: torch.cuda.CUDAGraph | None = None
        self.warmup = warmup
        self.pre_capture = pre_capture
        self.capture_error: Exception | None = None

    def capture(self) -> bool:
        """Warm up on a side stream, then capture. Returns False (eager fallback) on failure."""
        if not self.enabled:
            return False
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(self.warmup):
                self.fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.pre_capture is not None:
            self.pre_capture()
        g = torch.cuda.CUDAGraph()
        try:
            with gc_paused(), torch.cuda.graph(g):
                for _ in range(self.steps_per_graph):
                    self.fn()
        except Exception as e:  # pragma: no cover - depends on the device runtime
            self.capture_error = e
            self.graph = None
            torch.cuda.synchronize()
            return False
        self.graph = g
        _upload(g)
        return True

    def run(self) -> None:
        """Execute ``steps_per_graph`` steps (graph replay, or eagerly if not captured)."""
        if self.graph is not None:
            self.graph.replay()
        else:
            for _ in range(self.steps_per_graph):
                self.fn()
