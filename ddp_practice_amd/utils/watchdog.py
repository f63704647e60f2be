"""Python face of the native watchdog (csrc/runtime/watchdog.cpp).

The reference's only failure detection is ProcessGroupNCCL's watchdog
(10 min default, torch/distributed/constants.py:21) plus the launcher's
teardown (/root/reference/ddp_main.py:176 mp.spawn; torchrun).  Here:

    wd = Watchdog(comm, timeout=600)    # DPA_WATCHDOG_TIMEOUT overrides
    ...
    wd.tick()        # after each (graph-replayed) chunk of steps: device progress marker
    wd.heartbeat()   # host progress (CPU / gloo ranks)
    wd.stop()

If a marker is not reached within ``timeout`` seconds the watchdog prints the
reason, aborts the communicator (RCCL kernels spinning on a dead peer return,
leaving the GPU usable) and exits the process with ``exit_code`` so that the
launcher tears the remaining ranks down.
"""
from __future__ import annotations

import os

import torch

from .._ext import load as _load_ext


def default_timeout() -> float:
    return float(os.environ.get("DPA_WATCHDOG_TIMEOUT", "600"))


class Watchdog:
    def __init__(self, comm=None, timeout: float | None = None, exit_code: int = 124, tag: str = "train",
                 poll: float | None = None, exit_on_fire: bool = True):
        C = _load_ext()
        self.timeout = default_timeout() if timeout is None else float(timeout)
        native = None
        if comm is not None and getattr(comm, "active", False):
            native = comm.native
        poll = poll if poll is not None else min(0.5, max(0.01, self.timeout / 10))
        self._w = C.runtime.Watchdog(self.timeout, native, int(exit_code), tag, float(poll))
        self._w.set_exit(bool(exit_on_fire))
        self._device = getattr(comm, "device", torch.device("cpu")) if comm is not None else None

    def tick(self) -> None:
        """Device progress marker on the current stream (no-op on CPU and under capture)."""
        if self._device is not None and self._device.type == "cuda":
            self._w.tick()
        else:
            self._w.heartbeat()

    def heartbeat(self) -> None:
        self._w.heartbeat()

    def note(self, what: str) -> None:
        """What the rank last queued (named in a fire report with the communicator's
        in-kernel exchange state: csrc/comm/xgmi_allreduce.hip debug_state)."""
        self._w.note(what)

    def disarm(self) -> None:
        self._w.disarm()

    @property
    def fired(self) -> bool:
        return self._w.fired

    @property
    def reason(self) -> str:
        return self._w.reason

    def stop(self) -> None:
        self._w.stop()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
        return False
