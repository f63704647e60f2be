"""Environment-driven fault injection for failure-detection tests.

    DPA_FAULT="rank:step:kind[:arg][,rank:step:kind[:arg]...]"

``rank`` may be ``*``.  ``step`` counts optimizer steps from 0 over the run
(checked at step granularity by the training loop; graph-replayed chunks are
checked at their first step).  Kinds:

    exit[:code]    os._exit(code)          (a rank dies: peers must not hang)
    raise          RuntimeError            (Python exception path / spawn join)
    hang[:secs]    sleep (default forever)  (a rank stops entering collectives)
    slow:secs      sleep once               (straggler)
    inf            write +inf into a parameter gradient before the optimizer step
                   (GradScaler must skip the step and back off the scale)
    commerr        the communicator reports an asynchronous error from then on
                   (as after an xGMI exchange timeout): checkpoints must not be written

The reference has no fault injection.
"""
from __future__ import annotations

import os
import time

import torch

_KINDS = ("exit", "raise", "hang", "slow", "inf", "commerr")


class Fault:
    def __init__(self, rank, step: int, kind: str, arg: str | None):
        if kind not in _KINDS:
            raise ValueError(f"DPA_FAULT: unknown kind {kind!r} (one of {_KINDS})")
        self.rank, self.step, self.kind, self.arg = rank, step, kind, arg
        self.done = False

    def __repr__(self):
        return f"Fault(rank={self.rank}, step={self.step}, kind={self.kind}, arg={self.arg})"


def parse(spec: str) -> list[Fault]:
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        parts = item.split(":")
        if len(parts) < 3:
            raise ValueError(f"DPA_FAULT item {item!r}: expected rank:step:kind[:arg]")
        rank = None if parts[0] == "*" else int(parts[0])
        out.append(Fault(rank, int(parts[1]), parts[2], parts[3] if len(parts) > 3 else None))
    return out


class FaultInjector:
    def __init__(self, rank: int, spec: str | None = None, comm=None):
        spec = os.environ.get("DPA_FAULT", "") if spec is None else spec
        self.rank = rank
        self.comm = comm
        self.faults = [f for f in parse(spec) if f.rank is None or f.rank == rank]

    def __bool__(self):
        return bool(self.faults)

    def pending_in(self, lo: int, hi: int) -> bool:
        """Is a fault scheduled for a step in [lo, hi)?  (the loop then runs those steps one by one)"""
        return any(not f.done and lo <= f.step < hi for f in self.faults)

    def before_step(self, step: int) -> None:
        for f in self.faults:
            if f.done or f.step != step or f.kind == "inf":
                continue
            f.done = True
            print(f"[dpa fault] rank {self.rank} step {step}: injecting {f.kind}", flush=True)
            if f.kind == "exit":
                os._exit(int(f.arg) if f.arg else 13)
            if f.kind == "raise":
                raise RuntimeError(f"injected fault at step {step} on rank {self.rank}")
            if f.kind == "hang":
                secs = float(f.arg) if f.arg else float("inf")
                end = time.monotonic() + secs
                while time.monotonic() < end:
                    time.sleep(min(1.0, max(0.0, end - time.monotonic())))
            if f.kind == "slow":
                time.sleep(float(f.arg or 1.0))
            if f.kind == "commerr" and self.comm is not None:
                self.comm._injected_error = f"injected communicator error (rank {self.rank}, step {step})"

    def corrupt_grads(self, step: int, params) -> bool:
        """Called between backward and the optimizer step (eager steps only)."""
        for f in self.faults:
            if f.done or f.step != step or f.kind != "inf":
                continue
            f.done = True
            for p in params:
                if p.grad is not None:
                    with torch.no_grad():
                        p.grad.view(-1)[0] = float("inf")
                    print(f"[dpa fault] rank {self.rank} step {step}: +inf written into a gradient", flush=True)
                    return True
        return False
