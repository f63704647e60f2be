"""Collective-mismatch detection (``DPA_DEBUG_COLLECTIVES=1``).

The reference's only deadlock guidance is prose, and one piece of it is wrong
(README.md:425 says to call ``test()`` on rank 0 only, which deadlocks on the
``dist.reduce`` at /root/reference/ddp_main.py:108-109).  With
this wrapper every collective first all-gathers a fingerprint
``(sequence number, op, dtype, numel, root)`` through the same communicator;
if the ranks disagree the call raises a ``CollectiveMismatch`` naming what
each rank was about to do, instead of hanging or silently reducing mismatched
buffers.  (A rank that never calls any collective still blocks the fingerprint
exchange: that case is the watchdog's, utils/watchdog.py.)

Fingerprints are skipped while a HIP graph is being captured (the comparison
needs the host) — captured steps were checked during their eager warm-up.
"""
from __future__ import annotations

import torch

from ..parallel.comm import Communicator

_OPS = ["all_reduce", "broadcast", "reduce", "all_gather", "reduce_scatter", "all_to_all", "barrier"]
_RED = ["sum", "prod", "max", "min", "avg", "-"]
_DT = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.uint8,
       torch.int8]


class CollectiveMismatch(RuntimeError):
    pass


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


class CheckedCommunicator(Communicator):
    def __init__(self, inner: Communicator):
        self.inner = inner
        self.rank, self.world_size, self.device = inner.rank, inner.world_size, inner.device
        self.seq = 0
        self.history: list[tuple] = []

    @property
    def active(self) -> bool:
        return self.inner.active

    @property
    def native(self):
        from ..parallel.comm import RcclCommunicator

        if isinstance(self.inner, RcclCommunicator):
            return self.inner.native  # bucket all-reduces are issued from C++ (fingerprinted via history only)
        return Communicator.native.fget(self)

    def __getattr__(self, name):
        return getattr(self.__dict__["inner"], name)

    def async_error(self) -> str:
        return self._injected_error or self.inner.async_error()

    def _check(self, op: str, t: torch.Tensor | None, red: str = "-", root: int = -1) -> None:
        if _capturing():
            return
        from ..parallel.comm import _op_name

        red = _op_name(red) if red != "-" else "-"
        dt = _DT.index(t.dtype) if t is not None and t.dtype in _DT else -1
        fp = [self.seq, _OPS.index(op), _RED.index(red), dt, -1 if t is None else t.numel(), root]
        self.seq += 1
        self.history.append(tuple(fp))
        if self.world_size == 1:
            return
        mine = torch.tensor(fp, dtype=torch.int64, device=self.device)
        allfp = torch.empty(self.world_size * len(fp), dtype=torch.int64, device=self.device)
        self.inner.all_gather_into_tensor(allfp, mine)
        rows = allfp.view(self.world_size, -1).tolist()
        if any(r != rows[0] for r in rows):
            raise CollectiveMismatch("collective mismatch across ranks:\n" + "\n".join(
                f"  rank {i}: {self._describe(r)}" for i, r in enumerate(rows)))

    @staticmethod
    def _describe(r) -> str:
        seq, op, red, dt, n, root = r
        d = str(_DT[dt]).replace("torch.", "") if 0 <= dt < len(_DT) else "?"
        s = f"#{seq} {_OPS[op]}({d}[{n}]"
        if _RED[red] != "-":
            s += f", op={_RED[red]}"
        if root >= 0:
            s += f", root={root}"
        return s + ")"

    # -- collectives
    def all_reduce_(self, t, op="sum"):
        self._check("all_reduce", t, op)
        return self.inner.all_reduce_(t, op)

    def all_reduce(self, t, op="sum"):
        self._check("all_reduce", t, op)
        return self.inner.all_reduce(t, op)

    def broadcast_(self, t, src=0):
        self._check("broadcast", t, root=src)
        return self.inner.broadcast_(t, src)

    def reduce_(self, t, dst=0, op="sum"):
        self._check("reduce", t, op, root=dst)
        return self.inner.reduce_(t, dst, op)

    def all_gather_into_tensor(self, out, inp):
        self._check("all_gather", inp)
        return self.inner.all_gather_into_tensor(out, inp)

    def reduce_scatter_tensor(self, out, inp, op="sum"):
        self._check("reduce_scatter", inp, op)
        return self.inner.reduce_scatter_tensor(out, inp, op)

    def all_to_all_single(self, out, inp):
        self._check("all_to_all", inp)
        return self.inner.all_to_all_single(out, inp)

    def barrier(self):
        self._check("barrier", None)
        return self.inner.barrier()

    def destroy(self):
        self.inner.destroy()
