"""``torch.distributed``-style facade over this package's communicator.

    import ddp_practice_amd.distributed as dist
    dist.init_process_group("nccl", init_method="env://")   # RCCL underneath
    dist.reduce(t, 0, op=dist.ReduceOp.SUM)
    work = dist.all_reduce(t, async_op=True); ...; work.wait()
    dist.destroy_process_group()

reference: /root/reference/ddp_main.py:69-73 (init_ddp), :108-109 (dist.reduce),
:170 (destroy_process_group).

Every collective of the native communicator is stream-ordered: it is enqueued on
the communicator's stream behind the caller's current stream and the caller's
stream waits for it (csrc/comm/rccl_comm.cpp ``fenced``).  ``async_op=True``
therefore returns a :class:`Work` whose ``wait()`` -- as torch's for NCCL work --
only orders the *current* stream after the collective (no host block);
``synchronize()`` / ``is_completed()`` observe it from the host.  Host-side
communicators (gloo on CPU) complete before returning.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as _tdist

from .parallel.comm import (agree_on_errors, barrier as _barrier, default_comm,  # noqa: F401
                            destroy_process_group, get_rank, get_world_size, init_process_group,
                            is_initialized, max_over_ranks)

ReduceOp = _tdist.ReduceOp


def is_available() -> bool:
    return _tdist.is_available()


def get_backend(group=None) -> str:
    c = group or default_comm()
    return {"RcclCommunicator": "nccl", "XgmiCommunicator": "xgmi", "HostCommunicator": "host",
            "TorchCommunicator": "gloo"}.get(type(c).__name__, "local")


class Work:
    """torch.distributed.Work for a stream-ordered collective (see the module docstring)."""

    def __init__(self, result, device: torch.device | None, comm=None):
        self._result = result
        self._comm = comm if comm is not None else default_comm()
        self._event = None
        if device is not None and device.type == "cuda" and torch.cuda.is_available():
            self._event = torch.cuda.Event()
            self._event.record(torch.cuda.current_stream(device))

    def wait(self, timeout=None) -> bool:
        """Order the current stream after the collective (already true: the collective was
        enqueued on it); a different current stream waits on the collective's event.  With a
        ``timeout`` (seconds or ``datetime.timedelta``), also block the host until the
        collective completes, raising ``RuntimeError`` when it has not after ``timeout`` or
        when the communicator reported an error (torch's blocking-wait behaviour)."""
        if self._event is not None:
            torch.cuda.current_stream().wait_event(self._event)
        if timeout is not None:
            secs = timeout.total_seconds() if hasattr(timeout, "total_seconds") else float(timeout)
            deadline = time.monotonic() + max(secs, 0.0)
            while not self.is_completed():
                exc = self.exception()
                if exc is not None:
                    raise exc
                if time.monotonic() >= deadline:
                    raise RuntimeError(f"collective work timed out after {secs:.3f} s")
                time.sleep(1e-4)
            exc = self.exception()
            if exc is not None:
                raise exc
        return True

    def is_completed(self) -> bool:
        return self._event is None or self._event.query()

    def _error(self) -> str:
        fn = getattr(self._comm, "async_error", None)
        err = fn() if fn is not None else ""
        return "" if (not err or err == "destroyed") else err

    def is_success(self) -> bool:
        return not self._error()

    def exception(self):
        """The communicator's asynchronous error as an exception (None when healthy)."""
        err = self._error()
        return RuntimeError(f"collective failed: {err}") if err else None

    def synchronize(self) -> None:
        if self._event is not None:
            self._event.synchronize()

    def result(self):
        return self._result

    def get_future(self):
        fut = torch.futures.Future()
        self.synchronize()
        fut.set_result(self._result)
        return fut


def _done(result, comm, async_op: bool):
    if not async_op:
        return None
    dev = getattr(comm, "device", None)
    return Work(result, dev, comm)


def all_reduce(tensor: torch.Tensor, op=ReduceOp.SUM, group=None, async_op: bool = False):
    c = group or default_comm()
    c.all_reduce_(tensor, op)
    return _done([tensor], c, async_op)


def reduce(tensor: torch.Tensor, dst: int, op=ReduceOp.SUM, group=None, async_op: bool = False):
    c = group or default_comm()
    c.reduce_(tensor, dst, op)
    return _done([tensor], c, async_op)


def broadcast(tensor: torch.Tensor, src: int, group=None, async_op: bool = False):
    c = group or default_comm()
    c.broadcast_(tensor, src)
    return _done([tensor], c, async_op)


def all_gather_into_tensor(output: torch.Tensor, input: torch.Tensor, group=None, async_op: bool = False):
    c = group or default_comm()
    c.all_gather_into_tensor(output, input)
    return _done([output], c, async_op)


def all_gather(tensor_list: list, tensor: torch.Tensor, group=None, async_op: bool = False):
    """List form: one gather into a flat buffer, then views copied out."""
    c = group or default_comm()
    flat = torch.empty((c.world_size,) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device)
    c.all_gather_into_tensor(flat, tensor.contiguous())
    for i, t in enumerate(tensor_list):
        t.copy_(flat[i])
    return _done(tensor_list, c, async_op)


def reduce_scatter_tensor(output: torch.Tensor, input: torch.Tensor, op=ReduceOp.SUM, group=None,
                          async_op: bool = False):
    c = group or default_comm()
    c.reduce_scatter_tensor(output, input, op)
    return _done([output], c, async_op)


def all_to_all_single(output: torch.Tensor, input: torch.Tensor, group=None, async_op: bool = False):
    c = group or default_comm()
    c.all_to_all_single(output, input)
    return _done([output], c, async_op)


def barrier(group=None, async_op: bool = False, device_ids=None):
    c = group or default_comm()
    c.barrier()
    return _done([], c, async_op)
