"""Process group + communicator.

``init_process_group`` keeps the reference's contract (backend "nccl" and
``init_method="env://"``: MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE, as set
by /root/reference/ddp_main.py:61-65,72-73 or by torchrun,
ddp_main_torchrun.py:102-104).  torch.distributed does the rendezvous (TCPStore)
so ``torch.distributed.get_rank()`` etc. keep working in user code; on a HIP
device this package then builds its OWN RCCL communicator (C++,
csrc/comm/rccl_comm.cpp) whose unique id travels through that store, and
every collective of the framework (DDP buckets, SyncBN statistics, buffer
broadcast, metric reduce, barrier) goes through it.  On CPU (tests, the
plumbing config) the same interface is served by torch.distributed/gloo.

Communicator interface (all tensor ops are stream-ordered and
hipGraph-capturable on the RCCL path):
    all_reduce_(t, op)            in place
    all_reduce(t, op) -> Tensor   out of place
    broadcast_(t, src), reduce_(t, dst, op), all_gather_into_tensor(out, inp),
    reduce_scatter_tensor(out, inp, op), all_to_all_single(out, inp), barrier()
"""
from __future__ import annotations

import datetime
import os
import time

import torch
import torch.distributed as dist

from .._ext import load as _load_ext

_DEFAULT = None
_GEN = 0

_TORCH_OPS = {
    "sum": dist.ReduceOp.SUM, "prod": dist.ReduceOp.PRODUCT, "max": dist.ReduceOp.MAX,
    "min": dist.ReduceOp.MIN,
}


def _op_name(op) -> str:
    if isinstance(op, str):
        return op.lower()
    for k, v in _TORCH_OPS.items():
        if op == v:
            return k
    if op == getattr(dist.ReduceOp, "AVG", object()):
        return "avg"
    raise ValueError(f"unsupported reduce op {op}")


class Communicator:
    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    # DPA_FORCE_COLLECTIVES=1 runs every collective code path even in a world of
    # one (single-GPU tests of the RCCL / reducer / SyncBN paths under capture)
    force_active: bool = os.environ.get("DPA_FORCE_COLLECTIVES", "0") == "1"

    @property
    def active(self) -> bool:
        """True when collectives must actually run (world > 1, or forced)."""
        return self.world_size > 1 or self.force_active

    # -- in-place / out-of-place all-reduce
    def all_reduce_(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        raise NotImplementedError

    def all_reduce(self, t: torch.Tensor, op="sum") -> torch.Tensor:
        out = t.clone()
        return self.all_reduce_(out, op)

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def reduce_(self, t: torch.Tensor, dst: int = 0, op="sum") -> torch.Tensor:
        raise NotImplementedError

    def all_gather_into_tensor(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def reduce_scatter_tensor(self, out: torch.Tensor, inp: torch.Tensor, op="sum") -> torch.Tensor:
        raise NotImplementedError

    def all_to_all_single(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    # failure detection: a non-empty string once a collective failed asynchronously
    # (RCCL async error, an xGMI exchange that timed out or was aborted)
    _injected_error: str = ""  # utils/fault.py "commerr" (tests)

    def async_error(self) -> str:
        return self._injected_error

    @property
    def native(self):
        """C++ Collective handle used by the DDP reducer."""
        return _load_ext().comm.PyCollective(self)

    def destroy(self) -> None:
        pass


class LocalCommunicator(Communicator):
    """World of one: every collective is the identity."""

    def __init__(self, device=None):
        self.rank, self.world_size = 0, 1
        self.device = torch.device(device) if device is not None else torch.device("cpu")

    def all_reduce_(self, t, op="sum"):
        return t

    def all_reduce(self, t, op="sum"):
        return t

    def broadcast_(self, t, src=0):
        return t

    def reduce_(self, t, dst=0, op="sum"):
        return t

    def all_gather_into_tensor(self, out, inp):
        out.view(-1).copy_(inp.view(-1))
        return out

    def reduce_scatter_tensor(self, out, inp, op="sum"):
        out.view(-1).copy_(inp.view(-1))
        return out

    def all_to_all_single(self, out, inp):
        out.copy_(inp)
        return out

    def barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


class TorchCommunicator(Communicator):
    """torch.distributed-backed communicator (gloo on CPU; any backend/group)."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.device = torch.device("cpu")

    def all_reduce_(self, t, op="sum"):
        name = _op_name(op)
        if name == "avg":
            dist.all_reduce(t, dist.ReduceOp.SUM, group=self.group)
            t.div_(self.world_size)
        else:
            dist.all_reduce(t, _TORCH_OPS[name], group=self.group)
        return t

    def broadcast_(self, t, src=0):
        dist.broadcast(t, src, group=self.group)
        return t

    def reduce_(self, t, dst=0, op="sum"):
        dist.reduce(t, dst, _TORCH_OPS[_op_name(op)], group=self.group)
        return t

    def all_gather_into_tensor(self, out, inp):
        chunks = list(out.view(self.world_size, -1).unbind(0))
        dist.all_gather(chunks, inp.reshape(-1).contiguous(), group=self.group)
        return out

    def reduce_scatter_tensor(self, out, inp, op="sum"):
        tmp = inp.clone()
        self.all_reduce_(tmp, op)
        out.view(-1).copy_(tmp.view(self.world_size, -1)[self.rank])
        return out

    def all_to_all_single(self, out, inp):
        ins = list(inp.view(self.world_size, -1).unbind(0))
        outs = [torch.empty_like(x) for x in ins]
        for r in range(self.world_size):
            dist.scatter(outs[r], ins if r == self.rank else None, src=r, group=self.group)
        out.view(self.world_size, -1).copy_(torch.stack(outs))
        return out

    def barrier(self):
        dist.barrier(group=self.group)


class HostCommunicator(TorchCommunicator):
    """Device tensors staged through host memory over the gloo process group.

    The last-resort fallback of the one-GPU rehearsal (``bench.py --share-gpu``, where RCCL
    refuses several ranks on one device and the xGMI engine is what failed): slow,
    synchronous and not capturable (run it with graphs off), but it shares no device
    memory or spin-waits with a peer, so it cannot stall on one."""

    def __init__(self, device, group=None):
        super().__init__(group)
        self.device = torch.device(device)
        self.xgmi_status = "off (host-staged gloo)"

    @staticmethod
    def _staged(t, fn):
        if t.device.type == "cpu":
            fn(t)
            return t
        h = t.detach().cpu()
        fn(h)
        t.copy_(h)
        return t

    def all_reduce_(self, t, op="sum"):
        return self._staged(t, lambda h: TorchCommunicator.all_reduce_(self, h, op))

    def broadcast_(self, t, src=0):
        return self._staged(t, lambda h: TorchCommunicator.broadcast_(self, h, src))

    def reduce_(self, t, dst=0, op="sum"):
        return self._staged(t, lambda h: TorchCommunicator.reduce_(self, h, dst, op))

    def all_gather_into_tensor(self, out, inp):
        h = torch.empty(out.shape, dtype=out.dtype)
        TorchCommunicator.all_gather_into_tensor(self, h, inp.detach().cpu())
        out.copy_(h)
        return out

    def reduce_scatter_tensor(self, out, inp, op="sum"):
        h = torch.empty(out.shape, dtype=out.dtype)
        TorchCommunicator.reduce_scatter_tensor(self, h, inp.detach().cpu(), op)
        out.copy_(h)
        return out

    def all_to_all_single(self, out, inp):
        h = torch.empty(out.shape, dtype=out.dtype)
        TorchCommunicator.all_to_all_single(self, h, inp.detach().cpu())
        out.copy_(h)
        return out

    def barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)


class RcclCommunicator(Communicator):
    """The native RCCL communicator (one per process / GPU)."""

    def __init__(self, rank: int, world_size: int, device: torch.device, store=None, key: str = "dpa_rccl"):
        C = _load_ext()
        self.rank, self.world_size = rank, world_size
        self.device = torch.device(device)
        if world_size > 1:
            if store is None:
                store = dist.distributed_c10d._get_default_store()
            if rank == 0:
                uid = C.comm.RcclComm.unique_id()
                store.set(key, uid)
            else:
                store.wait([key], datetime.timedelta(seconds=600))
                uid = store.get(key)
        else:
            uid = C.comm.RcclComm.unique_id()
        self._c = C.comm.RcclComm(bytes(uid), rank, world_size, self.device.index)
        self.xgmi = None
        self.xgmi_status = "off (world_size 1)" if world_size == 1 else "off"
        if world_size > 1 or self.force_active:
            self.xgmi_status = setup_xgmi(self, store, key)

    @property
    def native(self):
        return self._c

    def all_reduce_(self, t, op="sum"):
        self._c.all_reduce(t, _op_name(op))
        return t

    def all_reduce(self, t, op="sum"):
        out = torch.empty_like(t)
        self._c.all_reduce(t, _op_name(op), out)
        return out

    def broadcast_(self, t, src=0):
        self._c.broadcast(t, int(src))
        return t

    def reduce_(self, t, dst=0, op="sum"):
        self._c.reduce(t, int(dst), _op_name(op))
        return t

    def all_gather_into_tensor(self, out, inp):
        self._c.all_gather(out, inp.contiguous())
        return out

    def reduce_scatter_tensor(self, out, inp, op="sum"):
        self._c.reduce_scatter(out, inp.contiguous(), _op_name(op))
        return out

    def all_to_all_single(self, out, inp):
        self._c.all_to_all(out, inp.contiguous())
        return out

    def barrier(self):
        self._c.barrier()

    def async_error(self) -> str:
        return self._injected_error or self._c.async_error()

    @property
    def xgmi_max_bytes(self) -> int:
        return int(self._c.xgmi_max_bytes)

    def abort(self):
        self._c.abort()

    def destroy(self):
        if self.xgmi is not None:
            self._c.attach_xgmi(None, 0)
            self.xgmi.close()
            self.xgmi = None
        self._c.destroy()


XGMI_DEFAULT_MAX_BYTES = 1 << 20  # one-shot: every ConvNet collective (<= 116 KB)
XGMI_DEFAULT_TWOSHOT_MAX_BYTES = 32 << 20  # two-shot above it: a 25 MiB DDP bucket; RCCL above


class XgmiCommunicator(Communicator):
    """All-reduce-only communicator on the one-shot xGMI engine.

    Every all-reduce (DDP buckets through the C++ reducer, SyncBN statistics)
    runs on the engine; the rare host-side collectives (broadcast at DDP
    construction, metric reduce, barrier) go through the torch process group
    (gloo).  This is what lets several processes share ONE GPU in the test tier
    (RCCL refuses duplicate devices); on a node, ``RcclCommunicator`` attaches
    the same engine for its small all-reduces.
    """

    def __init__(self, rank: int, world_size: int, device: torch.device, store=None, key: str = "dpa_xgmi",
                 max_bytes: int = 4 << 20, group=None, twoshot_max_bytes: int = XGMI_DEFAULT_TWOSHOT_MAX_BYTES):
        C = _load_ext()
        self.rank, self.world_size = rank, world_size
        self.device = torch.device(device)
        self.group = group
        if store is None:
            store = dist.distributed_c10d._get_default_store()
        # ranks may share one GPU (the test tier): every rank's one-shot grid (one 256-lane
        # workgroup per 8 KB of message) must be resident at once -> <= ~1024 workgroups total
        max_bytes = min(int(max_bytes), max(1, 1024 // max(world_size, 1)) * 8192)
        x, err = open_xgmi(rank, world_size, self.device, store, key, max_bytes,
                           float(os.environ.get("DPA_XGMI_TIMEOUT", "600")), twoshot_max_bytes)
        if x is None:
            raise RuntimeError(f"xgmi communicator: {err}")
        if twoshot_max_bytes > 0:
            # ranks may share one GPU here: every rank's two-shot grid must be resident at once
            x.set_twoshot_blocks(max(8, 192 // max(world_size, 1)))
        self.xgmi_status = f"one-shot <= {max_bytes} B, two-shot <= {max(twoshot_max_bytes, 0)} B"
        self.xgmi = x
        self._c = C.xgmi.XgmiCollective(x)

    @property
    def native(self):
        return self._c

    def all_reduce_(self, t, op="sum"):
        self._c.all_reduce(t, _op_name(op))
        return t

    def all_reduce(self, t, op="sum"):
        out = torch.empty_like(t)
        self._c.all_reduce(t.contiguous(), _op_name(op), out)
        return out

    def _host(self, fn, t):
        h = t.detach().cpu()
        fn(h)
        t.copy_(h)
        return t

    def broadcast_(self, t, src=0):
        if t.is_cuda and torch.cuda.is_current_stream_capturing():
            # inside a captured step (DDP's per-step buffer broadcast without SyncBN): the
            # host path cannot run; broadcast through the engine instead
            return self._broadcast_engine(t, src)
        return self._host(lambda h: dist.broadcast(h, src, group=self.group), t)

    def _broadcast_engine(self, t, src):
        """Bit-exact broadcast as an all-reduce: the bytes as 16-bit pieces, each an fp32 integer
        in [0, 65536) (exact), zero on every rank but ``src``; any dtype, NaN payloads and
        signed zeros included.  Graph-capturable."""
        flat = t.detach().reshape(-1)
        if (flat.numel() * flat.element_size()) % 2 or not flat.is_contiguous():
            raise RuntimeError("xgmi broadcast under capture: needs a contiguous tensor of whole 16-bit pieces")
        pieces = flat.view(torch.int16)
        f = (pieces.to(torch.int32) & 0xFFFF).to(torch.float32)
        if self.rank != src:
            f.zero_()
        self.all_reduce_(f)
        pieces.copy_(f.to(torch.int32).to(torch.int16))  # 16-bit truncation: the same bits
        return t

    def reduce_(self, t, dst=0, op="sum"):
        return self._host(lambda h: dist.reduce(h, dst, _TORCH_OPS[_op_name(op)], group=self.group), t)

    def all_gather_into_tensor(self, out, inp):
        # flat on both sides: gloo wants the output to be the inputs concatenated on dim 0
        h = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.detach().reshape(-1).cpu().contiguous(), group=self.group)
        out.view(-1).copy_(h)
        return out

    def barrier(self):
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)

    def async_error(self) -> str:
        return self._injected_error or self.xgmi.error_string()

    def abort(self):
        self.xgmi.abort()

    def destroy(self):
        torch.cuda.synchronize(self.device)
        self.xgmi.close()


# ------------------------------------------------------------------ xGMI one-shot engine


def open_xgmi(rank: int, world: int, device: torch.device, store, key: str, max_bytes: int, timeout_s: float,
              twoshot_max_bytes: int = 0):
    """Create this rank's xGMI workspace and map every peer's (handles via the store).
    ``max_bytes``: largest one-shot message; ``twoshot_max_bytes``: largest two-shot one."""
    C = _load_ext()
    x, err = None, ""
    try:
        x = C.xgmi.XgmiComm(rank, world, device.index, int(max_bytes), float(timeout_s), int(twoshot_max_bytes))
        h = x.handle()
    except Exception as e:  # noqa: BLE001 - any failure here means "use RCCL"
        x, h, err = None, b"", f"{type(e).__name__}: {e}"
    store.set(f"{key}_xgmi_{rank}", h)
    hs = [bytes(store.get(f"{key}_xgmi_{r}")) for r in range(world)]
    if x is not None and all(len(v) > 0 for v in hs):
        try:
            x.open(hs)
        except Exception as e:  # noqa: BLE001
            x, err = None, f"{type(e).__name__}: {e}"
    elif x is not None:
        x, err = None, "a peer failed to create its workspace"
    return x, err


def comm_mode() -> str:
    """Collective algorithm selection (``--comm`` / ``DPA_COMM``): auto | rccl | xgmi.

    auto: the xGMI engine for the messages where it is validated and faster (one-shot up to
    ``DPA_XGMI_MAX_BYTES``, default 1 MiB), RCCL above; rccl: RCCL only (no engine, no
    in-kernel exchanges); xgmi: the engine wherever it can take the message.
    ``DPA_XGMI=0`` is the legacy spelling of rccl.
    """
    m = os.environ.get("DPA_COMM", "auto").lower()
    if os.environ.get("DPA_XGMI", "1") == "0":
        m = "rccl"
    if m not in ("auto", "rccl", "xgmi", "host"):
        raise ValueError(f"DPA_COMM must be auto, rccl, xgmi or host, got {m!r}")
    return m


def setup_xgmi(rc: "RcclCommunicator", store, key: str) -> str:
    """Attach the xGMI engine (csrc/comm/xgmi_allreduce.hip) to ``rc``.

    ``comm_mode()`` rccl disables it.  One-shot up to DPA_XGMI_MAX_BYTES (default
    1 MiB: every ConvNet collective); above that the two-shot (reduce-scatter +
    all-gather over direct peer writes) up to DPA_XGMI_TWOSHOT_MAX_BYTES (default
    32 MiB: a 25 MiB DDP bucket).  In auto mode the two-shot range is then trimmed by
    a timing probe against RCCL (DPA_XGMI_PROBE=0 skips it); ``--comm xgmi`` keeps
    the whole range.  Before attaching, every rank runs a self-test against RCCL
    (values within fp32 tolerance, results bit-identical across ranks, bounded by a
    short timeout); any failure on any rank keeps every rank on RCCL.  Every rank
    issues exactly the same collectives whatever happens locally (a rank-local failure
    only flips its vote), so a misbehaving engine can never desynchronise the RCCL
    call sequence.  Returns a status string.
    """
    mode = comm_mode()
    if mode in ("rccl", "host"):
        return f"off (--comm {mode})"
    if store is None:
        store = dist.distributed_c10d._get_default_store()
    max_bytes = int(float(os.environ.get("DPA_XGMI_MAX_BYTES", XGMI_DEFAULT_MAX_BYTES)))
    ts_max = int(float(os.environ.get("DPA_XGMI_TWOSHOT_MAX_BYTES", XGMI_DEFAULT_TWOSHOT_MAX_BYTES)))
    timeout = float(os.environ.get("DPA_XGMI_TIMEOUT", "600"))
    if max_bytes <= 0 or rc.world_size > 8:
        return "off"
    x, err = open_xgmi(rc.rank, rc.world_size, rc.device, store, key, max_bytes, 20.0, max(ts_max, 0))
    ok = torch.tensor([1.0 if x is not None else 0.0], device=rc.device)
    rc.native.all_reduce(ok, "min")
    if ok.item() != 1.0:
        return f"off (setup failed: {err or 'on a peer'})"
    good, err = _xgmi_selftest(rc, x, max(ts_max, 0))
    if not good:
        return f"off (self-test failed: {err or 'on a peer'})"
    if ts_max > 0 and mode == "auto" and os.environ.get("DPA_XGMI_PROBE", "1") != "0":
        ts_max = _probe_twoshot(rc, x, max_bytes, ts_max)
        if ts_max < 0:
            # an engine failure during the probe (exception or error word on any rank): the
            # engine may be poisoned, so it is not attached at all -- every rank stays on RCCL
            return "off (two-shot probe failed)"
    x.set_timeout(timeout)
    rc.native.attach_xgmi(x, max_bytes, max(ts_max, 0))
    rc.xgmi = x
    return f"on (one-shot <= {max_bytes} B, two-shot <= {max(ts_max, 0)} B)"


def _probe_twoshot(rc: "RcclCommunicator", x, lo: int, hi: int) -> int:
    """Largest probed size in (lo, hi] up to which the two-shot beats RCCL on this node
    (fp32, 5 timed repetitions after 2 warm-ups; each rank's times max-reduced so
    every rank picks the same bound).  Returns 0 if RCCL wins at the smallest size and
    -1 if the engine failed on any rank (the caller must then not attach it).

    Every decision is made from max-reduced values only: a rank whose engine failed
    (an exception, or its error word set) contributes a failure flag to the same
    reduction, so every rank leaves the probe at the same size with the same bound and
    the ranks' collective sequences stay identical."""
    sizes = [b for b in (2 << 20, 8 << 20, 32 << 20, 128 << 20) if lo < b <= hi] or [hi]
    best = 0
    for nb in sizes:
        t = torch.ones(nb // 4, device=rc.device)
        times = torch.zeros(3, device=rc.device)  # [two-shot s, RCCL s, any local failure]
        failed = False
        for i, fn in enumerate((lambda: x.all_reduce_twoshot(t), lambda: rc.native.all_reduce(t, "sum"))):
            barrier_done = False
            try:
                for _ in range(2):
                    fn()
                torch.cuda.synchronize(rc.device)
                rc.native.barrier()
                barrier_done = True
                t0 = time.perf_counter()
                for _ in range(5):
                    fn()
                torch.cuda.synchronize(rc.device)
                times[i] = time.perf_counter() - t0
            except Exception:  # noqa: BLE001 - only the engine may throw: recorded as this rank's failure
                if i == 1:
                    raise
                failed = True
                if not barrier_done:
                    rc.native.barrier()  # the barrier the skipped warm-up would have reached
        if failed or x.error() != 0:
            times[2] = 1.0
        rc.native.all_reduce(times, "max")
        ts, rccl, bad = times.tolist()
        if bad != 0.0:
            return -1
        if ts <= rccl:
            best = nb
        else:
            break
    return best


def _xgmi_selftest(rc: "RcclCommunicator", x, twoshot_max_bytes: int = 0) -> tuple[bool, str]:
    """Engine vs RCCL on a few sizes/dtypes/ops.  Per case, every rank issues the same
    RCCL collectives (reference all-reduce, cross-rank equality all-gather, vote); the
    vote is a min all-reduce so all ranks leave the loop together.

    ``twoshot_max_bytes`` > 0 adds two-shot cases sized inside that bound (the engine
    counts it as fp32 elements for every dtype), so a small DPA_XGMI_TWOSHOT_MAX_BYTES
    can never turn a valid setting into a failed vote (and the engine off)."""
    g = torch.Generator(device="cpu").manual_seed(1234 + rc.rank)
    why = ""
    vote = torch.ones(1, device=rc.device)
    cases = [(33, torch.float32, "sum", 1), (4099, torch.float32, "sum", 1), (29034, torch.float32, "sum", 1),
             (8195, torch.bfloat16, "sum", 1), (1000, torch.float32, "max", 1)]
    ts_elems = int(twoshot_max_bytes) // 4
    if ts_elems > 0:
        # a whole-chunk fp32 size and an odd (ragged-tail) bf16 size, both within the bound
        cases += [(min(1 << 20, ts_elems), torch.float32, "sum", 2),
                  (max(1, min(700001, ts_elems - 1)), torch.bfloat16, "sum", 2)]
    for n, dt, op, how in cases:
        t = torch.randn(n, generator=g).to(device=rc.device, dtype=dt)
        mine = torch.zeros_like(t)
        good = True
        try:
            if how == 1:
                x.all_reduce(t, op, mine)
            else:
                x.all_reduce_twoshot(t, op, mine)
        except Exception as e:  # noqa: BLE001 - recorded as this rank's vote
            good, why = False, f"{type(e).__name__}: {e}"
        ref = torch.empty_like(t)
        rc.native.all_reduce(t, op, ref)
        every = torch.empty(rc.world_size * n, dtype=dt, device=rc.device)
        rc.native.all_gather(every, mine)
        torch.cuda.synchronize(rc.device)
        if x.error() != 0:
            good, why = False, why or x.error_string()
        tol = 1e-5 if dt == torch.float32 else 2e-2
        if good and not torch.allclose(mine.float(), ref.float(), rtol=tol, atol=tol * rc.world_size):
            good, why = False, f"mismatch vs RCCL (n={n}, {dt}, {op})"
        every = every.view(rc.world_size, n)
        if good and not bool((every == every[0:1]).all()):
            good, why = False, f"ranks disagree (n={n}, {dt}, {op})"
        vote.fill_(1.0 if good else 0.0)
        rc.native.all_reduce(vote, "min")
        if vote.item() != 1.0:
            return False, why
    # the in-kernel exchange sites (fused SyncBN consumers, the fused AMP-SGD gradient
    # average: csrc/comm/xsite.h) -- the same peer-write protocol run from inside a
    # multi-workgroup launch; every workgroup must see the rank-ordered sum
    # sizes within a SyncBN site's row (csrc/comm/xsite.h kSiteVals = 128 floats; the ConvNet's
    # rows are 2C+1 = 33 / 65 forward and 2C = 32 / 64 backward): a larger n is rejected by
    # site_probe, which would fail the vote and turn the engine off on every multi-GPU run
    for it, n in enumerate((33, 65, 128)):
        t = torch.randn(n, generator=g).to(device=rc.device)
        o = torch.empty(4 * n, device=rc.device)
        good = True
        try:
            x.site_probe(it % 2, t, o, 4)
        except Exception as e:  # noqa: BLE001 - recorded as this rank's vote
            good, why = False, f"{type(e).__name__}: {e}"
        ref = torch.empty_like(t)
        rc.native.all_reduce(t, "sum", ref)
        every = torch.empty(rc.world_size * 4 * n, device=rc.device)
        rc.native.all_gather(every, o)
        torch.cuda.synchronize(rc.device)
        if x.error() != 0:
            good, why = False, why or x.error_string()
        if good and not all(torch.allclose(o[b * n:(b + 1) * n], ref, rtol=1e-5, atol=1e-5 * rc.world_size)
                            for b in range(4)):
            good, why = False, f"site mismatch vs RCCL (n={n})"
        every = every.view(rc.world_size, 4 * n)
        if good and not bool((every == every[0:1]).all()):
            good, why = False, f"site: ranks disagree (n={n})"
        vote.fill_(1.0 if good else 0.0)
        rc.native.all_reduce(vote, "min")
        if vote.item() != 1.0:
            return False, why
    return True, ""


# ------------------------------------------------------------------ process group
def init_process_group(backend: str | None = None, init_method: str | None = "env://", world_size: int = -1,
                       rank: int = -1, timeout: datetime.timedelta | None = None, device=None):
    """Rendezvous (torch TCPStore, env://) + this package's communicator.

    ``backend``: "nccl"/"rccl" (GPU; the framework's collectives use the native
    RCCL communicator) or "gloo" (CPU).  Default: "nccl" if a GPU is present.
    Rehearsal backends for ranks sharing one GPU: "xgmi" (all-reduces on the xGMI
    engine, host collectives on gloo) and "host" (everything staged through gloo).
    """
    global _DEFAULT, _GEN
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    backend = backend.lower()
    torch_backend = "nccl" if backend in ("nccl", "rccl") else "gloo" if backend in ("xgmi", "host") else backend
    kw = {}
    if timeout is not None:
        kw["timeout"] = timeout
    if not dist.is_initialized():
        dist.init_process_group(torch_backend, init_method=init_method, world_size=world_size, rank=rank, **kw)
    r, w = dist.get_rank(), dist.get_world_size()
    if torch_backend == "gloo" and w > 1 and "OMP_NUM_THREADS" not in os.environ:
        # several CPU ranks on one host: do not oversubscribe the cores (torchrun's default too)
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // w))
    if backend == "xgmi":  # all-reduces on the xGMI engine, host collectives on gloo (see XgmiCommunicator)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        _GEN += 1
        _DEFAULT = XgmiCommunicator(r, w, device, key=f"dpa_xgmi_{_GEN}")
    elif backend == "host":
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        _DEFAULT = HostCommunicator(device)
    elif torch_backend == "nccl" and w == 1 and not Communicator.force_active:
        # a world of one has no collective to run: skip the RCCL communicator bring-up
        # (1.15 s of a 3-epoch ddp_main run at W=1, plus 0.3 s of teardown)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        _DEFAULT = LocalCommunicator(device)
    elif torch_backend == "nccl":
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        _GEN += 1
        _DEFAULT = RcclCommunicator(r, w, device, key=f"dpa_rccl_uid_{_GEN}")
    else:
        _DEFAULT = TorchCommunicator() if w > 1 else LocalCommunicator()
    if os.environ.get("DPA_DEBUG_COLLECTIVES", "0") == "1":
        from ..utils.debug import CheckedCommunicator

        _DEFAULT = CheckedCommunicator(_DEFAULT)
    return _DEFAULT


def is_initialized() -> bool:
    return _DEFAULT is not None or dist.is_initialized()


def default_comm() -> Communicator:
    global _DEFAULT
    if _DEFAULT is None:
        if dist.is_initialized():
            _DEFAULT = TorchCommunicator() if dist.get_world_size() > 1 else LocalCommunicator()
        else:
            dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
            _DEFAULT = LocalCommunicator(dev)
    return _DEFAULT


def set_default_comm(c: Communicator | None) -> None:
    global _DEFAULT
    _DEFAULT = c


def get_rank() -> int:
    if _DEFAULT is not None:
        return _DEFAULT.rank
    return dist.get_rank() if dist.is_initialized() else int(os.environ.get("RANK", "0"))


def get_world_size() -> int:
    if _DEFAULT is not None:
        return _DEFAULT.world_size
    return dist.get_world_size() if dist.is_initialized() else int(os.environ.get("WORLD_SIZE", "1"))


def barrier() -> None:
    if _DEFAULT is not None:
        _DEFAULT.barrier()
    elif dist.is_initialized():
        dist.barrier()


_HEALTH_SEQ = 0


def agree_on_errors(comm: Communicator | None = None, timeout_s: float = 600.0) -> str:
    """Every rank's communicator error word, gathered through the rendezvous store.

    Not through the communicator: it may be the broken part (an xGMI exchange that
    timed out leaves RCCL healthy but the engine poisoned; a dead peer leaves every
    collective hanging).  Every rank must call it at the same point (a collective in
    that sense); all of them return the same string: "" when every rank is healthy,
    else ``"rank r: <error>; ..."``.  Used before checkpointing and after every epoch,
    so no rank saves or reports a model trained through skipped updates.
    """
    global _HEALTH_SEQ
    comm = comm if comm is not None else _DEFAULT
    local = ""
    if comm is not None:
        if comm.device.type == "cuda":
            torch.cuda.synchronize(comm.device)  # the error word covers everything issued so far
        local = comm.async_error() or ""
        if local == "destroyed":
            local = ""
    world = comm.world_size if comm is not None else 1
    if world == 1 or not dist.is_initialized():
        return f"rank 0: {local}" if local else ""
    _HEALTH_SEQ += 1
    store = dist.distributed_c10d._get_default_store()
    key = f"dpa_health/{_GEN}/{_HEALTH_SEQ}"
    store.set(f"{key}/{comm.rank}", local)
    keys = [f"{key}/{r}" for r in range(world)]
    store.wait(keys, datetime.timedelta(seconds=timeout_s))
    errs = [(r, store.get(k).decode()) for r, k in enumerate(keys)]
    return "; ".join(f"rank {r}: {e}" for r, e in errs if e)


def max_over_ranks(x: float) -> float:
    c = _DEFAULT
    if c is None or c.world_size == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float32, device=c.device)
    c.all_reduce_(t, "max")
    return float(t.item())


def destroy_process_group() -> None:
    global _DEFAULT
    if _DEFAULT is not None:
        try:
            if _DEFAULT.device.type == "cuda":
                torch.cuda.synchronize(_DEFAULT.device)
            _DEFAULT.destroy()
        finally:
            _DEFAULT = None
    if dist.is_initialized():
        dist.destroy_process_group()
