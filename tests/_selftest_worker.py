"""Worker for tests/test_comm_cpu_selftest.py: the xGMI start-up self-test
(parallel/comm._xgmi_selftest) driven over gloo with a torch stand-in for the
engine, so its vote / collective symmetry runs on CPU."""
import os
import traceback

import torch
import torch.distributed as dist

from tests._dist import client_env


class _Native:
    """The RcclCommunicator.native calls the self-test makes, on gloo."""

    def __init__(self):
        self.calls = 0

    def all_reduce(self, t, op, out=None):
        self.calls += 1
        r = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if out is None:
            dist.all_reduce(t, op=r)
            return t
        out.copy_(t)
        dist.all_reduce(out, op=r)
        return out

    def barrier(self):
        self.calls += 1
        dist.barrier()

    def all_gather(self, out, t):
        self.calls += 1
        parts = list(out.view(dist.get_world_size(), -1).unbind(0))
        dist.all_gather(parts, t.contiguous())
        return out


class _RC:
    def __init__(self, rank, world):
        self.rank, self.world_size, self.device = rank, world, torch.device("cpu")
        self.native = _Native()


class _Engine:
    """Correct collectives, except on rank `bad` for the case kind `bad_kind`."""

    def __init__(self, rank, bad, bad_kind):
        self.rank, self.bad, self.bad_kind = rank, bad, bad_kind

    def _sum(self, t, op):
        o = t.clone()
        dist.all_reduce(o, op={"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX}[op])
        return o

    def all_reduce(self, t, op, out):
        out.copy_(self._sum(t, op))
        if self.rank == self.bad and self.bad_kind == "oneshot":
            out.add_(1.0)

    def all_reduce_twoshot(self, t, op="sum", out=None):
        if self.rank == self.bad and self.bad_kind == "twoshot_err":
            self.err = 1  # a timed-out exchange: the engine's error word, no exception
        if self.rank == self.bad and self.bad_kind == "twoshot_raise":
            raise RuntimeError("two-shot launch failed on this rank")
        self.ts_calls += 1
        if self.rank == self.bad and self.bad_kind == "twoshot_raise_late" and self.ts_calls > 2:
            # fails inside the timed loop, i.e. after the probe's barrier
            raise RuntimeError("two-shot launch failed on this rank (timed loop)")
        # the probe only times the engine: no stand-in gloo traffic that a failing rank
        # would leave unmatched (the real engine's peers time out instead)
        r = t.clone() if self.local_only else self._sum(t, op)
        (t if out is None else out).copy_(r)

    def site_probe(self, site, t, o, nblk):
        # the real engine's limits (csrc/comm/xgmi_allreduce.hip site_probe): a SyncBN site id
        # and at most kSiteVals = 128 floats -- checked AFTER the stand-in's gloo traffic so a
        # violation fails this rank's vote instead of desynchronising the stand-in
        s = self._sum(t, "sum")
        if t.numel() > 128 or not 0 <= site < 7:
            raise RuntimeError("site_probe: <= 128 contiguous f32 values")
        if self.rank == self.bad and self.bad_kind == "site":
            raise RuntimeError("site probe failed on this rank")
        o.copy_(s.repeat(nblk))

    err = 0
    ts_calls = 0
    local_only = False
    attached = False

    def set_timeout(self, s):
        pass

    def error(self):
        return self.err

    def error_string(self):
        return ""


def run(rank, world, port, bad, bad_kind, *rest):
    q = rest[-1]
    ts_max = rest[0] if len(rest) > 1 else 32 << 20  # optional two-shot bound (bytes)
    try:
        os.environ.update(client_env(rank, world, port))
        dist.init_process_group("gloo")
        torch.cuda.synchronize = lambda *a, **k: None  # CPU stand-in: nothing to wait for
        from ddp_practice_amd.parallel.comm import _xgmi_selftest

        rc = _RC(rank, world)
        good, why = _xgmi_selftest(rc, _Engine(rank, bad, bad_kind), twoshot_max_bytes=ts_max)
        # every rank issued the same number of collectives: the call sequences stayed matched
        calls = torch.tensor([rc.native.calls])
        every = [torch.zeros(1, dtype=calls.dtype) for _ in range(world)]
        dist.all_gather(every, calls)
        dist.destroy_process_group()
        q.put((rank, "ok", (good, why, [int(c) for c in every])))
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))


def run_probe(rank, world, port, bad, bad_kind, q):
    """parallel/comm._probe_twoshot with a stand-in engine failing on rank ``bad``."""
    try:
        os.environ.update(client_env(rank, world, port))
        dist.init_process_group("gloo")
        torch.cuda.synchronize = lambda *a, **k: None
        from ddp_practice_amd.parallel.comm import _probe_twoshot

        rc = _RC(rank, world)
        eng = _Engine(rank, bad, bad_kind)
        eng.local_only = True
        best = _probe_twoshot(rc, eng, 1 << 20, 8 << 20)
        calls = torch.tensor([rc.native.calls])
        every = [torch.zeros(1, dtype=calls.dtype) for _ in range(world)]
        dist.all_gather(every, calls)
        dist.destroy_process_group()
        q.put((rank, "ok", (best, [int(c) for c in every])))
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))


def run_setup(rank, world, port, bad, bad_kind, q):
    """parallel/comm.setup_xgmi with a stand-in engine whose two-shot probe fails on rank
    ``bad``: every rank must report the engine off and none may attach it."""
    try:
        os.environ.update(client_env(rank, world, port))
        os.environ["DPA_COMM"] = "auto"
        dist.init_process_group("gloo")
        torch.cuda.synchronize = lambda *a, **k: None
        from ddp_practice_amd.parallel import comm

        rc = _RC(rank, world)
        eng = _Engine(rank, bad, bad_kind)
        eng.local_only = True
        rc.native.attach_xgmi = lambda *a: setattr(eng, "attached", True)
        comm.open_xgmi = lambda *a, **k: (eng, "")
        comm._xgmi_selftest = lambda *a, **k: (True, "")
        status = comm.setup_xgmi(rc, store=object(), key="t")
        calls = torch.tensor([rc.native.calls])
        every = [torch.zeros(1, dtype=calls.dtype) for _ in range(world)]
        dist.all_gather(every, calls)
        dist.destroy_process_group()
        q.put((rank, "ok", (status, eng.attached, getattr(rc, "xgmi", None) is not None, [int(c) for c in every])))
    except Exception:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
