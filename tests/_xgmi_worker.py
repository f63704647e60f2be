"""Worker for tests/test_xgmi_gpu.py: W processes sharing ONE GPU run the
one-shot xGMI all-reduce against each other (IPC-mapped workspaces on the same
device exercise the whole protocol: peer stores, flags, epochs, parity reuse,
graph replay, bounded waits)."""
import os
import traceback
from datetime import timedelta

import torch
import torch.distributed  # noqa: F401  (TCPStore)

DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16}


def _data(rank, n, dt, it):
    g = torch.Generator(device="cpu").manual_seed(1000 * it + 17 * rank + n)
    return torch.randn(n, generator=g).to(dt)


def _expect(world, n, dt, it, op):
    xs = [_data(r, n, dt, it).float() for r in range(world)]
    acc = xs[0].clone()
    for x in xs[1:]:
        acc = torch.maximum(acc, x) if op == "max" else torch.minimum(acc, x) if op == "min" else acc + x
    if op == "avg":
        acc = acc / world
    return acc


def _check(got, exp, dt, what):
    tol = {torch.float32: 1e-5, torch.bfloat16: 1e-2, torch.float16: 2e-3}[dt]
    got = got.float().cpu()
    assert got.shape == exp.shape, what
    err = ((got - exp).abs() / (exp.abs() + 1.0)).max().item()
    assert err <= tol, (what, err)


def worker(rank, world, port, mode, q):
    try:
        if world >= 3:  # several ranks on one card: one HW queue each (runtime/device.shared_gpu_env)
            os.environ["GPU_MAX_HW_QUEUES"] = "1"
        from ddp_practice_amd import _ext

        C = _ext.load()
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        store = torch.distributed.TCPStore("127.0.0.1", port, world, False, timedelta(seconds=60))  # parent serves
        from ddp_practice_amd.parallel.comm import open_xgmi

        x, err = open_xgmi(rank, world, dev, store, "t", 1 << 20, 20.0, (32 << 20) if mode == "twoshot" else 0)
        assert x is not None, err
        store.set(f"ready{rank}", "1")
        store.wait([f"ready{r}" for r in range(world)])
        if mode == "site":
            # in-kernel SyncBN exchange: 4 workgroups per launch, 30 launches through two
            # sites (epochs, parity reuse), eager and graph-replayed; rank-ordered sums
            out = {}
            for it in range(30):
                n = 1 + (it * 37) % 128
                t = _data(rank, n, torch.float32, it).to(dev)
                o = torch.empty(4 * n, device=dev)
                x.site_probe(it % 2, t, o, 4)
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                exp = _expect(world, n, torch.float32, it, "sum")
                for b in range(4):
                    _check(o[b * n:(b + 1) * n], exp, torch.float32, ("site", it, b))
                out[f"site{it}"] = o.cpu().numpy().tobytes()
            t = torch.zeros(64, device=dev)
            o = torch.empty(2 * 64, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                x.site_probe(3, t, o, 2)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                x.site_probe(3, t, o, 2)
            for r in range(10):
                t.copy_(_data(rank, 64, torch.float32, 100 + r).to(dev))
                g.replay()
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                exp = _expect(world, 64, torch.float32, 100 + r, "sum")
                _check(o[:64], exp, torch.float32, ("site graph", r))
                _check(o[64:], exp, torch.float32, ("site graph", r))
            store.set(f"done{rank}", "1")
            store.wait([f"done{r}" for r in range(world)])
            x.close()
            q.put((rank, "ok", out))
            return
        if mode == "wide":
            # the ResNet statistics finishers' positioned exchange (csrc/comm/xsite.h, wide
            # site): rows up to 2*2048+1 floats split over 1..64 finisher workgroups, the
            # finisher count changing launch to launch (ticket lanes, idle-lane bumps), then
            # graph-replayed; rank-ordered sums bit-identical on every rank
            out = {}
            cases = [(4097, 16), (4097, 1), (129, 3), (2049, 64), (1, 1), (513, 8), (4097, 9), (300, 7)]
            for it in range(24):
                n, nb = cases[it % len(cases)]
                t = _data(rank, n, torch.float32, it).to(dev)
                o = torch.full((n,), float("nan"), device=dev)
                x.wide_probe(t, o, nb)
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                _check(o, _expect(world, n, torch.float32, it, "sum"), torch.float32, ("wide", it, n, nb))
                out[f"wide{it}"] = o.cpu().numpy().tobytes()
            t = torch.zeros(4097, device=dev)
            o = torch.empty(4097, device=dev)
            t2 = torch.zeros(257, device=dev)
            o2 = torch.empty(257, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                x.wide_probe(t, o, 32)
                x.wide_probe(t2, o2, 2)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                x.wide_probe(t, o, 32)
                x.wide_probe(t2, o2, 2)
            for r in range(8):
                t.copy_(_data(rank, 4097, torch.float32, 200 + r).to(dev))
                t2.copy_(_data(rank, 257, torch.float32, 300 + r).to(dev))
                g.replay()
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                _check(o, _expect(world, 4097, torch.float32, 200 + r, "sum"), torch.float32, ("wide graph", r))
                _check(o2, _expect(world, 257, torch.float32, 300 + r, "sum"), torch.float32, ("wide graph 2", r))
                out[f"wg{r}"] = o.cpu().numpy().tobytes()
            store.set(f"done{rank}", "1")
            store.wait([f"done{r}" for r in range(world)])
            x.close()
            q.put((rank, "ok", out))
            return
        if mode == "twoshot":
            x.set_twoshot_blocks(48)  # all ranks' grids resident together on the one shared GPU
            # reduce-scatter + all-gather engine: 1 / 8 / 32 MiB, ragged sizes, every dtype
            # and op, sizes interleaved (each block's slots are size-independent), results
            # bit-identical across ranks, graph replay, and the RcclComm-style routing via
            # XgmiCollective (one-shot <= 1 MiB, two-shot above)
            out = {}
            it = 0
            cases = [(262144, "f32", "sum"), (2 << 20, "f32", "sum"), (8 << 20, "f32", "sum"),
                     (262145, "f32", "avg"), (3000001, "bf16", "sum"), (1 << 20, "f16", "max"),
                     (777777, "f32", "min"), (5, "f32", "sum"), (2 << 20, "f32", "sum"), (300000, "bf16", "avg")]
            for n, dn, op in cases:
                dt = DTYPES[dn]
                t = _data(rank, n, dt, it).to(dev)
                o = torch.empty_like(t)
                x.all_reduce_twoshot(t, op, o)
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                _check(o, _expect(world, n, dt, it, op), dt, ("twoshot", n, dn, op))
                out[f"ts{it}"] = o.float().cpu().numpy().tobytes()
                it += 1
            xc = C.xgmi.XgmiCollective(x)
            for n in (100, 1 << 20, 3 << 20):
                t = _data(rank, n, torch.float32, it).to(dev)
                xc.all_reduce(t, "sum")
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                _check(t, _expect(world, n, torch.float32, it, "sum"), torch.float32, ("collective", n))
                it += 1
            a = torch.zeros(1 << 21, device=dev)
            b = torch.zeros(5 << 20, dtype=torch.bfloat16, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                x.all_reduce_twoshot(a)
                x.all_reduce_twoshot(b)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                x.all_reduce_twoshot(a)
                x.all_reduce_twoshot(b, "avg")
            for r in range(6):
                a.copy_(_data(rank, 1 << 21, torch.float32, it).to(dev))
                b.copy_(_data(rank, 5 << 20, torch.bfloat16, it + 1).to(dev))
                g.replay()
                torch.cuda.synchronize()
                assert x.error() == 0, x.error_string()
                _check(a, _expect(world, 1 << 21, torch.float32, it, "sum"), torch.float32, ("ts graph a", r))
                _check(b, _expect(world, 5 << 20, torch.bfloat16, it + 1, "avg"), torch.bfloat16, ("ts graph b", r))
                it += 2
            store.set(f"done{rank}", "1")
            store.wait([f"done{r}" for r in range(world)])
            x.close()
            q.put((rank, "ok", out))
            return
        if mode in ("site_timeout", "sgd_timeout"):
            # rank 0 runs an in-kernel exchange whose peer never comes: the kernel must end
            # with the error word set (1), and the fused AMP-SGD must take the skip path
            if rank == 0:
                x.set_timeout(0.5)
                if mode == "site_timeout":
                    o = torch.empty(3 * 16, device=dev)
                    x.site_probe(1, torch.ones(16, device=dev), o, 3)
                    torch.cuda.synchronize()
                else:
                    ps = [torch.randn(n, device=dev) for n in (100, 3000)]
                    before = [p.clone() for p in ps]
                    gs = [torch.randn_like(p) for p in ps]
                    sc = torch.tensor([8.0], device=dev)
                    tr = torch.zeros(1, dtype=torch.int32, device=dev)
                    fi = torch.zeros(1, device=dev)
                    sync = torch.zeros(4, dtype=torch.int64, device=dev)
                    C.optim.amp_sgd_fused(ps, gs, [], 0.1, 0.0, 0.0, 0.0, False, False, [], sc, tr, fi, 2.0, 0.5,
                                          2000, sync, x)
                    torch.cuda.synchronize()
                    for p, b in zip(ps, before):
                        assert torch.equal(p, b), "partial-sum update applied after a failed exchange"
                    assert sc.item() == 4.0 and tr.item() == 0  # skipped step: back-off, as for an inf
                    # the engine's error word stays set: the next fused step gives up at once
                    # (no new wait) and skips and backs off again -- the ranks' parameters
                    # never take a partial average after a failed exchange
                    C.optim.amp_sgd_fused(ps, gs, [], 0.1, 0.0, 0.0, 0.0, False, False, [], sc, tr, fi, 2.0, 0.5,
                                          2000, sync, x)
                    torch.cuda.synchronize()
                    for p, b in zip(ps, before):
                        assert torch.equal(p, b), "update applied with the engine's error word set"
                    assert sc.item() == 2.0 and tr.item() == 0
                assert x.error() == 1, x.error()
            store.set(f"done{rank}", "1")
            store.wait([f"done{r}" for r in range(world)])
            q.put((rank, "ok", None))
            return
        if mode == "timeout":
            # rank 0 waits for a peer that never comes: must return with error 1, not hang
            if rank == 0:
                x.set_timeout(0.5)
                t = torch.ones(100, device=dev)
                x.all_reduce(t)
                torch.cuda.synchronize()
                assert x.error() == 1, x.error()
            store.set(f"done{rank}", "1")
            store.wait([f"done{r}" for r in range(world)])
            q.put((rank, "ok", None))
            return
        out = {}
        it = 0
        # eager: sizes across the chunk boundaries, ragged tails, every dtype and op
        cases = [(33, "f32", "sum"), (2048, "f32", "sum"), (2049, "f32", "sum"), (29034, "f32", "sum"),
                 (262144, "f32", "sum"), (5, "bf16", "sum"), (8195, "bf16", "sum"), (4097, "f16", "sum"),
                 (1000, "f32", "max"), (1000, "f32", "min"), (3001, "f32", "avg")]
        for n, dn, op in cases:
            dt = DTYPES[dn]
            t = _data(rank, n, dt, it).to(dev)
            x.all_reduce(t, op)
            torch.cuda.synchronize()
            assert x.error() == 0, x.error_string()
            _check(t, _expect(world, n, dt, it, op), dt, (n, dn, op))
            out[f"{n}{dn}{op}"] = t.float().cpu().numpy().tobytes()
            it += 1
        # back-to-back reuse of the same slots (parity flips, epochs advance), out of place
        for k in range(40):
            n = (k * 977) % 5000 + 1
            t = _data(rank, n, torch.float32, it).to(dev)
            o = torch.empty_like(t)
            x.all_reduce(t, "sum", o)
            _check(o.cpu() if k % 7 else o, _expect(world, n, torch.float32, it, "sum"), torch.float32, ("loop", k))
            it += 1
        torch.cuda.synchronize()
        assert x.error() == 0, x.error_string()
        # tensors larger than the workspace slot (1 MiB here): XgmiCollective splits them
        # into back-to-back slot-sized launches (ResNet-50-sized DDP buckets)
        xc = C.xgmi.XgmiCollective(x)
        for n, dn, op in ((700001, "f32", "sum"), (600000, "bf16", "avg"), (524288, "f32", "max")):
            dt = DTYPES[dn]
            t = _data(rank, n, dt, it).to(dev)
            xc.all_reduce(t, op)
            torch.cuda.synchronize()
            assert x.error() == 0, x.error_string()
            _check(t, _expect(world, n, dt, it, op), dt, ("chunked", n, dn, op))
            out[f"chunked{n}{dn}{op}"] = t.float().cpu().numpy().tobytes()
            it += 1
        # hipGraph: capture two collectives, replay with fresh inputs each time
        a = torch.zeros(4099, device=dev)
        b = torch.zeros(70000, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            x.all_reduce(a)  # warm-up on the capture stream
            x.all_reduce(b)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            x.all_reduce(a)
            x.all_reduce(b, "max")
        for r in range(12):
            a.copy_(_data(rank, 4099, torch.float32, it).to(dev))
            b.copy_(_data(rank, 70000, torch.float32, it + 1).to(dev))
            g.replay()
            torch.cuda.synchronize()
            assert x.error() == 0, x.error_string()
            _check(a, _expect(world, 4099, torch.float32, it, "sum"), torch.float32, ("graph a", r))
            _check(b, _expect(world, 70000, torch.float32, it + 1, "max"), torch.float32, ("graph b", r))
            it += 2
        store.set(f"done{rank}", "1")
        store.wait([f"done{r}" for r in range(world)])
        x.close()
        q.put((rank, "ok", out))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        q.close()
        q.join_thread()
        os._exit(0)
