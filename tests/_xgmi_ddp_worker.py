"""Worker for tests/test_xgmi_ddp_gpu.py: DDP + SyncBN ConvNet training with W
processes on ONE GPU, every all-reduce (SyncBN statistics, DDP bucket) on the
xGMI engine, compared with a single-process run on the global batch."""
import copy
import hashlib
import os
import traceback

import torch


def _train(model, ds, batch, scaler_on, use_graph, sampler=None, epochs=2):
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader
    from ddp_practice_amd.engine import TrainLoop
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD

    loader = DeviceLoader(ds, batch_size=batch, shuffle=False, sampler=sampler, device="cuda",
                          dtype=torch.bfloat16 if scaler_on else torch.float32)
    opt = SGD(model.parameters(), lr=0.05)
    scaler = GradScaler() if scaler_on else None
    loop = TrainLoop(model, CrossEntropyLoss(), opt, loader, scaler, use_graph=use_graph, steps_per_graph=4)
    if (scaler_on or opt.plain_fused) and hasattr(model, "defer_grad_sync_to"):
        # DDP + fused step (AMP, or fp32's plain one) over the xGMI engine: gradients averaged
        # inside the optimizer kernel
        assert getattr(opt, "_deferred_ddp", None) is not None
    for e in range(epochs):
        if sampler is not None:
            sampler.set_epoch(e)
        loop.run_epoch()
        if os.environ.get("DPA_TEST_PROGRESS") == "1":
            import sys

            torch.cuda.synchronize()
            print(f"[pid {os.getpid()}] epoch {e} done", file=sys.stderr, flush=True)
    assert loop.graph_error is None, loop.graph_error
    return model


def _stall_report(c, rank, after_s):
    """Print this rank's engine state (host-issued counts, every site's epoch words and the
    peers' newest granule epochs: XgmiComm.debug_state) if the worker is still running
    after ``after_s`` -- a stall then names its exchange instead of timing out silently."""
    import sys
    import threading

    def dump():
        try:
            print(f"[rank {rank}] still running after {after_s:.0f} s: {c.xgmi.debug_state(1.0)}", file=sys.stderr,
                  flush=True)
        except Exception as e:  # pragma: no cover - diagnostics only
            print(f"[rank {rank}] debug_state failed: {e!r}", file=sys.stderr, flush=True)

    t = threading.Timer(after_s, dump)
    t.daemon = True
    t.start()


def _digest(sd):
    h = hashlib.sha1()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().float().cpu().numpy().tobytes())
    return h.hexdigest()


def worker(rank, world, port, amp, graph, q):
    try:
        from ._dist import client_env

        os.environ.update(client_env(rank, world, port))
        if world >= 3:
            # several ranks on one card (runtime/device.shared_gpu_env: one HW queue each, and
            # no launch whose own grid barrier needs a whole card per rank -- the deferred conv1
            # weight gradient); the in-kernel SyncBN sites and the AMP-SGD gradient exchange
            # forced on
            from ddp_practice_amd.runtime.device import shared_cu_mask, shared_gpu_env

            shared_gpu_env(world)
            shared_cu_mask(world, rank)  # this rank's own CU range: a small "GPU" per rank
            os.environ["DPA_FUSED_SYNC"] = "1"
            os.environ["DPA_FUSED_GRAD"] = "1"
            # a stalled exchange gives up (error word) well inside the test's budget
            os.environ.setdefault("DPA_XGMI_TIMEOUT", "45")
        torch.cuda.set_device(0)
        import ddp_practice_amd.distributed as dist
        from ddp_practice_amd.data import DistributedSampler, synthetic
        from ddp_practice_amd.models import ConvNet
        from ddp_practice_amd.parallel import DistributedDataParallel, XgmiCommunicator, convert_sync_batchnorm

        c = dist.init_process_group("xgmi")
        assert isinstance(c, XgmiCommunicator)
        if world >= 3:
            _stall_report(c, rank, 40.0)
        from ddp_practice_amd.ops.convnet_fused import _fused_site_engine

        # the SyncBN sums are exchanged inside the kernels (not one launch per collective)
        assert _fused_site_engine(c, 16 if world <= 2 else 4, torch.bfloat16 if amp else torch.float32) is not None
        # 8 ranks on one card, 32 CUs each (shared_cu_mask): 4 images per rank, so every
        # exchanging grid (in-kernel SyncBN sites, the AMP-SGD gradient exchange) is co-resident
        # within the rank's CUs
        per_rank = 16 if world <= 2 else 4
        ds = synthetic(per_rank * world * 9 + 3 * world, seed=11)  # 9 full steps + a partial step per epoch
        torch.manual_seed(rank)  # different init per rank: DDP must broadcast rank 0's
        dt = torch.bfloat16 if amp else None
        ddp = DistributedDataParallel(convert_sync_batchnorm(ConvNet(amp_dtype=dt).cuda()), device_ids=[0],
                                      gradient_as_bucket_view=True)
        assert ddp.reducer is not None
        init = copy.deepcopy(ddp.module.state_dict())
        # one step, gradients: DDP-averaged grads of the rank batches == grads of the global batch
        from ddp_practice_amd.ops.head import cross_entropy

        g = torch.Generator().manual_seed(99)
        gx = torch.rand(per_rank * world, 1, 28, 28, generator=g).cuda()
        gy = torch.randint(0, 10, (per_rank * world,), generator=g).cuda()
        one = copy.deepcopy(ddp.module)
        ddp1 = DistributedDataParallel(one, device_ids=[0], gradient_as_bucket_view=True)
        sl = slice(rank * per_rank, (rank + 1) * per_rank)
        cross_entropy(ddp1(gx[sl].to(dt or torch.float32)), gy[sl]).backward()
        grads = {k: p.grad.detach().clone() for k, p in one.named_parameters()}
        del ddp1
        sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=5)
        _train(ddp, ds, per_rank, amp, graph, sampler=sampler)
        torch.cuda.synchronize()
        assert c.async_error() == "", c.async_error()
        res = {"digest": _digest(ddp.module.state_dict())}
        if rank == 0:
            # the same optimisation on ONE process over the global batch, in the
            # order the distributed sampler interleaves the ranks' samples
            from ddp_practice_amd.data import ImageDataset

            plain = ConvNet(amp_dtype=dt).cuda()
            plain.load_state_dict(init)
            plain1 = copy.deepcopy(plain)
            cross_entropy(plain1(gx.to(dt or torch.float32)), gy).backward()
            gtol = 2e-5 if not amp else 2e-2
            gerrs = {}
            for k, p in plain1.named_parameters():
                if k.endswith("0.bias"):  # analytically 0 (BN follows): noise only
                    continue
                gerrs[k] = ((grads[k] - p.grad).norm() / (p.grad.norm() + 1e-12)).item()
            res["grad_errs"] = gerrs
            assert all(e < gtol for e in gerrs.values()), gerrs
            n = len(ds)
            imgs, labels = [], []
            for e in range(2):
                order = torch.randperm(n, generator=torch.Generator().manual_seed(5 + e))
                shards = [order[r::world] for r in range(world)]
                for s0 in range(0, n // world, per_rank):
                    idx = torch.cat([sh[s0:s0 + per_rank] for sh in shards])
                    imgs.append(ds.images[idx])
                    labels.append(ds.labels[idx])
            # one global batch per step: the rank-major concatenation above
            steps_ds = ImageDataset(torch.cat(imgs), torch.cat(labels))
            sizes = [len(x) for x in labels]
            from ddp_practice_amd.engine import TrainLoop  # noqa: F401
            pos = 0
            ref = plain
            for sz in sizes:
                sub = ImageDataset(steps_ds.images[pos:pos + sz], steps_ds.labels[pos:pos + sz])
                _train(ref, sub, sz, amp, False, epochs=1)
                pos += sz
            # 20 SGD steps at lr 0.05 amplify reduction-order differences (the conv1
            # weight grad is a sum of ~B*784 cancelling terms): a loose trajectory check
            tol = 2e-3 if not amp else 6e-2
            errs = {}
            for (k, p), (_, r) in zip(ddp.module.state_dict().items(), ref.state_dict().items()):
                if p.dtype.is_floating_point:
                    errs[k] = ((p.float() - r.float()).norm() / (r.float().norm() + 1e-6)).item()
                else:
                    assert torch.equal(p, r), (k, p, r)
            res["errs"] = errs
            assert all(e < tol for e in errs.values()), errs
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        q.close()
        q.join_thread()
        os._exit(0)


def worker_poison(rank, world, port, q):
    """Pre-checked AMP step under DDP over the xGMI engine: rank 1's gradients overflow (its
    scale is made infinite), rank 0's are finite -- rank 1's AMP step pushes NaN in place of
    its values, so rank 0 skips the step too: parameters unchanged, scale backed off."""
    try:
        from ._dist import client_env

        os.environ.update(client_env(rank, world, port))
        torch.cuda.set_device(0)
        import ddp_practice_amd.distributed as dist
        from ddp_practice_amd import _ext
        from ddp_practice_amd.amp import GradScaler
        from ddp_practice_amd.data import DeviceLoader, DistributedSampler, synthetic
        from ddp_practice_amd.engine import TrainLoop
        from ddp_practice_amd.models import ConvNet
        from ddp_practice_amd.nn import CrossEntropyLoss
        from ddp_practice_amd.optim import SGD
        from ddp_practice_amd.parallel import DistributedDataParallel, convert_sync_batchnorm

        dist.init_process_group("xgmi")
        torch.manual_seed(0)
        ddp = DistributedDataParallel(convert_sync_batchnorm(ConvNet(amp_dtype=torch.bfloat16).cuda()), device_ids=[0],
                                      gradient_as_bucket_view=True)
        ds = synthetic(16 * world * 6, seed=11)
        sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=False)
        loader = DeviceLoader(ds, batch_size=16, shuffle=False, sampler=sampler, device="cuda", dtype=torch.bfloat16)
        opt, scaler = SGD(ddp.parameters(), lr=0.05), GradScaler()
        loop = TrainLoop(ddp, CrossEntropyLoss(), opt, loader, scaler, use_graph=False)
        assert getattr(opt, "_deferred_ddp", None) is not None
        C = _ext.load()
        orig = C.optim.amp_sgd_fused
        seen = []

        def spy(*a, **k):
            seen.append(len(a) > 20 and a[-1] is not None)
            return orig(*a, **k)

        C.optim.amp_sgd_fused = spy
        loader.start_epoch()
        for _ in range(3):
            loop._eager_step()
        torch.cuda.synchronize()
        before = {k: p.detach().clone() for k, p in ddp.module.named_parameters()}
        s0 = scaler._scale.item()
        if rank == 1:
            scaler._scale.fill_(float("inf"))
        seen.clear()
        loop._eager_step()
        torch.cuda.synchronize()
        C.optim.amp_sgd_fused = orig
        assert seen == [True], seen  # the step ran pre-checked (no grid barrier) on this rank
        changed = [k for k, p in ddp.module.named_parameters() if not torch.equal(p.detach(), before[k])]
        assert changed == [], changed
        if rank == 0:
            assert scaler._scale.item() == s0 * 0.5, (s0, scaler._scale.item())
        dist.destroy_process_group()
        q.put((rank, "ok", {"scale": scaler._scale.item()}))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        q.close()
        q.join_thread()
        os._exit(0)


def worker_resnet(rank, world, port, q):
    """ResNet-50 (native bf16 kernels) with SyncBN under DDP over the xGMI engine, one
    forward + backward on each rank's slice of a global batch: the DDP-averaged gradients
    are bit-identical on every rank; the SyncBN statistics equal one process's on the
    global batch; the gradients are as close to that process's as its own are to a run on
    the same batch in another order (a random-init ResNet-50 in bf16 is chaotic: the BN
    summation order alone moves its gradients by O(1), profiles/r6aq_resnet50_ddp_conditioning.txt);
    then one SGD step keeps the ranks bit-identical."""
    try:
        from ._dist import client_env

        os.environ.update(client_env(rank, world, port))
        torch.cuda.set_device(0)
        import ddp_practice_amd.distributed as dist
        from ddp_practice_amd.models import resnet50
        from ddp_practice_amd.ops.head import cross_entropy
        from ddp_practice_amd.optim import SGD
        from ddp_practice_amd.parallel import DistributedDataParallel, XgmiCommunicator, convert_sync_batchnorm

        c = dist.init_process_group("xgmi")
        assert isinstance(c, XgmiCommunicator)
        per_rank = 4
        torch.manual_seed(rank)  # different init per rank: DDP must broadcast rank 0's
        model = convert_sync_batchnorm(resnet50(num_classes=10, amp_dtype=torch.bfloat16)).cuda()
        ddp = DistributedDataParallel(model, device_ids=[0], gradient_as_bucket_view=True)
        init = copy.deepcopy(ddp.module.state_dict())
        g = torch.Generator().manual_seed(21)
        hw = int(os.environ.get("DPA_TEST_IMG", "64"))
        gx = torch.rand(per_rank * world, 3, hw, hw, generator=g).cuda()
        gx += torch.arange(per_rank * world, device="cuda").div(per_rank, rounding_mode="floor").view(-1, 1, 1, 1)
        # (rank r's images brighter by r: unsynchronised statistics would differ by tens of percent)
        gy = torch.randint(0, 10, (per_rank * world,), generator=g).cuda()
        sl = slice(rank * per_rank, (rank + 1) * per_rank)
        cross_entropy(ddp(gx[sl]), gy[sl]).backward()
        torch.cuda.synchronize()
        assert c.async_error() == "", c.async_error()
        bufs_after = {k: b.detach().clone() for k, b in ddp.module.named_buffers()}
        grads = {k: p.grad.detach().clone() for k, p in ddp.module.named_parameters()}
        res = {"grad_digest": _digest(grads)}
        opt = SGD(ddp.module.parameters(), lr=0.01, momentum=0.9)
        opt.step()
        torch.cuda.synchronize()
        res["digest"] = _digest(ddp.module.state_dict())
        if rank == 0:
            def run(order):
                m = resnet50(num_classes=10, amp_dtype=torch.bfloat16).cuda()  # plain BN, one process
                m.load_state_dict(init)
                cross_entropy(m(gx[order]), gy[order]).backward()
                return m

            def rel(a, b):
                return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-30)).item()

            med = lambda d: sorted(d.values())[len(d) // 2]  # noqa: E731
            one = run(torch.arange(per_rank * world).cuda())
            two = run(torch.cat([torch.arange(per_rank, per_rank * world), torch.arange(per_rank)]).cuda())
            gone, gtwo = dict(one.named_parameters()), dict(two.named_parameters())
            errs = {k: rel(grads[k], p.grad) for k, p in gone.items() if p.grad.norm() > 0}
            spread = {k: rel(gtwo[k].grad, p.grad) for k, p in gone.items() if p.grad.norm() > 0}
            # SyncBN statistics: the running-statistics update of the stem BN and layer1 (before the
            # chaos builds up) vs the single process's
            berr = {}
            for k, b in one.named_buffers():
                if b.dtype.is_floating_point and k.startswith(("bn1.", "layer1.")):
                    d = b.float() - init[k].float()
                    berr[k] = rel(bufs_after[k].float() - init[k].float(), d)
            res.update(grad_err_median=med(errs), spread_median=med(spread), stat_err_max=max(berr.values()))
            assert max(berr.values()) < 2e-3, sorted(berr.items(), key=lambda t: -t[1])[:5]
            assert med(errs) < 1.5 * med(spread) + 0.05, (med(errs), med(spread))
        dist.destroy_process_group()
        q.put((rank, "ok", res))
    except Exception:  # pragma: no cover - reported to the parent
        q.put((rank, "err", traceback.format_exc()))
    finally:
        q.close()
        q.join_thread()
        os._exit(0)
