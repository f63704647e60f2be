"""Whole-ConvNet fused op (ops/convnet_fused.py) vs the torch module tree (fp32 reference)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(seed=0, n=10):
    from ddp_practice_amd.models import ConvNet

    torch.manual_seed(seed)
    m = ConvNet(num_classes=n)
    with torch.no_grad():
        for bn in (m.layer1[1], m.layer2[1]):
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
    return m.to(DEV)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _torch_fwd(m, x):
    out = m.layer2(m.layer1(x))
    return m.fc(out.reshape(out.size(0), -1))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B,N", [(32, 10), (7, 10), (100, 10), (16, 64)])
def test_convnet_fused_fwd_bwd(C, dtype, B, N):
    """Error of the fused op vs a float64 reference must be within 2x of torch's
    own error at the same precision (fp32 eager, or autocast) plus a small floor."""
    from ddp_practice_amd.ops import convnet_fused

    m = _model(n=N)
    m64, mt = copy.deepcopy(m).double(), copy.deepcopy(m)
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.rand(B, 1, 28, 28, generator=g).to(DEV)
    assert convnet_fused.supported(m, x)
    out = convnet_fused.convnet_forward(m, x, cdtype=dtype)
    bn_out = {}  # float64 BN outputs (pre-ReLU) and their grads: the size of one routing flip
    def keep(k):
        def hook(mod, inp, o):
            o.retain_grad()
            bn_out[k] = (inp[0], o)
        return hook

    hooks = [bnm.register_forward_hook(keep(k)) for k, bnm in (("layer1", m64.layer1[1]), ("layer2", m64.layer2[1]))]
    ref = _torch_fwd(m64, x.double())
    for h in hooks:
        h.remove()
    if dtype == torch.float32:
        ref_t = _torch_fwd(mt, x)
    else:
        with torch.autocast("cuda", dtype=dtype):
            ref_t = _torch_fwd(mt, x)

    lp = dtype != torch.float32
    # fp32: the conv1 weight grad sums ~B*784 terms of a BN-backward output whose
    # channel sums cancel, so both implementations sit at the same 1e-4-level
    # conditioning error with order-dependent spread: allow 4x torch's own error
    fac = 2.0 if lp else 4.0

    def bound(a, r, t, floor, what):
        e = _rel(a, r)
        lim = max(fac * _rel(t, r), floor)
        assert e < lim, (what, e, lim)

    assert out.dtype == dtype and out.shape == (B, N)
    bound(out, ref, ref_t, 1e-5 if not lp else 2e-3, "logits")
    for bn, bnr, bnt in ((m.layer1[1], m64.layer1[1], mt.layer1[1]), (m.layer2[1], m64.layer2[1], mt.layer2[1])):
        bound(bn.running_mean, bnr.running_mean, bnt.running_mean, 1e-5 if not lp else 2e-3, "running_mean")
        bound(bn.running_var, bnr.running_var, bnt.running_var, 1e-5 if not lp else 2e-3, "running_var")
        assert int(bn.num_batches_tracked) == 1
    go = torch.randn(ref.shape, generator=g).to(DEV)
    ref.backward(go.double())
    out.backward(go.to(dtype))
    ref_t.backward(go.to(ref_t.dtype))
    named_t = dict(mt.named_parameters())
    for (n, p), (_, q) in zip(m.named_parameters(), m64.named_parameters()):
        assert p.grad is not None and p.grad.shape == p.shape, n
        if n.endswith("0.bias"):
            # conv bias grad is 0 analytically (BN follows), so only noise is compared.
            # In low precision the fused op normalises the stored (rounded) conv output
            # with statistics of the unrounded fp32 accumulators, so its sum(xhat) over
            # the batch is a random walk of rounding errors rather than ~0: allow 4x
            # torch's noise (which normalises with statistics of the rounded values)
            e = (p.grad.double() - q.grad).abs().max().item()
            lim = (2.0 if not lp else 4.0) * (named_t[n].grad.double() - q.grad).abs().max().item() + \
                (1e-4 if not lp else 1e-2)
            assert e < lim, (n, e, lim)
            continue
        if not lp and n.split(".")[1] == "1":
            # BN affine grads in fp32: a value within an ulp of the ReLU threshold or of
            # its pool-window neighbour can route differently from the float64
            # reference (for either implementation: ~1 such element per 1e6 at these
            # sizes).  One flip moves d(beta) by one |dy| and d(gamma) by one |dy*xhat|,
            # so allow up to 2 flips per channel on top of torch's own error.
            _, o = bn_out[n.split(".")[0]]
            dy = o.grad
            xhat = (o.detach() - bn_out_beta(m64, n)) / bn_out_gamma(m64, n)
            step = (dy * xhat if n.endswith("weight") else dy).abs().amax(dim=(0, 2, 3))
            e = (p.grad.double() - q.grad).abs()
            lim = 2.0 * (named_t[n].grad.double() - q.grad).abs() + 2.0 * step + 1e-6
            assert bool((e <= lim).all()), (n, e.max().item(), (e / lim).max().item())
            continue
        bound(p.grad, q.grad, named_t[n].grad, 1e-5 if not lp else 2e-3, n)


def bn_out_gamma(m, name):
    return getattr(m, name.split(".")[0])[1].weight.detach().view(1, -1, 1, 1)


def bn_out_beta(m, name):
    return getattr(m, name.split(".")[0])[1].bias.detach().view(1, -1, 1, 1)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_convnet_fused_eval(C, dtype):
    from ddp_practice_amd.ops import convnet_fused

    m = _model().eval()
    x = torch.rand(24, 1, 28, 28, device=DEV)
    with torch.no_grad():
        out = convnet_fused.convnet_forward(m, x, cdtype=dtype)
        ref = _torch_fwd(m, x)
    assert _rel(out, ref) < (3e-5 if dtype == torch.float32 else 2e-2)


def test_convnet_fused_matches_layer_path(C):
    """fp32: whole-model op == per-layer ops (same math, different reduction order)."""
    m = _model()
    ml = copy.deepcopy(m)
    ml.fused = "layer"
    x = torch.rand(32, 1, 28, 28, device=DEV)
    for _ in range(3):
        for mod in (m, ml):
            mod.zero_grad(set_to_none=True)
            mod(x).square().mean().backward()
            with torch.no_grad():
                for p in mod.parameters():
                    p.add_(p.grad, alpha=-0.1)
    for (n, p), (_, q) in zip(m.state_dict().items(), ml.state_dict().items()):
        torch.testing.assert_close(p.float(), q.float(), rtol=1e-4, atol=1e-4, msg=n)


def test_convnet_model_dispatches_fused(C):
    from ddp_practice_amd.ops import convnet_fused

    m = _model()
    calls = []
    orig = convnet_fused.ConvNetFn.apply

    def spy(*a):
        calls.append(1)
        return orig(*a)

    convnet_fused.ConvNetFn.apply = spy
    try:
        m(torch.rand(8, 1, 28, 28, device=DEV)).sum().backward()
    finally:
        convnet_fused.ConvNetFn.apply = orig
    assert calls == [1]


def _step(m, x, y, paired, scaler):
    from ddp_practice_amd.data import DeviceLoader
    from ddp_practice_amd.ops.head import cross_entropy

    xx = x.clone()
    if paired:
        DeviceLoader.pair(xx, y)
    if scaler is not None:
        scaler._lazy_init(x.device)  # the active scaler (as after its first step)
    out = m(xx)
    loss = cross_entropy(out, y)
    (scaler.scale(loss) if scaler is not None else loss).backward()
    return out, loss


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("B", [32, 12, 64])
@pytest.mark.parametrize("use_scaler", [True, False])
def test_head_step_matches_three_launch_head(C, dtype, B, use_scaler):
    """Head forward + loss + head backward in one launch (labels paired with the batch,
    csrc/kernels/convnet_head.hip) == the three-launch head (head_fwd, ce_fwd, head_bwd),
    and the loss / head-backward launches really disappear."""
    from ddp_practice_amd.amp import GradScaler

    m1 = _model()
    m1.amp_dtype = None if dtype == torch.float32 else dtype
    m2 = copy.deepcopy(m1)
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.rand(B, 1, 28, 28, generator=g).to(DEV, dtype if dtype != torch.float32 else torch.float32)
    y = torch.randint(0, 10, (B,), generator=g).to(DEV)
    y[1] = -100  # an ignored row
    calls = {"head_bwd": 0, "ce_fwd": 0}
    orig = {"head_bwd": C.convnet.head_bwd, "ce_fwd": C.head.ce_fwd}

    def spy(name):
        def f(*a):
            calls[name] += 1
            return orig[name](*a)
        return f

    out_a, loss_a = _step(m1, x, y, False, GradScaler() if use_scaler else None)
    C.convnet.head_bwd, C.head.ce_fwd = spy("head_bwd"), spy("ce_fwd")
    try:
        out_b, loss_b = _step(m2, x, y, True, GradScaler() if use_scaler else None)
    finally:
        C.convnet.head_bwd, C.head.ce_fwd = orig["head_bwd"], orig["ce_fwd"]
    torch.cuda.synchronize()
    assert calls["ce_fwd"] == 0, "the loss was not taken from the head launch"
    # the head backward rows ran in the head launch: seeded by the GradScaler's scale, or
    # without one by the unit seed of loss.backward() (ops/head.seed_scale)
    assert calls["head_bwd"] == 0
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out_b, out_a) < tol
    assert abs(loss_b.item() - loss_a.item()) <= tol * max(1.0, abs(loss_a.item()))
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        if n.endswith("0.bias"):  # conv bias grad: 0 analytically (BN follows), rounding noise only
            continue
        assert _rel(q.grad, p.grad) < (1e-4 if dtype == torch.float32 else 3e-2), n
    for (n, a), (_, b) in zip(m1.named_buffers(), m2.named_buffers()):
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_deferred_gather_in_conv1(C, dtype):
    """The batch gather folded into conv1 (DeviceLoader.fill_(defer=True), PRO 3) fills
    the same batch buffers, advances the same device step counter and trains to the
    same parameters as the separate gather launch, eagerly and graph-replayed."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, accepts_deferred, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.runtime import CapturedStep

    ds = synthetic(32 * 12, seed=3)
    amp = None if dtype == torch.float32 else dtype
    runs = []
    for defer in (False, True):
        m = _model()
        m.amp_dtype = amp
        loader = DeviceLoader(ds, batch_size=32, shuffle=False, device=DEV, dtype=dtype)
        images, labels = loader.static_batch()
        assert accepts_deferred(m, images)
        opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(enabled=amp is not None), CrossEntropyLoss()
        seen = []

        def step():
            loader.fill_(images, labels, defer=defer)
            loss = crit(m(images), labels)
            opt.zero_grad(set_to_none=True)
            if amp is not None:
                scaler.scale(loss).backward()
                scaler.step(opt)
                scaler.update()
            else:
                loss.backward()
                opt.step()

        loader.start_epoch()
        for _ in range(3):  # eager
            step()
            seen.append((images.clone(), labels.clone()))
        runner = CapturedStep(step, warmup=1, steps_per_graph=2)
        assert runner.capture()
        loader.set_step(5)
        for _ in range(3):
            runner.run()
        seen.append((images.clone(), labels.clone()))
        torch.cuda.synchronize()
        runs.append((copy.deepcopy(m.state_dict()), seen, loader._ctr.clone()))
    (sd_a, seen_a, ctr_a), (sd_b, seen_b, ctr_b) = runs
    assert torch.equal(ctr_a, ctr_b) and int(ctr_b[0]) == 11 and int(ctr_b[1]) == 0
    for (xa, ya), (xb, yb) in zip(seen_a, seen_b):
        assert torch.equal(xa, xb) and torch.equal(ya, yb)
    for k in sd_a:
        torch.testing.assert_close(sd_a[k].float(), sd_b[k].float(), rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.parametrize("defer", [False, True])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_slab_sink_matches_separate_sums(C, dtype, defer, monkeypatch):
    """With a slab sink the conv1 weight gradient and the BN1 / conv1 / conv2 gradient column
    sums run inside the optimizer's fused launch (SGD.defer_wgrad1, convnet.convnet_amp_step:
    5 launches per step; opt-in, ``defer``) -- or only the conv1 column sums (SGD.defer_slab,
    the default) -- == the separate launches, bitwise, eagerly and graph-replayed; no
    slab_reduce launch is left once the fused step runs."""
    from ddp_practice_amd.ops import convnet_fused

    monkeypatch.setattr(convnet_fused, "_DEFER_WGRAD1", defer)
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.runtime import CapturedStep

    ds = synthetic(32 * 12, seed=4)
    runs = []
    orig = C.convblock.slab_reduce
    orig_cas = C.convnet.convnet_amp_step
    for sink in (False, True):
        m = _model()
        m.amp_dtype = dtype
        loader = DeviceLoader(ds, batch_size=32, shuffle=False, device=DEV, dtype=dtype)
        images, labels = loader.static_batch()
        opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(), CrossEntropyLoss()
        if sink:
            assert m.set_slab_sink(opt)
        calls = [0, 0]

        def spy(*a, **k):
            calls[0] += 1
            return orig(*a, **k)

        def spy_cas(*a, **k):
            calls[1] += 1
            return orig_cas(*a, **k)

        def step():
            loader.fill_(images, labels, defer=True)
            loss = crit(m(images), labels)
            opt.zero_grad(set_to_none=True)
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()

        C.convblock.slab_reduce = spy
        C.convnet.convnet_amp_step = spy_cas
        try:
            loader.start_epoch()
            step()  # the first step is unfused: unscale_ flushes the deferred work
            calls[0] = calls[1] = 0
            for _ in range(2):
                step()
            eager_calls = list(calls)
            runner = CapturedStep(step, warmup=1, steps_per_graph=2)
            assert runner.capture()
            for _ in range(3):
                runner.run()
        finally:
            C.convblock.slab_reduce = orig
            C.convnet.convnet_amp_step = orig_cas
        torch.cuda.synchronize()
        assert "_pending_slab" not in opt.__dict__ and "_pending_wgrad1" not in opt.__dict__
        runs.append((copy.deepcopy(m.state_dict()), eager_calls))
    (sd_a, calls_a), (sd_b, calls_b) = runs
    assert calls_a == [2, 0] and calls_b == [0, 2 if defer else 0], (calls_a, calls_b)
    # the merged launch sums in the separate launches' association: bitwise the same training
    for k in sd_a:
        assert torch.equal(sd_a[k], sd_b[k]), k


def test_fp32_plain_fused_step_with_slab_sink(C, monkeypatch):
    """fp32 without a GradScaler: SGD.step() runs the fused launch (no scale), which also sums
    the conv1 weight-gradient slab -- no slab_reduce, no multi-tensor SGD launch -- and the fc
    weight gradient rides in the conv2 weight-gradient launch; the training equals the
    separate launches (DPA_PLAIN_FUSED=0 path) bit for bit, eagerly and graph-replayed."""
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD, sgd as sgd_mod
    from ddp_practice_amd.runtime import CapturedStep

    ds = synthetic(32 * 12, seed=5)
    runs = []
    orig_sr, orig_sgd, orig_fc = C.convblock.slab_reduce, C.optim.sgd_step, C.convnet.fc_wgrad
    for fused in (False, True):
        monkeypatch.setattr(sgd_mod, "_PLAIN_FUSED", fused)
        m = _model()
        loader = DeviceLoader(ds, batch_size=32, shuffle=False, device=DEV, dtype=torch.float32)
        images, labels = loader.static_batch()
        opt, crit = SGD(m.parameters(), lr=0.05, momentum=0.9), CrossEntropyLoss()
        if fused:
            assert m.set_slab_sink(opt)
        calls = [0, 0, 0]

        def spy(i, f):
            def g(*a, **k):
                calls[i] += 1
                return f(*a, **k)
            return g

        def step():
            loader.fill_(images, labels, defer=True)
            loss = crit(m(images), labels)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()

        C.convblock.slab_reduce, C.optim.sgd_step = spy(0, orig_sr), spy(1, orig_sgd)
        C.convnet.fc_wgrad = spy(2, orig_fc)
        try:
            loader.start_epoch()
            step()  # momentum buffers created: the first step may take either path
            calls[:] = [0, 0, 0]
            for _ in range(2):
                step()
            eager_calls = list(calls)
            runner = CapturedStep(step, warmup=1, steps_per_graph=2)
            assert runner.capture()
            for _ in range(3):
                runner.run()
        finally:
            C.convblock.slab_reduce, C.optim.sgd_step, C.convnet.fc_wgrad = orig_sr, orig_sgd, orig_fc
        torch.cuda.synchronize()
        assert "_pending_slab" not in opt.__dict__
        runs.append((copy.deepcopy(m.state_dict()), eager_calls))
    (sd_a, calls_a), (sd_b, calls_b) = runs
    assert calls_a == [2, 2, 0] and calls_b == [0, 0, 0], (calls_a, calls_b)
    # bit-identical: the slab columns are summed in slab_reduce's order and every SGD kernel
    # rounds through one rule (common.h sgd_rule); with a tolerance instead, the 1-ulp
    # differences of two roundings grew past it within ten steps of this fp32 training
    for k in sd_a:
        assert torch.equal(sd_a[k], sd_b[k]), (k, (sd_a[k].float() - sd_b[k].float()).abs().max().item())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [32, 7])
def test_convnet_fused_bitwise_deterministic(C, dtype, B):
    """Two identical fused forward + backward passes give bit-identical logits, running
    statistics and gradients: every reduction of the fused kernels (BN partial rows, ticket
    trees, weight-gradient slabs) has a fixed order, whatever the workgroups' timing."""
    from ddp_practice_amd.ops import convnet_fused

    g = torch.Generator(device="cpu").manual_seed(11)
    x = torch.rand(B, 1, 28, 28, generator=g).to(DEV)
    go = torch.randn(B, 10, generator=g).to(DEV)
    res = []
    for _ in range(2):
        m = _model()
        outs = []
        for _ in range(3):  # three passes: the running statistics feed the next forward's shift
            out = convnet_fused.convnet_forward(m, x, cdtype=dtype)
            out.backward(go.to(dtype))
            outs.append(out.detach().clone())
        torch.cuda.synchronize()
        state = {k: v.detach().clone() for k, v in m.state_dict().items()}
        state.update({"grad." + n: p.grad.detach().clone() for n, p in m.named_parameters()})
        res.append((outs, state))
    (oa, sa), (ob, sb) = res
    for i, (a, b) in enumerate(zip(oa, ob)):
        assert torch.equal(a, b), ("logits", i, (a.float() - b.float()).abs().max().item())
    for k in sa:
        assert torch.equal(sa[k], sb[k]), (k, (sa[k].float() - sb[k].float()).abs().max().item())


def test_slab_sink_flushes_for_grad_readers(C):
    """With a slab sink, .grad read through GradScaler.unscale_ (or accumulated over two
    backward passes) equals the no-sink gradients."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD

    g = torch.Generator(device="cpu").manual_seed(9)
    x = torch.rand(32, 1, 28, 28, generator=g).to(DEV, torch.bfloat16)
    y = torch.randint(0, 10, (32,), generator=g).to(DEV)
    grads = []
    for sink in (False, True):
        m = _model()
        m.amp_dtype = torch.bfloat16
        opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(), CrossEntropyLoss()
        if sink:
            m.set_slab_sink(opt)
        opt.zero_grad(set_to_none=True)
        for _ in range(2):  # two backward passes accumulate into .grad
            scaler.scale(crit(m(x), y)).backward()
        scaler.unscale_(opt)
        torch.cuda.synchronize()
        grads.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_deferred_wgrad1_grads_match_flush(C, dtype, monkeypatch):
    """The optimizer's merged launch (convnet.convnet_amp_step: conv1 weight gradient by
    producer workgroups, BN1 / conv1 / conv2 column sums by slab workgroups) writes the same
    unscaled gradients as the flush path (conv1_wgrad_slab2 + slab_reduce), bitwise, per
    parameter, from the same backward (lr = 0: the update is a no-op)."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.ops import convnet_fused
    from ddp_practice_amd.optim import SGD

    monkeypatch.setattr(convnet_fused, "_DEFER_WGRAD1", True)  # opt-in path (DPA_DEFER_WGRAD1=1)
    g = torch.Generator(device="cpu").manual_seed(11)
    m = _model()
    m.amp_dtype = dtype
    opt, scaler, crit = SGD(m.parameters(), lr=0.0), GradScaler(init_scale=256.0), CrossEntropyLoss()
    assert m.set_slab_sink(opt)
    for it in range(3):
        x = torch.rand(32, 1, 28, 28, generator=g).to(DEV, dtype)
        y = torch.randint(0, 10, (32,), generator=g).to(DEV)
        opt.zero_grad(set_to_none=True)
        scaler.scale(crit(m(x), y)).backward()
        pending = opt.__dict__.get("_pending_wgrad1")
        if it == 0 or pending is None:
            scaler.step(opt)  # first step: unfused (flushes)
            scaler.update()
            continue
        inv = 1.0 / scaler._scale.item()
        opt.flush_slab()
        ref = {n: p.grad.detach().clone() * inv for n, p in m.named_parameters()}
        # the merged launch must recompute every conv1 partial row before its slab owners
        # read them: poisoned rows would surface as NaN gradients
        pending["wslab1"].fill_(float("nan"))
        opt._pending_wgrad1 = pending  # the same deferred work, now through the merged launch
        scaler.step(opt)
        scaler.update()
        torch.cuda.synchronize()
        assert "_pending_wgrad1" not in opt.__dict__
        for n, p in m.named_parameters():  # the flush path's association: bitwise
            assert torch.equal(p.grad, ref[n]), (n, (p.grad - ref[n]).abs().max().item())


def test_deferred_wgrad1_graph_replay_waits_for_producers(C, monkeypatch):
    """Graph-replayed merged steps (convnet.convnet_amp_step) with the conv1 partial rows
    poisoned (NaN) before every replay: the slab owners wait for the in-launch producers,
    so no step sees a NaN gradient (found_inf would halve the scale and skip the step)."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.ops import convnet_fused
    from ddp_practice_amd.runtime import CapturedStep

    monkeypatch.setattr(convnet_fused, "_DEFER_WGRAD1", True)  # opt-in path (DPA_DEFER_WGRAD1=1)
    ds = synthetic(32 * 24, seed=6)
    m = _model()
    m.amp_dtype = torch.bfloat16
    loader = DeviceLoader(ds, batch_size=32, shuffle=False, device=DEV, dtype=torch.bfloat16)
    images, labels = loader.static_batch()
    opt, scaler, crit = SGD(m.parameters(), lr=0.01), GradScaler(init_scale=256.0), CrossEntropyLoss()
    assert m.set_slab_sink(opt)
    slabs = []
    orig = opt.defer_wgrad1

    def record(w):
        slabs.append(w["wslab1"])
        return orig(w)

    opt.defer_wgrad1 = record

    def step():
        loader.fill_(images, labels, defer=True)
        loss = crit(m(images), labels)
        opt.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()

    loader.start_epoch()
    step()
    runner = CapturedStep(step, warmup=1, steps_per_graph=1)
    assert runner.capture()
    wslab1 = slabs[-1]  # the captured step's buffer (graph pool: fixed across replays)
    s0 = scaler._scale.item()
    for _ in range(8):
        wslab1.fill_(float("nan"))
        runner.run()
    torch.cuda.synchronize()
    assert scaler._scale.item() == s0, "a replay saw a non-finite gradient (stale / poisoned conv1 rows)"
    assert all(torch.isfinite(p).all() for p in m.parameters())


def _amp_run(dtype, precheck, monkeypatch, steps=3, scale=None, poison=False, graph=True):
    """ConvNet AMP training with the slab sink (as engine.TrainLoop sets it up); returns the
    final state, the scaler state and how many fused steps ran pre-checked."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.ops import convnet_fused
    from ddp_practice_amd.optim import SGD
    from ddp_practice_amd.runtime import CapturedStep

    monkeypatch.setattr(convnet_fused, "_PRECHECK", precheck)
    ds = synthetic(32 * 12, seed=7)
    if poison:
        ds.images[5] = 255  # a saturated image is still finite: the check must not trip on it
    m = _model(seed=3)
    m.amp_dtype = dtype
    loader = DeviceLoader(ds, batch_size=32, shuffle=False, device=DEV, dtype=dtype)
    images, labels = loader.static_batch()
    opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(), CrossEntropyLoss()
    assert m.set_slab_sink(opt)
    C = __import__("ddp_practice_amd._ext", fromlist=["load"]).load()
    orig = C.optim.amp_sgd_fused
    seen = []

    def spy(*a, **k):
        seen.append(a[-1] is not None if len(a) > 20 else k.get("prechk") is not None)
        return orig(*a, **k)

    def step():
        loader.fill_(images, labels, defer=True)
        loss = crit(m(images), labels)
        opt.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()

    C.optim.amp_sgd_fused = spy
    try:
        loader.start_epoch()
        step()
        if scale is not None:
            scaler._scale.fill_(scale)
        for _ in range(steps):
            step()
        if graph:
            runner = CapturedStep(step, warmup=1, steps_per_graph=2)
            assert runner.capture()
            for _ in range(2):
                runner.run()
    finally:
        C.optim.amp_sgd_fused = orig
    torch.cuda.synchronize()
    return copy.deepcopy(m.state_dict()), scaler._scale.item(), scaler._growth_tracker.item(), seen


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_prechecked_amp_step_matches_barrier(C, dtype, monkeypatch):
    """Producer-checked gradients (the backward launches record per workgroup whether a
    gradient they finish is non-finite once unscaled; the fused AMP step then needs no grid
    barrier) == the barrier step, bitwise, eagerly and graph-replayed."""
    sd_a, s_a, t_a, seen_a = _amp_run(dtype, False, monkeypatch)
    sd_b, s_b, t_b, seen_b = _amp_run(dtype, True, monkeypatch)
    assert not any(seen_a) and all(seen_b[1:]), (seen_a, seen_b)
    assert (s_a, t_a) == (s_b, t_b)
    for k in sd_a:
        assert torch.equal(sd_a[k], sd_b[k]), k


@pytest.mark.parametrize("scale", [2.0 ** 127, float("inf"), 0.25])
def test_prechecked_amp_step_skips_overflow(C, scale, monkeypatch):
    """A scale that overflows the scaled gradients (or is infinite): every pre-checked step is
    skipped and the scale backs off exactly as with the barrier step; parameters stay equal.
    A scale below 1 (the words describe scaled values) takes the barrier inside the launch."""
    runs = [_amp_run(torch.float16, pc, monkeypatch, steps=2, scale=scale, graph=False) for pc in (False, True)]
    (sd_a, s_a, t_a, _), (sd_b, s_b, t_b, seen_b) = runs
    assert all(seen_b[1:])
    assert (s_a, t_a) == (s_b, t_b) and (s_b < 2.0 ** 127 or scale == float("inf"))  # inf * backoff stays inf
    for k in sd_a:
        assert torch.equal(sd_a[k], sd_b[k]), k


@pytest.mark.parametrize("dp,xval,flagged", [(4e36, 0.0, True), (1.0, 0.0, False), (1.0, 0.5, False)])
def test_conv1_bias_partials_are_prechecked(C, dp, xval, flagged):
    """The producer-side gradient check covers the conv1 BIAS partial rows, not only the
    weight partials: with a zero input image every weight partial is exactly 0 while the
    bias partials (sums of BN1's backward output over a workgroup's pixels) exceed the row
    bound FLT_MAX / rows -- the check word must be set (a step would otherwise apply an
    overflowing bias sum unskipped)."""
    cn, cb = C.convnet, C.convblock
    B, dt = 2, torch.bfloat16
    g = torch.Generator().manual_seed(4)
    x = torch.full((B, 1, 28, 28), xval).to(DEV, dt)
    y1 = torch.randn(B, 16, 28, 28, generator=g).to(DEV, dt)
    dp1 = torch.full((B, 16, 14, 14), dp).to(DEV, dt)
    idx1 = torch.full((B, 16, 14, 14), 4, dtype=torch.uint8, device=DEV)  # window position 0, ReLU open
    n = float(B * 28 * 28)
    fstats1 = torch.zeros(cb.stats_len(16), device=DEV)
    fstats1[16:32] = n  # sum((y - shift)^2) = n: unit variance, zero mean, zero shift
    fstats1[32] = n
    gsum1 = torch.zeros(cn.dgrad2_rows(B) * 32, device=DEV)  # BN1 backward sums: zero
    g1 = torch.ones(16, device=DEV)
    dg1, dbe1 = torch.empty(16, device=DEV), torch.empty(16, device=DEV)
    nwg1, rows2 = cn.wgrad_bn_rows(1, B), cn.wgrad_bn_rows(2, B)
    wslab1 = torch.empty(nwg1 * (16 * 25 + 16), device=DEV)
    wslab2 = torch.zeros(rows2 * (32 * 400 + 32), device=DEV)
    out2 = torch.empty(32 * 400 + 32, device=DEV)
    chk = torch.zeros(2, dtype=torch.int32, device=DEV)
    cn.conv1_wgrad_slab2(x, y1, dp1, idx1, fstats1, gsum1, None, g1, 1e-5, dg1, dbe1, wslab1, wslab2, out2, None, chk)
    torch.cuda.synchronize()
    rows = wslab1.view(nwg1, 16 * 25 + 16)
    if xval == 0.0:
        assert bool((rows[:, :400] == 0).all())  # the weight partials: exactly zero
    assert bool(torch.isfinite(rows).all())
    if flagged:
        assert rows[:, 400:].abs().max().item() > 3.402823466e38 / nwg1  # only the bias partials exceed
    assert (int(chk[0]) != 0) == flagged, (int(chk[0]), rows[:, 400:].abs().max().item())


def test_prechecked_dropped_by_grad_readers(C, monkeypatch):
    """Reading .grad between backward and step (GradScaler.unscale_ flushes the deferred work)
    drops the producer checks: that step agrees on found_inf at the barrier instead."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.data import DeviceLoader, synthetic
    from ddp_practice_amd.nn import CrossEntropyLoss
    from ddp_practice_amd.ops import convnet_fused
    from ddp_practice_amd.optim import SGD

    monkeypatch.setattr(convnet_fused, "_PRECHECK", True)
    m = _model(seed=1)
    m.amp_dtype = torch.bfloat16
    loader = DeviceLoader(synthetic(64, seed=2), batch_size=32, shuffle=False, device=DEV, dtype=torch.bfloat16)
    images, labels = loader.static_batch()
    opt, scaler, crit = SGD(m.parameters(), lr=0.05), GradScaler(), CrossEntropyLoss()
    assert m.set_slab_sink(opt)
    loader.start_epoch()
    for unscale in (False, True):
        loader.fill_(images, labels, defer=True)
        loss = crit(m(images), labels)
        opt.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        assert "_prechecked" in opt.__dict__
        if unscale:
            scaler.unscale_(opt)
            assert "_prechecked" not in opt.__dict__
        scaler.step(opt)
        scaler.update()
        assert "_prechecked" not in opt.__dict__
    torch.cuda.synchronize()
    assert all(torch.isfinite(p).all() for p in m.parameters())
