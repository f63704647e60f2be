"""Numerics of the native HIP kernels vs plain PyTorch fp32 references."""
import copy

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _block(cin, cout, seed=0):
    torch.manual_seed(seed)
    conv = nn.Conv2d(cin, cout, 5, 1, 2)
    bn = nn.BatchNorm2d(cout)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.1, 0.1)
        bn.running_var.uniform_(0.5, 1.5)
    return conv.to(DEV), bn.to(DEV)


def _ref_block(x, conv, bn):
    y = F.conv2d(x, conv.weight, conv.bias, 1, 2)
    return F.max_pool2d(F.relu(bn(y)), 2, 2)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("cin,cout,hw", [(1, 16, 28), (16, 32, 14)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("B", [32, 12])
def test_conv_block_fwd_bwd(C, cin, cout, hw, dtype, B):
    """fp32: tight vs the fp32 reference.  bf16/fp16: error vs the fp32
    reference must be within 2x of torch's own autocast error (+ floor)."""
    from ddp_practice_amd.ops.convblock import conv_block

    conv, bn = _block(cin, cout)
    conv_r, bn_r = copy.deepcopy(conv), copy.deepcopy(bn)
    conv_l, bn_l = copy.deepcopy(conv), copy.deepcopy(bn)
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.rand(B, cin, hw, hw, generator=g).to(DEV)
    xr = x.clone().requires_grad_(cin > 1)
    xl = x.clone().requires_grad_(cin > 1)
    xn = x.clone().to(dtype).requires_grad_(cin > 1)
    out = conv_block(xn, conv, bn, cdtype=dtype)
    ref = _ref_block(xr, conv_r, bn_r)
    lp = dtype != torch.float32
    if lp:
        with torch.autocast("cuda", dtype=dtype):
            ref_l = _ref_block(xl, conv_l, bn_l)

    def bound(a, r, l, floor):
        e = _rel(a, r)
        lim = max(2.0 * _rel(l, r), floor) if lp else floor
        assert e < lim, (e, lim)

    assert out.dtype == dtype
    bound(out, ref, ref_l if lp else None, 2e-5 if not lp else 5e-3)
    st = 1e-4 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(bn.running_mean, bn_r.running_mean, rtol=st, atol=st)
    torch.testing.assert_close(bn.running_var, bn_r.running_var, rtol=st, atol=st)
    assert int(bn.num_batches_tracked) == int(bn_r.num_batches_tracked) == 1
    go = torch.randn(ref.shape, generator=g).to(DEV)
    ref.backward(go)
    out.backward(go.to(dtype))
    if lp:
        ref_l.backward(go.to(ref_l.dtype))
    fl = 1e-4 if not lp else 5e-3
    bound(conv.weight.grad, conv_r.weight.grad, conv_l.weight.grad if lp else None, fl)
    bound(bn.weight.grad, bn_r.weight.grad, bn_l.weight.grad if lp else None, fl)
    bound(bn.bias.grad, bn_r.bias.grad, bn_l.bias.grad if lp else None, fl)
    # conv bias grad is ~0 analytically (BN follows); compare absolutely
    db_err = (conv.bias.grad - conv_r.bias.grad).abs().max().item()
    db_lim = 2.0 * (conv_l.bias.grad - conv_r.bias.grad).abs().max().item() + 1e-2 if lp else 2e-3
    assert db_err < db_lim, (db_err, db_lim)
    if cin > 1:
        bound(xn.grad, xr.grad, xl.grad if lp else None, fl)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_block_eval(C, dtype):
    from ddp_practice_amd.ops.convblock import conv_block

    conv, bn = _block(16, 32)
    bn.eval()
    x = torch.rand(8, 16, 14, 14, device=DEV)
    with torch.no_grad():
        out = conv_block(x.to(dtype), conv, bn, cdtype=dtype)
        ref = _ref_block(x, conv, bn)
    assert _rel(out, ref) < (2e-5 if dtype == torch.float32 else 2e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K", [(32, 10, 1568), (7, 10, 1568), (40, 33, 100), (128, 1000, 2048)])
def test_linear(C, dtype, M, N, K):
    from ddp_practice_amd.ops.head import linear

    torch.manual_seed(0)
    lin = nn.Linear(K, N).to(DEV)
    x = torch.randn(M, K, device=DEV)
    xr = x.clone().requires_grad_()
    xn = x.clone().to(dtype).requires_grad_()
    w = lin.weight.detach().clone().requires_grad_()
    b = lin.bias.detach().clone().requires_grad_()
    out = linear(xn, w, b, cdtype=dtype)
    ref = F.linear(xr, lin.weight, lin.bias)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol
    go = torch.randn(M, N, device=DEV)
    out.backward(go.to(dtype))
    ref.backward(go)
    assert _rel(w.grad, lin.weight.grad) < tol * 2
    assert _rel(b.grad, lin.bias.grad) < tol * 2
    assert _rel(xn.grad, xr.grad) < tol * 2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_cross_entropy(C, dtype):
    from ddp_practice_amd.ops.head import cross_entropy

    torch.manual_seed(0)
    logits = (torch.randn(32, 10, device=DEV) * 3).to(dtype)
    tgt = torch.randint(0, 10, (32,), device=DEV)
    tgt[3] = -100
    a = logits.clone().requires_grad_()
    r = logits.float().clone().requires_grad_()
    loss = cross_entropy(a, tgt)
    ref = F.cross_entropy(r, tgt)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    (loss * 3).backward()
    (ref * 3).backward()
    torch.testing.assert_close(a.grad.float(), r.grad, rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("B,N", [(128, 1000), (257, 100), (96, 1024)])
def test_cross_entropy_many_rows(C, B, N):
    """B > 64: the multi-workgroup CE kernel (rows held in registers, loss partials summed
    by the last-arriving workgroup) vs torch; called twice (the ticket re-arms itself)."""
    from ddp_practice_amd.ops.head import cross_entropy

    torch.manual_seed(1)
    logits = (torch.randn(B, N, device=DEV) * 3).to(torch.bfloat16)
    tgt = torch.randint(0, N, (B,), device=DEV)
    tgt[5] = -100
    r = logits.float().clone().requires_grad_()
    ref = F.cross_entropy(r, tgt)
    (ref * 3).backward()
    for _ in range(2):
        a = logits.clone().requires_grad_()
        loss = cross_entropy(a, tgt)
        torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
        (loss * 3).backward()
        torch.testing.assert_close(a.grad.float(), r.grad, rtol=1e-2, atol=1e-4)


def test_accuracy(C):
    from ddp_practice_amd.ops.head import accuracy_

    logits = torch.randn(37, 10, device=DEV)
    tgt = torch.randint(0, 10, (37,), device=DEV)
    cnt = torch.zeros(2, device=DEV)
    accuracy_(logits, tgt, cnt)
    assert cnt[0].item() == 37
    assert cnt[1].item() == (logits.argmax(1) == tgt).sum().item()


def test_sgd_and_scaler_kernels(C):
    torch.manual_seed(0)
    ps = [torch.randn(n, device=DEV) for n in (5, 5000, 29034)]
    gs = [torch.randn_like(p) * 1024 for p in ps]
    scale = torch.tensor([1024.0], device=DEV)
    fi = torch.zeros(1, device=DEV)
    ref_p = [p.clone() for p in ps]
    ref_g = [g.clone() / 1024 for g in gs]
    C.optim.unscale_check(gs, scale, fi)
    assert fi.item() == 0
    for g, r in zip(gs, ref_g):
        torch.testing.assert_close(g, r)
    bufs = [torch.zeros_like(p) for p in ps]
    C.optim.sgd_step(ps, gs, bufs, 0.1, 0.9, 0.0, 1e-4, False, False, [1, 1, 1], fi, None)
    opt = torch.optim.SGD([torch.nn.Parameter(p) for p in ref_p], lr=0.1, momentum=0.9, weight_decay=1e-4)
    for p, g in zip(opt.param_groups[0]["params"], ref_g):
        p.grad = g
    opt.step()
    for p, r in zip(ps, opt.param_groups[0]["params"]):
        torch.testing.assert_close(p, r.detach())
    # inf -> found_inf set, step skipped
    gs[1][7] = float("inf")
    before = [p.clone() for p in ps]
    fi.zero_()
    C.optim.unscale_check(gs, scale, fi)
    assert fi.item() == 1
    C.optim.sgd_step(ps, gs, bufs, 0.1, 0.9, 0.0, 0.0, False, False, [], fi, None)
    for p, b in zip(ps, before):
        assert torch.equal(p, b)
    # update_scale semantics
    tr = torch.zeros(1, dtype=torch.int32, device=DEV)
    C.optim.update_scale(scale, tr, fi, 2.0, 0.5, 3)
    assert scale.item() == 512 and tr.item() == 0
    fi.zero_()
    for i in range(3):
        C.optim.update_scale(scale, tr, fi, 2.0, 0.5, 3)
    assert scale.item() == 1024 and tr.item() == 0


def test_flat_copy(C):
    ts = [torch.randn(n, device=DEV) for n in (3, 4097, 10)]
    offs = [0, 3, 4100]
    flat = torch.zeros(4110, device=DEV)
    C.optim.flat_copy(ts, offs, flat, 0.5, 0)
    torch.testing.assert_close(flat, torch.cat(ts) * 0.5)
    outs = [torch.empty_like(t) for t in ts]
    C.optim.flat_copy(outs, offs, flat, 2.0, 1)
    for o, t in zip(outs, ts):
        torch.testing.assert_close(o, t)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gather(C, dtype):
    imgs = torch.randint(0, 256, (100, 28, 28), dtype=torch.uint8, device=DEV)
    labels = torch.randint(0, 10, (100,), device=DEV)
    order = torch.randperm(100, device=DEV)
    ctr = torch.zeros(2, dtype=torch.int32, device=DEV)
    out = torch.empty(32, 1, 28, 28, dtype=dtype, device=DEV)
    lab = torch.empty(32, dtype=torch.long, device=DEV)
    for step in range(3):
        C.data.gather(imgs, labels, order, ctr, -1, out, lab, 1 / 255.0, 0.0)
        sel = order[step * 32:(step + 1) * 32]
        torch.testing.assert_close(out.float(), (imgs[sel].float() / 255).unsqueeze(1).to(dtype).float())
        assert torch.equal(lab, labels[sel])
    assert ctr.tolist() == [3, 0]


@pytest.mark.parametrize("momentum", [0.0, 0.9])
# granules per lane chosen by size: U=1, U=2, U=4, and a grid of one
@pytest.mark.parametrize("sizes", [(7, 3000, 29034), (5, 200001, 33), (5, 300001, 33), (7, 33, 100)])
def test_fused_amp_sgd_matches_unfused(C, momentum, sizes):
    """Grid-barrier fused unscale+check+SGD+update == the three unfused kernels, over
    several launches sharing one barrier state (generations / parity reuse), with
    non-finite grads injected on some of them, eager and graph-replayed."""
    torch.manual_seed(0)
    ps = [torch.randn(n, device=DEV) for n in sizes]
    pa, pb = [p.clone() for p in ps], [p.clone() for p in ps]
    ba, bb = [torch.zeros_like(p) for p in ps], [torch.zeros_like(p) for p in ps]
    sa, sb = torch.tensor([512.0], device=DEV), torch.tensor([512.0], device=DEV)
    ta, tb = torch.zeros(1, dtype=torch.int32, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV)
    fa, fb = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    sync = torch.zeros(4, dtype=torch.int64, device=DEV)
    ga = [torch.empty_like(p) for p in ps]

    def fused(first):
        C.optim.amp_sgd_fused(pa, ga, ba, 0.1, momentum, 0.0, 1e-4, False, False, [int(first)] * len(ps), sa, ta,
                              fa, 2.0, 0.5, 2, sync, None)

    graph = None
    for it in range(8):
        gs = [torch.randn_like(p) * 512 for p in ps]
        if it in (1, 4, 6):
            g = gs[it % len(gs)]
            g[it % g.numel()] = float("nan") if it != 4 else float("inf")
        for x, g in zip(ga, gs):
            x.copy_(g)
        gb = [g.clone() for g in gs]
        first = it == 0
        if it < 4:
            fused(first)
        else:  # graph replay of the same launch (not first: momentum buffers exist)
            if graph is None:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    fused(False)
            graph.replay()
        C.optim.unscale_check(gb, sb, fb)
        C.optim.sgd_step(pb, gb, bb, 0.1, momentum, 0.0, 1e-4, False, False, [int(first)] * len(ps), fb, None)
        C.optim.update_scale(sb, tb, fb, 2.0, 0.5, 2)
        torch.cuda.synchronize()
        for x, y in zip(pa + ga + ba, pb + gb + bb):
            torch.testing.assert_close(x, y, equal_nan=True)
        assert sa.item() == sb.item() and ta.item() == tb.item() and fa.item() == fb.item() == 0.0, it
    # multi-workgroup grid: one barrier generation per launch (4 eager + 4 graph replays;
    # capture runs nothing); a grid of one workgroup (<= 256 lanes x 1 granule at the
    # default granules-per-lane choice) skips the barrier
    solo = sum((n + 3) // 4 for n in sizes) <= 256
    assert int(sync[0]) == (0 if solo else 8)


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("kw", [dict(lr=0.05, momentum=0.9), dict(lr=0.1, momentum=0.9, weight_decay=5e-4),
                                dict(lr=0.1, momentum=0.9, dampening=0.1),
                                dict(lr=0.1, momentum=0.9, nesterov=True, weight_decay=1e-4), dict(lr=0.01),
                                dict(lr=0.05, momentum=0.9, maximize=True)])
def test_sgd_bitwise_equals_torch_foreach_sgd(C, kw, fused, monkeypatch):
    """optim.SGD -- the multi-tensor launch and the fused plain launch -- gives the same bits
    as torch.optim.SGD(foreach=True) over several steps: every update kernel rounds through
    common.h sgd_rule (one fma per ATen foreach op, momentum*buf rounded on its own)."""
    from ddp_practice_amd.optim import SGD, sgd as sgd_mod

    monkeypatch.setattr(sgd_mod, "_PLAIN_FUSED", fused)
    shapes = [(400,), (16,), (32, 16, 5, 5), (10, 1568), (7,), (4099,)]
    res = []
    for make in (lambda ps: torch.optim.SGD(ps, foreach=True, **kw), lambda ps: SGD(ps, **kw)):
        g = torch.Generator(device="cpu").manual_seed(0)
        ps = [torch.randn(s, generator=g).to(DEV).requires_grad_() for s in shapes]
        opt = make(ps)
        for _ in range(4):
            for p in ps:
                p.grad = torch.randn(p.shape, generator=g).to(DEV)
            opt.step()
        torch.cuda.synchronize()
        res.append(([p.detach().clone() for p in ps], [opt.state[p].get("momentum_buffer") for p in ps]))
    (rp, rb), (mp, mb) = res
    for i, (a, b) in enumerate(zip(mp, rp)):
        assert torch.equal(a, b), ("param", i, (a - b).abs().max().item())
    for i, (a, b) in enumerate(zip(mb, rb)):
        assert (a is None) == (b is None), i
        assert a is None or torch.equal(a, b), ("momentum_buffer", i, (a - b).abs().max().item())


@pytest.mark.parametrize("momentum,damp,nesterov", [(0.0, 0.0, False), (0.9, 0.0, True), (0.9, 0.1, False)])
@pytest.mark.parametrize("sizes", [(7, 3000, 29034), (5, 200001, 33), (7, 33, 100)])
def test_fused_plain_sgd_matches_torch_sgd(C, momentum, damp, nesterov, sizes):
    """The fused launch without a scale (optim.SGD's plain step) == torch.optim.SGD bit for
    bit: no unscale, no skip on non-finite gradients (torch applies them), no barrier
    generation used; eager and graph-replayed."""
    torch.manual_seed(1)
    ps = [torch.randn(n, device=DEV) for n in sizes]
    pa = [p.clone() for p in ps]
    pr = [nn.Parameter(p.clone()) for p in ps]
    ref = torch.optim.SGD(pr, lr=0.05, momentum=momentum, dampening=damp, nesterov=nesterov, weight_decay=1e-4)
    ba = [torch.zeros_like(p) for p in ps]
    ga = [torch.empty_like(p) for p in ps]
    sync = torch.zeros(4, dtype=torch.int64, device=DEV)

    def fused(first):
        C.optim.amp_sgd_fused(pa, ga, ba if momentum else [], 0.05, momentum, damp, 1e-4, nesterov, False,
                              [int(first)] * len(ps) if momentum and damp else [], None, None, None, 1.0, 1.0, 1,
                              sync, None)

    graph = None
    for it in range(6):
        gs = [torch.randn_like(p) for p in ps]
        if it == 5:
            gs[0][3] = float("nan")
        for x, g in zip(ga, gs):
            x.copy_(g)
        for q, g in zip(pr, gs):
            q.grad = g.clone()
        if it < 3:
            fused(it == 0)
        else:
            if graph is None:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    fused(False)
            graph.replay()
        ref.step()
        torch.cuda.synchronize()
        for x, q, g in zip(pa, pr, gs):  # bit for bit (common.h sgd_rule rounds as ATen's foreach SGD)
            torch.testing.assert_close(x, q.detach(), rtol=0, atol=0, equal_nan=True)
        for x, g in zip(ga, gs):
            assert torch.equal(x, g) or torch.equal(x.isnan(), g.isnan())  # the gradient is left as it was
        if momentum:
            for b, q in zip(ba, pr):
                torch.testing.assert_close(b, ref.state[q]["momentum_buffer"], rtol=1e-6, atol=1e-6, equal_nan=True)
    assert bool(pa[0][3].isnan())  # applied, as torch does
    assert int(sync[0]) == 0 and int(sync[3]) == 0  # no barrier generation, no error


def test_grad_scaler_fast_backward_and_fused_step(C):
    """scaler.scale(loss).backward() seeds with the scale; fused step == torch GradScaler + SGD."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.ops.head import cross_entropy
    from ddp_practice_amd.optim import SGD

    torch.manual_seed(0)
    w0 = torch.randn(10, 20, device=DEV)
    x = torch.randn(8, 20, device=DEV)
    y = torch.randint(0, 10, (8,), device=DEV)
    wa = torch.nn.Parameter(w0.clone())
    wb = torch.nn.Parameter(w0.clone())
    sa = GradScaler(init_scale=1024.0, growth_interval=2)
    sb = torch.amp.GradScaler("cuda", init_scale=1024.0, growth_interval=2)
    oa, ob = SGD([wa], lr=0.1), torch.optim.SGD([wb], lr=0.1)
    for it in range(4):
        la = cross_entropy(x @ wa.t(), y)
        lb = torch.nn.functional.cross_entropy(x @ wb.t(), y)
        oa.zero_grad()
        ob.zero_grad()
        sa.scale(la).backward()
        sb.scale(lb).backward()
        sa.step(oa)
        sb.step(ob)
        sa.update()
        sb.update()
        assert sa._fused_done is False
        torch.testing.assert_close(wa, wb, rtol=1e-5, atol=1e-6)
        assert sa.get_scale() == sb.get_scale()
    assert sa._single_opt_iters >= 3  # the fused path was taken from iteration 2 on


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cross_entropy_prescaled_by_active_scaler(C, dtype):
    """With an active GradScaler the CE kernel writes loss*scale and d(scale*loss)/dlogits;
    scaler.scale(loss).backward() then returns that gradient without a launch, and the
    generic autograd path (scaled loss used in an expression) stays exact."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.ops.head import cross_entropy

    torch.manual_seed(0)
    sc = GradScaler(init_scale=256.0)
    sc._lazy_init(torch.device(DEV))
    logits = (torch.randn(32, 10, device=DEV) * 3).to(dtype)
    tgt = torch.randint(0, 10, (32,), device=DEV)
    r = logits.float().clone().requires_grad_()
    ref = torch.nn.functional.cross_entropy(r, tgt)
    (ref * 256.0).backward()
    for generic in (False, True):
        a = logits.clone().requires_grad_()
        loss = cross_entropy(a, tgt)
        assert getattr(loss, "_dpa_ce", None) is not None
        scaled = sc.scale(loss)
        torch.testing.assert_close(scaled.float(), ref.detach() * 256.0, rtol=1e-5, atol=1e-3)
        if generic:
            (scaled * 1.0).backward()
        else:
            scaled.backward()
        tol = 1e-5 if dtype == torch.float32 else 1e-2
        torch.testing.assert_close(a.grad.float(), r.grad, rtol=tol, atol=tol * 256)


@pytest.mark.parametrize("momentum,damp,nesterov", [(0.0, 0.0, False), (0.9, 0.0, True), (0.9, 0.1, False)])
def test_large_fused_amp_sgd_matches_unfused(C, momentum, damp, nesterov):
    """Large-model fused step (device tensor table, grid-stride two-phase launch) ==
    the unfused unscale / SGD / update kernels: 161 tensors (ResNet-50's count) with
    ragged sizes and 6.1M floats (> the small kernel's 2^19), non-finite grads on some
    steps, eager and graph-replayed, the table built once and reused."""
    torch.manual_seed(1)
    g = torch.Generator().manual_seed(3)
    sizes = [int(x) for x in torch.randint(1, 90000, (161,), generator=g)]
    sizes[0], sizes[7], sizes[100] = 1, 3, 2_000_001
    ps = [torch.randn(n, device=DEV) for n in sizes]
    pa, pb = [p.clone() for p in ps], [p.clone() for p in ps]
    ba = [torch.zeros_like(p) for p in ps] if momentum else []
    bb = [torch.zeros_like(p) for p in ps] if momentum else []
    sa, sb = torch.tensor([1024.0], device=DEV), torch.tensor([1024.0], device=DEV)
    ta, tb = torch.zeros(1, dtype=torch.int32, device=DEV), torch.zeros(1, dtype=torch.int32, device=DEV)
    fa, fb = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    sync = torch.zeros(4, dtype=torch.int64, device=DEV)
    ga = [torch.empty_like(p) for p in ps]
    tables = {f: C.optim.amp_sgd_table(pa, ga, ba, [int(f)] * len(ps) if damp else []) for f in (True, False)}

    def fused(first):
        C.optim.amp_sgd_large(tables[first], 0.05, momentum, damp, 1e-4, nesterov, False, sa, ta, fa, 2.0, 0.5, 3,
                              sync)

    graph = None
    for it in range(8):
        gs = [torch.randn_like(p) * 1024 for p in ps]
        if it in (2, 5):
            x = gs[(it * 37) % len(gs)]
            x[it % x.numel()] = float("nan") if it == 2 else float("-inf")
        for x, y in zip(ga, gs):
            x.copy_(y)
        gb = [y.clone() for y in gs]
        first = it == 0
        if it < 4:
            fused(first)
        else:
            if graph is None:
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    fused(False)
            graph.replay()
        C.optim.unscale_check(gb, sb, fb)
        C.optim.sgd_step(pb, gb, bb, 0.05, momentum, damp, 1e-4, nesterov, False,
                         [int(first)] * len(ps) if damp else [], fb, None)
        C.optim.update_scale(sb, tb, fb, 2.0, 0.5, 3)
        torch.cuda.synchronize()
        for x, y in zip(pa + ga + ba, pb + gb + bb):
            torch.testing.assert_close(x, y, equal_nan=True)
        assert sa.item() == sb.item() and ta.item() == tb.item() and fa.item() == fb.item() == 0.0, it
    assert int(sync[0]) == 8 and int(sync[3]) == 0


def test_sgd_picks_large_fused_step(C):
    """GradScaler + SGD on a ResNet-sized parameter set take the one-launch large path."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.optim import SGD

    ps = [torch.nn.Parameter(torch.randn(n, device=DEV)) for n in (600000, 5, 9408, 2048) * 10]
    opt = SGD(ps, lr=0.1, momentum=0.9)
    sc = GradScaler()
    calls = {"large": 0, "sgd": 0}
    orig_l, orig_s = C.optim.amp_sgd_large, C.optim.sgd_step

    def spy_l(*a):
        calls["large"] += 1
        return orig_l(*a)

    def spy_s(*a, **k):
        calls["sgd"] += 1
        return orig_s(*a, **k)

    C.optim.amp_sgd_large, C.optim.sgd_step = spy_l, spy_s
    try:
        for _ in range(3):
            loss = sum((p * p).sum() for p in ps)
            opt.zero_grad(set_to_none=False)
            sc.scale(loss).backward()
            sc.step(opt)
            sc.update()
    finally:
        C.optim.amp_sgd_large, C.optim.sgd_step = orig_l, orig_s
    assert opt._fuse_kind() == "large"
    assert calls["large"] >= 2  # the first iteration runs unfused (GradScaler learns the optimizer count)


def test_grad_scaler_scale_twice_on_native_ce(C):
    """A second GradScaler.scale() of the same native CE loss (logging, a retry) takes the
    generic multiply instead of failing on the already-consumed pre-scaled value;
    both scaled values and the resulting gradient are right."""
    from ddp_practice_amd.amp import GradScaler
    from ddp_practice_amd.ops.head import cross_entropy

    torch.manual_seed(0)
    sc = GradScaler(init_scale=64.0)
    sc._lazy_init(torch.device(DEV))
    logits = torch.randn(16, 10, device=DEV)
    tgt = torch.randint(0, 10, (16,), device=DEV)
    r = logits.clone().requires_grad_()
    ref = torch.nn.functional.cross_entropy(r, tgt)
    (ref * 64.0).backward()
    a = logits.clone().requires_grad_()
    loss = cross_entropy(a, tgt)
    first = sc.scale(loss)
    second = sc.scale(loss)
    torch.testing.assert_close(first.float(), ref.detach() * 64.0, rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(second.float(), ref.detach() * 64.0, rtol=1e-5, atol=1e-3)
    second.backward()
    torch.testing.assert_close(a.grad, r.grad, rtol=1e-5, atol=1e-4)


def test_large_table_pinned_when_reused_under_capture(C):
    """The large fused step's device table built by an eager warm-up and then looked up from
    the cache during capture stays referenced for the optimizer's life, and the
    cache key carries each tensor's size."""
    from ddp_practice_amd.optim import SGD

    ps = [torch.nn.Parameter(torch.randn(n, device=DEV)) for n in (600000, 5, 9408, 2048) * 10]
    opt = SGD(ps, lr=0.1)
    for p in ps:
        p.grad = torch.randn_like(p)
    params, grads = list(ps), [p.grad for p in ps]
    t_eager = opt._large_table(params, grads, [], [])
    assert not opt.__dict__.get("_amp_tables_pinned")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            t_cap = opt._large_table(params, grads, [], [])
    assert t_cap is t_eager
    assert any(x is t_eager for x in opt._amp_tables_pinned)
    key = next(iter(opt._amp_tables))
    assert key[0][0] == (ps[0].data_ptr(), ps[0].numel())


def test_synthetic_set_generated_on_device_matches_host(C):
    """The synthetic MNIST set generated in HBM (csrc/kernels/data.hip synth) is the host
    formula (data/mnist.py _noise_np): labels identical, pixels equal up to a rare +-1 from
    float rounding of the noise (logf / cosf vs numpy)."""
    from ddp_practice_amd.data import synthetic

    host = synthetic(3000, seed=5)
    dev = synthetic(3000, seed=5, device=DEV)
    assert dev.images.is_cuda and dev.images.shape == host.images.shape
    assert torch.equal(dev.labels.cpu(), host.labels)
    d = (dev.images.cpu().int() - host.images.int()).abs()
    assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 1e-3
    ims, lab = dev.to_device(torch.device(DEV))
    assert ims.data_ptr() == dev.images.data_ptr()  # no copy of a set built on the device
