"""NHWC implicit-GEMM convolution on MFMA (csrc/kernels/conv_igemm.hip) vs a
plain PyTorch fp32 reference of the same op, and its fused BN statistics vs
the statistics of the storage-rounded output."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _run(C, N, Cin, H, W, K, R, stride, pad, dtype, stats):
    g = torch.Generator().manual_seed(R * 131 + K + H)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, dtype).contiguous(memory_format=CL)
    w = (torch.randn(K, Cin, R, R, generator=g) / (Cin * R * R) ** 0.5).to(DEV, dtype).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // stride + 1
    OW = (W + 2 * pad - R) // stride + 1
    y = torch.empty(N, K, OH, OW, dtype=dtype, device=DEV, memory_format=CL)
    ref = F.conv2d(x.float(), w.float(), None, stride, pad)
    if stats:
        M = N * OH * OW
        part = torch.empty(C.conv_igemm.stat_part_len(M, K), device=DEV)
        tk = torch.zeros(C.conv_igemm.stat_tickets_len(M, K), dtype=torch.int32, device=DEV)
        st = torch.empty(3 * K + 4, device=DEV)
        shift = torch.randn(K, generator=g).to(DEV) * 0.1
        nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
        for _ in range(2):  # the tickets re-arm themselves
            C.conv_igemm.conv_fwd(x, w, y, stride, pad, part, tk, st, shift, nbt)
        assert int(tk.abs().sum()) == 0
    else:
        C.conv_igemm.conv_fwd(x, w, y, stride, pad)
    torch.cuda.synchronize()
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < tol, err
    if stats:
        yr = y.float().permute(0, 2, 3, 1).reshape(-1, K) - shift
        torch.testing.assert_close(st[:K], yr.sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(st[K:2 * K], (yr * yr).sum(0), rtol=1e-4, atol=1e-2)
        assert st[2 * K].item() == M and int(nbt) == 2
        torch.testing.assert_close(st[2 * K + 4:3 * K + 4], shift)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # 3x3 s1, BN=64 tile
    (2, 128, 15, 15, 128, 3, 2, 1),   # 3x3 s2, odd input
    (3, 64, 7, 7, 256, 1, 1, 0),      # 1x1 expand, ragged M = 147
    (2, 256, 14, 14, 128, 1, 2, 0),   # 1x1 s2 projection
    (1, 192, 9, 9, 192, 3, 1, 1),     # Cout = 192: BN=64 tiles
    (8, 64, 56, 56, 64, 1, 1, 0),     # 196 pixel tiles: two-level statistics tree (G1 = 32)
])
@pytest.mark.parametrize("stats", [False, True])
def test_conv_fwd_matches_torch(C, dtype, shape, stats):
    _run(C, *shape, dtype, stats)


@pytest.mark.parametrize("shape", [(2, 64, 14, 14, 128, 3, 1, 1), (2, 128, 9, 9, 64, 3, 2, 1), (2, 64, 8, 8, 64, 1, 1, 0),
                                   (2, 128, 14, 14, 64, 1, 1, 0)])
def test_conv_ops_fwd_bwd_with_stats(C, shape):
    """ops conv_nhwc / conv1x1 with the implicit-GEMM forward (+BN statistics) and the
    stride-1 data gradient on the same kernel == fp32 torch autograd."""
    from ddp_practice_amd.ops.conv1x1 import conv1x1
    from ddp_practice_amd.ops.conv_nhwc import conv_nhwc

    N, Cin, H, W, K, R, stride, pad = shape
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(N, Cin, H, W, generator=g)
    w0 = torch.randn(K, Cin, R, R, generator=g) / (Cin * R * R) ** 0.5
    dy0 = torch.randn(N, K, (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1, generator=g)
    xr, wr = x0.clone().requires_grad_(), w0.clone().requires_grad_()
    F.conv2d(xr, wr, None, stride, pad).backward(dy0)
    bn = torch.nn.BatchNorm2d(K).to(DEV)
    x = x0.to(DEV, torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    w = w0.to(DEV).requires_grad_()
    if R == 1:
        y, st = conv1x1(x, w, stride, torch.bfloat16, None, bn)
    else:
        y, st = conv_nhwc(x, w, (stride, stride), (pad, pad), torch.bfloat16, bn)
    assert st is not None and int(bn.num_batches_tracked) == 1
    y.backward(dy0.to(DEV, torch.bfloat16).contiguous(memory_format=CL))
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad)):
        err = ((got.float().cpu() - ref).abs().max() / ref.abs().max()).item()
        assert err < 2e-2, err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # 64 x 576: BM=64, BN=64
    (2, 128, 15, 15, 128, 3, 2, 1),   # stride 2, odd input
    (3, 256, 7, 7, 128, 1, 1, 0),     # 1x1, ragged pixel count
    (2, 128, 14, 14, 256, 1, 2, 0),   # 1x1 s2 projection
    (4, 64, 28, 28, 128, 3, 1, 1),    # several pixel splits
])
def test_conv_wgrad_matches_torch(C, dtype, shape):
    from ddp_practice_amd.ops.conv_igemm import conv_wgrad

    N, Cin, H, W, K, R, stride, pad = shape
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, dtype).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, K, OH, OH, generator=g).to(DEV, dtype).contiguous(memory_format=CL)
    w = torch.zeros(K, Cin, R, R, device=DEV, requires_grad=True)
    F.conv2d(x.float(), w, None, stride, pad).backward(dy.float())
    got = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
    err = ((got - w.grad).abs().max() / w.grad.abs().max()).item()
    assert err < 1e-2, err


def test_conv1x1_tapped_dgrad_accumulates(C):
    """Identity-block conv1: the residual gradient handed over by the block's last BN
    (GradTap) is accumulated by the 1x1 data-gradient kernel in its epilogue."""
    from ddp_practice_amd.ops.conv1x1 import GradTap, conv1x1

    g = torch.Generator().manual_seed(3)
    N, Cin, H, K = 2, 256, 14, 64
    x0 = torch.randn(N, Cin, H, H, generator=g)
    w0 = torch.randn(K, Cin, 1, 1, generator=g) / Cin ** 0.5
    dy0 = torch.randn(N, K, H, H, generator=g)
    res0 = torch.randn(N, Cin, H, H, generator=g)
    xr = x0.clone().requires_grad_()
    F.conv2d(xr, w0).backward(dy0)
    ref = xr.grad + res0
    x = x0.to(DEV, torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    w = w0.to(DEV).requires_grad_()
    tap = GradTap()
    y = conv1x1(x, w, 1, torch.bfloat16, tap)
    tap.grad = res0.to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    y.backward(dy0.to(DEV, torch.bfloat16).contiguous(memory_format=CL))
    err = ((x.grad.float().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H", [(2, 32), (3, 23)])
def test_stem_conv_fwd_wgrad(C, dtype, N, H):
    """7x7 / stride-2 / pad-3 stem on the kernel's stem mode (4-channel NHWC image,
    (r, s, c) K space padded to 8x8x4) == fp32 torch: output, BN statistics and the
    weight gradient (the padded columns dropped)."""
    from ddp_practice_amd.ops import conv_igemm as I

    g = torch.Generator().manual_seed(5 + H)
    x0 = torch.rand(N, 3, H, H, generator=g)
    conv = torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False)
    w0 = conv.weight.detach().clone()
    wr = w0.clone().requires_grad_()
    ref = F.conv2d(x0, wr, None, 2, 3)
    dy0 = torch.randn(ref.shape, generator=g)
    ref.backward(dy0)
    conv = conv.to(DEV)
    bn = torch.nn.BatchNorm2d(64).to(DEV)
    assert I.stem_usable(x0.to(DEV), conv, dtype)
    y, st = I.stem_conv(x0.to(DEV), conv, dtype, bn)
    assert y.is_contiguous(memory_format=CL) and y.dtype == dtype
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    err = ((y.float().cpu() - ref.detach()).abs().max() / ref.detach().abs().max()).item()
    assert err < tol, err
    yr = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    torch.testing.assert_close(st[:64], yr.sum(0), rtol=1e-4, atol=1e-2)
    y.backward(dy0.to(DEV, dtype).contiguous(memory_format=CL))
    err = ((conv.weight.grad.cpu() - wr.grad).abs().max() / wr.grad.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 64, 16, 16, 64), (2, 128, 14, 14, 192), (3, 64, 10, 10, 128)])
def test_conv3x3_s2_dgrad(C, dtype, shape):
    """Data gradient of a 3x3 / stride-2 conv as four output-parity sub-convolutions
    (MODE_S2T) == fp32 torch autograd, through ops/conv_nhwc."""
    from ddp_practice_amd.ops.conv_nhwc import conv_nhwc

    N, Cin, H, W, K = shape
    g = torch.Generator().manual_seed(17)
    x0 = torch.randn(N, Cin, H, W, generator=g)
    w0 = torch.randn(K, Cin, 3, 3, generator=g) / (Cin * 9) ** 0.5
    xr = x0.clone().requires_grad_()
    out = F.conv2d(xr, w0, None, 2, 1)
    dy0 = torch.randn(out.shape, generator=g)
    out.backward(dy0)
    x = x0.to(DEV, dtype).contiguous(memory_format=CL).requires_grad_()
    w = w0.to(DEV).requires_grad_()
    y = conv_nhwc(x, w, (2, 2), (1, 1), dtype)
    y.backward(dy0.to(DEV, dtype).contiguous(memory_format=CL))
    err = ((x.grad.float().cpu() - xr.grad).abs().max() / xr.grad.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("stride,order", [(1, "ds_first"), (2, "ds_first"), (2, "conv1_first")])
def test_projection_block_shared_input_grad(C, stride, order):
    """A projection block's conv1 (stride 1) and downsample conv (stride s) share the
    input gradient through one tap: the second backward folds the first's product into
    its own (stride 2: added at the even pixels in the conv epilogue)."""
    from ddp_practice_amd.ops.conv1x1 import GradTap, conv1x1

    g = torch.Generator().manual_seed(23 + stride)
    N, Cin, H, K1, Kd = 2, 128, 28, 64, 256
    x0 = torch.randn(N, Cin, H, H, generator=g)
    w1 = torch.randn(K1, Cin, 1, 1, generator=g) / Cin ** 0.5
    wd = torch.randn(Kd, Cin, 1, 1, generator=g) / Cin ** 0.5
    d1 = torch.randn(N, K1, H, H, generator=g)
    dd = torch.randn(N, Kd, H // stride, H // stride, generator=g)
    xr = x0.clone().requires_grad_()
    (F.conv2d(xr, w1) * d1).sum().add((F.conv2d(xr, wd, stride=stride) * dd).sum()).backward()
    x = x0.to(DEV, torch.bfloat16).contiguous(memory_format=CL).requires_grad_()
    tap = GradTap()
    y1 = conv1x1(x, w1.to(DEV), 1, torch.bfloat16, None, None, None, tap)
    yd = conv1x1(x, wd.to(DEV), stride, torch.bfloat16, None, None, None, tap)
    g1 = d1.to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    gd = dd.to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    # order the two backward nodes explicitly (autograd.backward of both outputs picks its own)
    first, second = ((yd, gd), (y1, g1)) if order == "ds_first" else ((y1, g1), (yd, gd))
    torch.autograd.backward([first[0]], [first[1]], retain_graph=True)
    assert x.grad is None and tap.grad is not None
    torch.autograd.backward([second[0]], [second[1]])
    assert tap.grad is None
    err = ((x.grad.float().cpu() - xr.grad).abs().max() / xr.grad.abs().max()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("bp", [128, 256])
@pytest.mark.parametrize("shape", [
    (3, 64, 7, 7, 256, 1),      # ragged M = 147 (one partial tile), BN = 128
    (2, 256, 14, 14, 128, 2),   # stride 2
    (2, 128, 9, 9, 64, 1),      # BN = 64 tiles, ragged M
    (8, 64, 56, 56, 64, 1),     # many pixel tiles: two-level statistics tree
])
def test_conv1x1_glds_kernel_tiles(C, bp, shape):
    """conv_glds_kernel (glds-staged 1x1 GEMM) with each pixel tile forced == fp32 torch:
    output, fused BN statistics (tickets re-armed), accumulate and the even-pixel aux add."""
    K_ = C.conv_igemm
    prev = K_.g1x1_config(1, bp)
    try:
        N, Cin, H, W, K, stride = shape
        _run(C, N, Cin, H, W, K, 1, stride, 0, torch.bfloat16, True)
        _run(C, N, Cin, H, W, K, 1, stride, 0, torch.float16, False)
        g = torch.Generator().manual_seed(bp + K)
        x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
        w = (torch.randn(K, Cin, 1, 1, generator=g) / Cin ** 0.5).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
        ref = F.conv2d(x.float(), w.float(), None, stride)
        y0 = torch.randn(ref.shape, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
        y = y0.clone()
        K_.conv_fwd(x, w, y, stride, 0, accumulate=True)
        err = ((y.float() - (ref + y0.float())).abs().max() / ref.abs().max()).item()
        assert err < 2e-2, err
        OH, OW = ref.shape[2], ref.shape[3]
        if OH % 2 == 0 and OW % 2 == 0:
            aux = torch.randn(N, K, OH // 2, OW // 2, generator=g).to(DEV, torch.bfloat16).contiguous(
                memory_format=CL)
            K_.conv_fwd(x, w, y, stride, 0, aux=aux)
            exp = ref.clone()
            exp[:, :, ::2, ::2] += aux.float()
            err = ((y.float() - exp).abs().max() / exp.abs().max()).item()
            assert err < 2e-2, err
    finally:
        K_.g1x1_config(*prev)


@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # general kernel, 3x3
    (3, 64, 7, 7, 256, 1, 1, 0),      # 1x1 kernel, ragged M
    (8, 64, 56, 56, 64, 1, 1, 0),     # 1x1, 196 pixel tiles: one-level reduction
    (12, 64, 56, 56, 64, 1, 1, 0),    # 294 pixel tiles: one level, 64 rows in flight per lane
    (48, 64, 56, 56, 64, 1, 1, 0),    # 1176 pixel tiles: two-level tree
    (2, 128, 15, 15, 128, 3, 2, 1),   # general kernel, stride 2
])
@pytest.mark.parametrize("defer_min", [0, -1])
def test_conv_fwd_deferred_statistics(C, shape, defer_min):
    """StatArgs.defer (defer_min 0, the default): the conv stores its level-1 partial rows
    and a reduction launch (one or two levels) follows; defer_min -1: the in-launch ticket
    tree -- same statistics, tickets re-armed."""
    K_ = C.conv_igemm
    prev = K_.stat_defer_config(defer_min)
    try:
        _run(C, *shape, torch.bfloat16, True)
    finally:
        K_.stat_defer_config(prev)


@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # 3x3: padding taps read the zero page
    (2, 128, 15, 15, 128, 3, 2, 1),   # stride 2, odd input
    (3, 256, 7, 7, 128, 1, 1, 0),     # 1x1, ragged pixel count (split past the end)
    (2, 128, 14, 14, 256, 1, 2, 0),   # 1x1 stride 2
    (4, 64, 28, 28, 128, 3, 1, 1),    # several pixel splits
])
def test_conv_wgrad_glds_matches_register_staged(C, shape):
    """conv_wgrad_glds_kernel (LDS-DMA staging, zero page for padding) == the register-staged
    weight-gradient kernel bit for bit (same tiles, same MFMA order) and == fp32 torch."""
    from ddp_practice_amd.ops.conv_igemm import conv_wgrad

    K_ = C.conv_igemm
    N, Cin, H, W, K, R, stride, pad = shape
    g = torch.Generator().manual_seed(29)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, K, OH, OH, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    prev = K_.wgrad_config(2)  # the glds kernel for every shape (default: 1x1 only)
    try:
        got = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
        K_.wgrad_config(0)
        old = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
    finally:
        K_.wgrad_config(prev)
    assert torch.equal(got, old)
    w = torch.zeros(K, Cin, R, R, device=DEV, requires_grad=True)
    F.conv2d(x.float(), w, None, stride, pad).backward(dy.float())
    err = ((got - w.grad).abs().max() / w.grad.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # 3x3, one tile x splits
    (3, 256, 7, 7, 128, 1, 1, 0),     # 1x1, ragged pixel count (split past the end)
    (2, 128, 14, 14, 256, 1, 2, 0),   # 1x1 stride 2
    (4, 64, 28, 28, 128, 3, 1, 1),    # several pixel splits
    (8, 256, 14, 14, 512, 1, 1, 0),   # 4 x 2 tiles
])
def test_conv_wgrad_fixup_matches_reduce_launch(C, shape):
    """The split-K reduction inside the weight-gradient launch (the tile's last arriver sums
    the splits, conv_igemm.wgrad_fixup_config) == the separate wgrad_reduce launch up to
    summation order, == fp32 torch, bit-identical from run to run (the tickets re-arm), and
    graph-replayable."""
    from ddp_practice_amd.ops.conv_igemm import conv_wgrad

    K_ = C.conv_igemm
    N, Cin, H, W, K, R, stride, pad = shape
    g = torch.Generator().manual_seed(31)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, K, OH, OH, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    prev_g, prev_f = K_.wgrad_config(2), K_.wgrad_fixup_config(0)
    try:
        ref = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
        K_.wgrad_fixup_config(1 << 20)
        got = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
        again = conv_wgrad(dy, x, (K, Cin, R, R), stride, pad)
        out = torch.empty_like(got)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            out.copy_(conv_wgrad(dy, x, (K, Cin, R, R), stride, pad))
        for _ in range(2):
            out.zero_()
            gr.replay()
            torch.cuda.synchronize()
            assert torch.equal(out, got)
    finally:
        K_.wgrad_config(prev_g)
        K_.wgrad_fixup_config(prev_f)
    assert torch.equal(got, again)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
    w = torch.zeros(K, Cin, R, R, device=DEV, requires_grad=True)
    F.conv2d(x.float(), w, None, stride, pad).backward(dy.float())
    err = ((got - w.grad).abs().max() / w.grad.abs().max()).item()
    assert err < 1e-2, err


@pytest.mark.parametrize("act,R", [(1, 1), (2, 1), (2, 3)])
@pytest.mark.parametrize("shape", [(2, 128, 14, 14, 64), (3, 64, 7, 7, 256), (2, 256, 28, 28, 128),
                                   (12, 64, 56, 56, 64)])
def test_dgrad_epilogue_bn_backward_sums(C, act, R, shape):
    """1x1 data gradient with the producing BatchNorm's backward sums in its epilogue
    (ops/conv_igemm.dgrad_bn, kernel BS modes): dx == fp32 torch (accumulated onto the
    tapped residual gradient for act 1) and S1 = sum dz, S2 = sum dz * xhat of the STORED
    dx == the same sums in fp64 (dz = dx * relu', mask from y (act 1) or recomputed from x)."""
    from ddp_practice_amd.ops.bn_nhwc import BNTap
    from ddp_practice_amd.ops.conv_igemm import dgrad_bn

    N, K, H, W, Cc = shape
    g = torch.Generator().manual_seed(41 + act + Cc)
    bf = dict(device=DEV, dtype=torch.bfloat16)
    dy = torch.randn(N, K, H, W, generator=g).to(**bf).contiguous(memory_format=CL)
    wt = (torch.randn(Cc, K, R, R, generator=g) / (K * R * R) ** 0.5).to(**bf).contiguous(memory_format=CL)
    x = torch.randn(N, Cc, H, W, generator=g).to(**bf).contiguous(memory_format=CL)
    mean = torch.randn(Cc, generator=g) * 0.1
    invstd = torch.rand(Cc, generator=g) + 0.5
    gamma, beta = torch.randn(Cc, generator=g), torch.randn(Cc, generator=g) * 0.3
    bt = BNTap()
    y = acc = None
    if act == 1:
        y = torch.randn(N, Cc, H, W, generator=g).to(**bf).contiguous(memory_format=CL)
        acc = torch.randn(N, Cc, H, W, generator=g).to(**bf).contiguous(memory_format=CL)
    bt.bind_tensors(x, y, act, torch.cat([mean, invstd]).to(DEV), gamma.to(DEV), beta.to(DEV))
    acc0 = acc.clone() if acc is not None else None
    dx = dgrad_bn(dy, wt, bt, acc, R // 2)
    assert dx is not None and bt.matches(dx)
    ref = F.conv2d(dy.float(), wt.float(), None, 1, R // 2)
    if acc0 is not None:
        ref = ref + acc0.float()
    err = ((dx.float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 2e-2, err
    xd, dd = x.double().cpu(), dx.double().cpu()
    if act == 1:
        mask = bt.y.double().cpu() > 0
    else:
        s = (gamma * invstd).double().view(1, -1, 1, 1)
        b = (beta.double() - mean.double() * gamma.double() * invstd.double()).view(1, -1, 1, 1)
        mask = (xd * s + b) > 0
    dz = torch.where(mask, dd, torch.zeros_like(dd))
    xhat = (xd - mean.double().view(1, -1, 1, 1)) * invstd.double().view(1, -1, 1, 1)
    s1, s2 = dz.sum((0, 2, 3)), (dz * xhat).sum((0, 2, 3))
    out, dgamma, dbeta = (t.double().cpu() for t in bt.sums)
    scale = dz.abs().sum((0, 2, 3)) + 1.0
    assert ((out[:Cc] - s1).abs() / scale).max() < 1e-4
    assert ((out[Cc:] - s2).abs() / scale).max() < 1e-4
    assert torch.equal(dbeta, out[:Cc]) and torch.equal(dgamma, out[Cc:])


@pytest.mark.parametrize("on", [0, 1])
@pytest.mark.parametrize("shape", [
    (2, 64, 14, 14, 64, 3, 1, 1),     # 3x3 s1 p1: padding taps read the zero page
    (2, 128, 15, 15, 128, 3, 2, 1),   # 3x3 s2, odd input
    (1, 192, 9, 9, 192, 3, 1, 1),     # Cout = 192: 64-channel tiles
    (2, 64, 12, 12, 128, 5, 1, 2),    # 5x5
])
def test_conv_kxk_glds_and_register_kernels(C, on, shape):
    """KxK convs on the glds kernel (on = 1, the default) and on the register-staged
    general kernel (on = 0) == fp32 torch, with statistics."""
    K_ = C.conv_igemm
    prev = K_.g3x3_config(on)
    try:
        _run(C, *shape, torch.bfloat16, True)
        _run(C, *shape, torch.float16, False)
    finally:
        K_.g3x3_config(prev)


@pytest.mark.parametrize("shape", [
    (3, 64, 7, 7, 256, 1, 1, 0),      # 1x1, ragged M, one K-step (no second tile in flight)
    (2, 256, 14, 14, 128, 1, 2, 0),   # 1x1 stride 2, 4 K-steps
    (4, 1024, 7, 7, 64, 1, 1, 0),     # 1x1, 16 K-steps, 64-channel tiles
    (2, 128, 15, 15, 128, 3, 2, 1),   # 3x3 stride 2: 18 K-steps through the zero page
    (2, 64, 14, 14, 64, 3, 1, 1),     # 3x3, 9 K-steps
])
def test_conv_glds_three_stage_pipeline_bitwise(C, shape):
    """conv_glds_kernel with three LDS buffers (two tiles in flight across a raw barrier)
    == the two-buffer loop bit for bit (same tiles, same MFMA order), statistics included."""
    K_ = C.conv_igemm
    N, Cin, H, W, K, R, stride, pad = shape
    g = torch.Generator().manual_seed(53 + K)
    x = torch.randn(N, Cin, H, W, generator=g).to(DEV, torch.bfloat16).contiguous(memory_format=CL)
    w = (torch.randn(K, Cin, R, R, generator=g) / (Cin * R * R) ** 0.5).to(DEV, torch.bfloat16).contiguous(
        memory_format=CL)
    OH = (H + 2 * pad - R) // stride + 1
    M = N * OH * OH
    outs = []
    prev = K_.glds_config(2)
    try:
        for stages in (2, 3, 2, 3):
            K_.glds_config(stages)
            y = torch.empty(N, K, OH, OH, dtype=torch.bfloat16, device=DEV, memory_format=CL)
            part = torch.empty(K_.stat_part_len(M, K), device=DEV)
            tk = torch.zeros(K_.stat_tickets_len(M, K), dtype=torch.int32, device=DEV)
            st = torch.empty(3 * K + 4, device=DEV)
            K_.conv_fwd(x, w, y, stride, pad, part, tk, st, torch.zeros(K, device=DEV), None)
            torch.cuda.synchronize()
            outs.append((y, st))
    finally:
        K_.glds_config(prev)
    def defined(st):  # [sums | sumsq | rows], shift copy (the 3 floats between are padding)
        return torch.cat([st[:2 * K + 1], st[2 * K + 4:3 * K + 4]])

    for y, st in outs[1:]:
        assert torch.equal(y, outs[0][0]) and torch.equal(defined(st), defined(outs[0][1]))
    ref = F.conv2d(x.float(), w.float(), None, stride, pad)
    assert ((outs[1][0].float() - ref).abs().max() / ref.abs().max()).item() < 2e-2
