"""1x1 convolution of a channels_last activation as GEMMs over its NHWC rows.

Used by the ResNet-50 stress model (models/resnet.py): 36 of its 53 convolutions
are 1x1.  With the activation stored NHWC, a 1x1 conv is a plain GEMM on the
[P = N*H*W, C] row matrix, so it runs on hipBLASLt with no layout work:

  forward  out[P, Cout] = rows[P, Cin] @ W^T
  dgrad    d_rows[P, Cin] = dY[P, Cout] @ W
  wgrad    dW[Cout, Cin] = dY^T @ rows   -- K = P is huge (401,408 at 56x56, bs 128)
           and the output tiny, so a single GEMM leaves the chip idle (hipBLASLt
           picks a 16-workgroup tile: 650 us for a 13 GFLOP problem).  It runs as
           a split-K batched GEMM instead: the rows are cut into S chunks of
           ~2-4k rows, one fp32 [Cout, Cin] partial per chunk (bmm, fp32
           output), summed in fp32 -- 7-13x faster at 56x56 / 28x28 (measured:
           profiles/r1_gemm1x1_bs128.txt).
The fp32 weight is cast to the compute dtype inside the op and its gradient
comes back in fp32 straight from the fp32 partial sum (no bf16 round trip).
"""
from __future__ import annotations

import torch

from . import conv_igemm as _igemm

WGRAD_CHUNK_ROWS = 2048
WGRAD_MAX_SPLIT = 64


def wgrad_split(P: int) -> int:
    """Number of K chunks for a wgrad over P rows: the largest power of two
    <= min(64, P // 2048) that divides P."""
    s = 1
    while s * 2 <= min(WGRAD_MAX_SPLIT, P // WGRAD_CHUNK_ROWS) and P % (s * 2) == 0:
        s *= 2
    return s


def _wgrad(dyr: torch.Tensor, rows: torch.Tensor) -> torch.Tensor:
    """fp32 dY^T @ rows for [P, Cout] / [P, Cin] row matrices."""
    if not dyr.is_cuda:
        return torch.mm(dyr.t().float(), rows.float())
    P = rows.shape[0]
    S = wgrad_split(P)
    if S == 1:
        return torch.mm(dyr.t(), rows, out_dtype=torch.float32)
    part = torch.bmm(dyr.view(S, P // S, -1).transpose(1, 2), rows.view(S, P // S, -1), out_dtype=torch.float32)
    return part.sum(0)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (any layout) -> contiguous [N*H*W, C] row matrix."""
    r = t.permute(0, 2, 3, 1)
    if not r.is_contiguous():
        r = r.contiguous()
    return r.reshape(-1, t.shape[1])


class GradTap:
    """Hand-off of a residual gradient between two autograd nodes of one block.

    A bottleneck without projection computes ``relu(bn3(...) + x)`` where ``x``
    also feeds ``conv1``; autograd would add the two gradients of ``x`` with a
    separate elementwise kernel.  With a tap, the BN (ops/bn_nhwc.py) stores
    d(res) here instead of returning it, and ``conv1``'s dgrad GEMM accumulates
    onto it in place (``addmm_``: C = C + dY @ W in the GEMM epilogue).  bn3's
    backward always runs before conv1's (conv1 is upstream of bn3), so the
    gradient is present when conv1 needs it.
    """

    __slots__ = ("grad",)

    def __init__(self):
        self.grad = None


class Conv1x1Fn(torch.autograd.Function):
    """``xtap``: a :class:`GradTap` shared by the two 1x1 convs that read the same input
    (a projection block's conv1 and its downsample conv).  Whichever backward runs
    first deposits its data gradient there (stride 2: the compact [N, C, H/2, W/2]
    product, not scattered) and returns none; the second folds it into its own -- the
    stride-1 conv's implicit-GEMM epilogue adds a compact one at the even pixels
    (``aux``) or accumulates onto a full one -- so autograd's separate gradient add,
    the zero-filled stride-2 gradient and its scatter disappear."""

    @staticmethod
    def forward(ctx, x, weight, stride: int, cdtype: torch.dtype, tap: GradTap | None = None, bn=None, packed=None,
                xtap: GradTap | None = None, btap=None):
        in_shape = x.shape
        ctx.btap = btap if stride == 1 else None  # ops/bn_nhwc.BNTap of the BN that produced x
        if tap is not None and stride != 1:
            raise ValueError("conv1x1: a gradient tap needs stride 1")
        ctx.tap = tap
        ctx.xtap = xtap
        ctx.wshape = weight.shape
        ctx.wparam = weight  # the leaf parameter (ops/conv_igemm.WgradBatch)
        C = x.shape[1]
        # packed: this step's compute-dtype filter (and its transpose) from ops/conv_igemm.WeightPack
        w = packed[0].view(weight.shape[0], C) if packed is not None else weight.reshape(weight.shape[0], C).to(cdtype)
        ctx.wt = packed[1] if packed is not None else None
        if _igemm.usable(x, weight, cdtype):
            # implicit-GEMM kernel: strided rows read in place, the BN statistics fused
            xc = x.to(cdtype)
            xc = xc if xc.is_contiguous(memory_format=torch.channels_last) else \
                xc.contiguous(memory_format=torch.channels_last)
            out, stats = _igemm.conv_fwd(xc, w.view(weight.shape[0], C, 1, 1), stride, 0, bn)
            N, _, H, W = out.shape
            ctx.save_for_backward(xc, w)
            ctx.lazy_rows = True
        else:
            if stride != 1:
                x = x[:, :, ::stride, ::stride]
            N, C, H, W = x.shape
            rows = _rows(x.to(cdtype))
            out = torch.mm(rows, w.t()).view(N, H, W, -1).permute(0, 3, 1, 2)
            stats = None
            ctx.save_for_backward(rows, w)
            ctx.lazy_rows = False
        ctx.geom = (N, C, H, W, stride, in_shape)
        ctx.n_out = 1 if bn is None else 2
        if bn is None:
            return out
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        # no zero tensor materialised for the statistics output's (absent) gradient
        ctx.set_materialize_grads(False)
        return out, stats

    @staticmethod
    def backward(ctx, dy, *_):
        saved, w = ctx.saved_tensors
        N, C, H, W, stride, in_shape = ctx.geom
        dyc = dy.to(w.dtype)
        if not dyc.is_contiguous(memory_format=torch.channels_last):
            dyc = dyc.contiguous(memory_format=torch.channels_last)
        dyr = _rows(dyc)
        dx = dw = None
        acc = None
        if ctx.tap is not None:
            acc, ctx.tap.grad = ctx.tap.grad, None
        K = w.shape[0]
        mine = (ctx.needs_input_grad[0] and _igemm.dgrad_1x1_here(K, H)
                and _igemm.usable(dyc, w.t().reshape(C, K, 1, 1), w.dtype))
        wt = None
        if mine:
            # dX = dY @ W as a 1x1 conv of dy with the transposed filter on the
            # implicit-GEMM kernel (accumulating onto a tapped residual gradient)
            wt = ctx.wt if ctx.wt is not None else w.t().contiguous().view(C, K, 1, 1)
        xt = ctx.xtap
        if ctx.needs_input_grad[0] and xt is not None:
            dx = Conv1x1Fn._shared_dgrad(xt, dyc, dyr, w, wt, (N, C, H, W), stride, in_shape)
        elif ctx.needs_input_grad[0] and stride != 1:
            # compact dY @ W, scattered into the zero-filled input gradient
            cpt = Conv1x1Fn._compact(dyc, dyr, w, wt, (N, C, H, W))
            n0, c0, h0, w0 = in_shape
            dx = torch.zeros((n0, h0, w0, c0), dtype=cpt.dtype, device=cpt.device).permute(0, 3, 1, 2)
            dx[:, :, ::stride, ::stride] = cpt
        elif ctx.needs_input_grad[0] and acc is not None:
            if acc.shape != (N, C, H, W) or not acc.is_contiguous(memory_format=torch.channels_last):
                raise RuntimeError("conv1x1: tapped gradient does not match the input")
            if mine and _igemm.dgrad_bn(dyc, wt, ctx.btap, acc) is not None:
                pass  # accumulated, with the producing BN's backward sums (ops/bn_nhwc.BNTap)
            elif mine:
                _igemm.conv_acc(dyc, wt, acc)
            else:
                _rows(acc).addmm_(dyr, w)  # acc <- acc + dY @ W (GEMM epilogue accumulate)
            dx = acc
        elif ctx.needs_input_grad[0]:
            dx = _igemm.dgrad_bn(dyc, wt, ctx.btap) if mine else None
            if dx is None:
                dx = Conv1x1Fn._compact(dyc, dyr, w, wt, (N, C, H, W))
        ctx.btap = None
        if ctx.needs_input_grad[1]:
            if ctx.lazy_rows and _igemm.usable(dyc, w.view(ctx.wshape), w.dtype):
                # implicit-GEMM weight gradient over the (strided) input pixels, fp32 out
                dw = _igemm.conv_wgrad(dyc, saved, tuple(ctx.wshape), stride, 0, ctx.wparam)
            else:
                # saved: the [P, C] rows, or (lazy) the unstrided input
                rows = _rows(saved[:, :, ::stride, ::stride] if stride != 1 else saved) if ctx.lazy_rows else saved
                dw = _wgrad(dyr, rows).view(ctx.wshape)
        ctx.wparam = None
        return dx, dw, None, None, None, None, None, None, None

    @staticmethod
    def _compact(dyc, dyr, w, wt, geom):
        """dY @ W over the output pixels: [N, C, H, W] channels_last (H, W of dy)."""
        N, C, H, W = geom
        if wt is not None:
            return _igemm.conv_fwd(dyc, wt, 1, 0)[0]
        return torch.mm(dyr, w).view(N, H, W, C).permute(0, 3, 1, 2)

    @staticmethod
    def _shared_dgrad(xt, dyc, dyr, w, wt, geom, stride, in_shape):
        other = xt.grad
        xt.grad = None
        if other is None:  # first of the pair: leave the (compact) product for the second
            xt.grad = (Conv1x1Fn._compact(dyc, dyr, w, wt, geom), stride)
            return None
        t, ostride = other
        if stride == 1 and ostride == 1:
            if wt is not None:
                _igemm.conv_acc(dyc, wt, t)
            else:
                _rows(t).addmm_(dyr, w)
            return t
        if stride == 1 and ostride == 2:
            if wt is not None and t.is_contiguous(memory_format=torch.channels_last):
                return _igemm.conv_fwd(dyc, wt, 1, 0, aux=t)[0]  # + t at the even pixels, in the epilogue
            dx = Conv1x1Fn._compact(dyc, dyr, w, None, geom)
            dx[:, :, ::2, ::2] += t
            return dx
        cpt = Conv1x1Fn._compact(dyc, dyr, w, wt, geom)
        if ostride == 1:  # the stride-1 conv ran first: its full gradient takes ours at the strided pixels
            t[:, :, ::stride, ::stride] += cpt
            return t
        n0, c0, h0, w0 = in_shape
        dx = torch.zeros((n0, h0, w0, c0), dtype=cpt.dtype, device=cpt.device).permute(0, 3, 1, 2)
        dx[:, :, ::stride, ::stride] = cpt
        dx[:, :, ::ostride, ::ostride] += t
        return dx


def conv1x1(x: torch.Tensor, weight: torch.Tensor, stride: int, cdtype: torch.dtype,
            tap: GradTap | None = None, bn=None, packed=None, xtap: GradTap | None = None, btap=None):
    """Bias-free 1x1 conv (stride 1 or 2) of ``x`` with the fp32 ``weight``; the
    output is a channels_last [N, Cout, H', W'] tensor in ``cdtype``.  ``tap``:
    see :class:`GradTap`.  With ``bn`` (the training BatchNorm that follows): returns
    (output, its statistics or None) -- ops/conv_igemm.py.  ``btap``: the
    ops/bn_nhwc.BNTap of the BatchNorm that produced ``x`` -- the data gradient then also
    takes that BN's backward sums."""
    return Conv1x1Fn.apply(x, weight, int(stride), cdtype, tap, bn, packed, xtap, btap)
