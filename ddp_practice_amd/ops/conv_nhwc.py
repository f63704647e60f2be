"""KxK convolution (3x3 / 7x7, bias-free) of a channels_last activation on MIOpen,
with the fp32-master / low-precision weight handling done once per call.

Through ``F.conv2d(x, weight.to(bf16))`` every conv costs three layout/cast
copies per step: fp32->bf16 cast, NCHW->NHWC weight copy (MIOpen wants the
weight in the activation's layout), and the bf16 NHWC weight gradient cast back
to an fp32 NCHW ``.grad``.  Here the forward does the cast and the layout change
in one copy and the backward one combined copy, straight into the fp32 gradient.
Used by the ResNet-50 stress model (models/resnet.py) for its 16 3x3 convs: the
hand-written implicit-GEMM kernel (ops/conv_igemm.py) takes every forward, weight
gradient and data gradient (stride 1, and stride 2 as four parity sub-convolutions);
MIOpen remains the fallback for shapes outside it.  The 7x7 stem has its own mode
(ops/conv_igemm.stem_conv).
"""
from __future__ import annotations

import torch

from . import conv_igemm as _igemm

_CL = torch.channels_last


class ConvNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding, cdtype: torch.dtype, bn=None, packed=None, btap=None):
        x = x if x.is_contiguous(memory_format=_CL) else x.contiguous(memory_format=_CL)
        if packed is not None:  # this step's filters from ops/conv_igemm.WeightPack
            w = packed[0]
        else:
            w = torch.empty(weight.shape, dtype=cdtype, device=weight.device, memory_format=_CL)
            w.copy_(weight)  # fp32 NCHW -> cdtype NHWC in one kernel
        ctx.wt = packed[1] if packed is not None else None
        ctx.btap = btap  # ops/bn_nhwc.BNTap of the BN that produced x (stride-1 dgrad takes its sums)
        ctx.wparam = weight  # the leaf parameter (ops/conv_igemm.WgradBatch)
        stats = None
        if (_igemm.usable(x, weight, cdtype) and stride[0] == stride[1] and padding[0] == padding[1]):
            # hand-written implicit GEMM (+ the next BN's statistics in its epilogue)
            xc = x.to(cdtype)
            xc = xc if xc.is_contiguous(memory_format=_CL) else xc.contiguous(memory_format=_CL)
            out, stats = _igemm.conv_fwd(xc, w, stride[0], padding[0], bn)
        else:
            out = torch.ops.aten.convolution(x.to(cdtype), w, None, stride, padding, [1, 1], False, [0, 0], 1)
            out = out if out.is_contiguous(memory_format=_CL) else out.contiguous(memory_format=_CL)
        ctx.save_for_backward(x, w)
        ctx.conf = (list(stride), list(padding))
        ctx.wdtype = weight.dtype
        if bn is None:
            return out
        if stats is not None:
            ctx.mark_non_differentiable(stats)
        # no zero tensor materialised for the statistics output's (absent) gradient
        ctx.set_materialize_grads(False)
        return out, stats

    @staticmethod
    def backward(ctx, dy, *_):
        x, w = ctx.saved_tensors
        stride, padding = ctx.conf
        dy = dy.to(w.dtype)
        dy = dy if dy.is_contiguous(memory_format=_CL) else dy.contiguous(memory_format=_CL)
        dx = None
        if (ctx.needs_input_grad[0] and stride == [1, 1] and padding[0] == padding[1]
                and w.shape[2] == w.shape[3] and _igemm.usable(dy, w.transpose(0, 1), w.dtype)):
            # stride-1 data gradient = a forward conv of dy with the flipped, transposed
            # filter on the implicit-GEMM kernel (pad R-1-p)
            R = w.shape[2]
            wt = ctx.wt
            if wt is None:
                wt = torch.empty((w.shape[1], w.shape[0], R, R), dtype=w.dtype, device=w.device, memory_format=_CL)
                wt.copy_(w.flip(2, 3).transpose(0, 1))
            dx = _igemm.dgrad_bn(dy, wt, ctx.btap, None, R - 1 - padding[0])
            if dx is None:
                dx, _ = _igemm.conv_fwd(dy, wt, 1, R - 1 - padding[0])
        elif (ctx.needs_input_grad[0] and stride == [2, 2] and padding == [1, 1] and tuple(w.shape[2:]) == (3, 3)
              and _igemm.usable(dy, w.transpose(0, 1), w.dtype)):
            # stride-2 data gradient: four output-parity sub-convolutions in one launch
            wt = ctx.wt
            if wt is None:
                wt = torch.empty((w.shape[1], w.shape[0], 3, 3), dtype=w.dtype, device=w.device, memory_format=_CL)
                wt.copy_(w.flip(2, 3).transpose(0, 1))
            dx = _igemm.dgrad_s2(dy, wt, tuple(x.shape[2:]))
        dw = None
        xc = x.to(w.dtype)
        if (ctx.needs_input_grad[1] and ctx.wdtype == torch.float32 and stride[0] == stride[1]
                and padding[0] == padding[1] and _igemm.usable(dy, w, w.dtype)):
            # weight gradient on the implicit-GEMM kernel, written as the fp32 OIHW .grad
            dw = _igemm.conv_wgrad(dy, xc, tuple(w.shape), stride[0], padding[0], ctx.wparam)
        mask = [ctx.needs_input_grad[0] and dx is None, ctx.needs_input_grad[1] and dw is None, False]
        if mask[0] or mask[1]:
            dx2, dw2, _ = torch.ops.aten.convolution_backward(dy, xc, w, None, stride, padding, [1, 1], False,
                                                              [0, 0], 1, mask)
            if dx is None:
                dx = dx2
            if dw2 is not None:
                dw = torch.empty(dw2.shape, dtype=ctx.wdtype, device=dw2.device)
                dw.copy_(dw2)  # cdtype NHWC -> fp32 NCHW in one kernel
        ctx.btap = None
        ctx.wparam = None
        return dx, dw, None, None, None, None, None, None


def conv_nhwc(x: torch.Tensor, weight: torch.Tensor, stride, padding, cdtype: torch.dtype, bn=None, packed=None,
              btap=None):
    """Bias-free conv of channels_last ``x`` with the fp32 ``weight`` in ``cdtype``.  With
    ``bn`` (the training BatchNorm that follows): returns (output, its statistics or None).
    ``btap``: the ops/bn_nhwc.BNTap of the BN that produced ``x`` (a stride-1 data gradient
    then also takes that BN's backward sums)."""
    return ConvNHWCFn.apply(x, weight, tuple(stride), tuple(padding), cdtype, bn, packed, btap)
