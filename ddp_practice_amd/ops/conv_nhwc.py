"""KxK convolution (3x3 / 7x7, bias-free) of a channels_last activation on MIOpen,
with the fp32-master / low-precision weight handling done once per call.

Through ``F.conv2d(x, weight.to(bf16))`` every conv costs three layout/cast
copies per step: fp32->bf16 cast, NCHW->NHWC weight copy (MIOpen wants the
weight in the activation's layout), and the bf16 NHWC weight gradient cast back
to an fp32 NCHW ``.grad``.  Here the forward does the cast and the layout change
in one copy and the backward one combined copy, straight into the fp32 gradient.
Used by the ResNet-50 stress model (models/resnet.py) for its 16 3x3 convs and
the 7x7 stem.
"""
from __future__ import annotations

import torch

from . import conv_igemm as _igemm

_CL = torch.channels_last


class ConvNHWCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, padding, cdtype: torch.dtype, bn=None):
        x = x if x.is_contiguous(memory_format=_CL) else x.contiguous(memory_format=_CL)
        w = torch.empty(weight.shape, dtype=cdtype, device=weight.device, memory_format=_CL)
        w.copy_(weight)  # fp32 NCHW -> cdtype NHWC in one kernel
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
        return out, stats

    @staticmethod
    def backward(ctx, dy, *_):
        x, w = ctx.saved_tensors
        stride, padding = ctx.conf
        dy = dy.to(w.dtype)
        dy = dy if dy.is_contiguous(memory_format=_CL) else dy.contiguous(memory_format=_CL)
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], False]
        dx, dw, _ = torch.ops.aten.convolution_backward(dy, x.to(w.dtype), w, None, stride, padding, [1, 1], False,
                                                        [0, 0], 1, mask)
        if dw is not None:
            g = torch.empty(dw.shape, dtype=ctx.wdtype, device=dw.device)
            g.copy_(dw)  # cdtype NHWC -> fp32 NCHW in one kernel
            dw = g
        return dx, dw, None, None, None, None


def conv_nhwc(x: torch.Tensor, weight: torch.Tensor, stride, padding, cdtype: torch.dtype, bn=None):
    """Bias-free conv of channels_last ``x`` with the fp32 ``weight`` in ``cdtype``.  With
    ``bn`` (the training BatchNorm that follows): returns (output, its statistics or None)."""
    return ConvNHWCFn.apply(x, weight, tuple(stride), tuple(padding), cdtype, bn)
