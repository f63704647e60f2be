"""Linear and CrossEntropyLoss on the native head kernels (csrc/kernels/head.hip).

reference: /root/reference/origin_main.py:24,30 (``nn.Linear(7*7*32, 10)``),
:63 / ddp_main.py:89 (``nn.CrossEntropyLoss()`` on the model output; under the
reference's AMP path the logits are fp16 because the loss is computed outside
the autocast region — here the logits keep the compute dtype likewise and the
loss math is fp32).
"""
from __future__ import annotations

import torch

from .._ext import load as _load_ext


def _H():
    return _load_ext().head


class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, cdtype):
        H = _H()
        x2 = x.reshape(-1, x.shape[-1]).to(cdtype).contiguous()
        out = torch.empty((x2.shape[0], w.shape[0]), dtype=cdtype, device=x.device)
        H.linear_fwd(x2, w, b, out)
        ctx.save_for_backward(x2, w)
        ctx.has_bias = b is not None
        ctx.in_shape = x.shape
        ctx.in_dtype = x.dtype
        return out.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dout):
        H = _H()
        x2, w = ctx.saved_tensors
        d2 = dout.reshape(-1, w.shape[0]).to(x2.dtype).contiguous()
        dw = torch.empty_like(w)
        db = torch.empty(w.shape[0], dtype=torch.float32, device=w.device) if ctx.has_bias else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x2)
        H.linear_bwd(d2, x2, w, dx, dw, db)
        if dx is not None:
            dx = dx.reshape(ctx.in_shape)
            if dx.dtype != ctx.in_dtype:
                dx = dx.to(ctx.in_dtype)
        return dx, dw, db, None


def linear(x, weight, bias=None, cdtype=None):
    if cdtype is None:
        from ..amp import compute_dtype

        cdtype = compute_dtype(x)
    return LinearFn.apply(x, weight, bias, cdtype)


class CrossEntropyFn(torch.autograd.Function):
    """mean-reduced cross entropy; forward also produces the analytic gradient."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing):
        H = _H()
        lg = logits.contiguous()
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        dlog = torch.empty(lg.shape, dtype=torch.float32, device=logits.device)
        H.ce_fwd(lg, target.contiguous(), loss.view(1), dlog, int(ignore_index), float(smoothing))
        ctx.save_for_backward(dlog)
        ctx.ldtype = lg.dtype
        return loss

    @staticmethod
    def backward(ctx, grad):
        (dlog,) = ctx.saved_tensors
        out = torch.empty(dlog.shape, dtype=ctx.ldtype, device=dlog.device)
        g = grad.reshape(1).to(torch.float32).contiguous()
        _H().ce_bwd(dlog, g, out)
        return out, None, None, None


def cross_entropy(logits, target, ignore_index=-100, label_smoothing=0.0):
    if logits.dim() != 2:
        raise ValueError("native cross_entropy expects [B, C] logits")
    return CrossEntropyFn.apply(logits, target, ignore_index, label_smoothing)


def accuracy_(logits, target, counters):
    """counters[0] += B; counters[1] += #correct  (device-side, no sync)."""
    _H().accuracy(logits.contiguous(), target.contiguous(), counters)
