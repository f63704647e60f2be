"""Linear and CrossEntropyLoss on the native head kernels (csrc/kernels/head.hip).

reference: /root/reference/origin_main.py:24,30 (``nn.Linear(7*7*32, 10)``),
:63 / ddp_main.py:89 (``nn.CrossEntropyLoss()`` on the model output; under the
reference's AMP path the logits are fp16 because the loss is computed outside
the autocast region — here the logits keep the compute dtype likewise and the
loss math is fp32).
"""
from __future__ import annotations

import os

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


class _ScaledSeed:
    """Token shared by a native CE loss and the GradScaler that scales it.

    When the scaler's fast backward seeds the loss with exactly its scale
    tensor, the CE backward returns the gradient the forward kernel already
    wrote for the scaled loss (d(scale*loss)/dlogits, in the logits dtype): the
    ``loss * scale`` multiply and the CE backward launch disappear from the
    step (amp/grad_scaler.py)."""

    __slots__ = ("scale", "seeded")

    def __init__(self, scale):
        self.scale = scale
        self.seeded = False


class CrossEntropyFn(torch.autograd.Function):
    """mean-reduced cross entropy; forward also produces the analytic gradient."""

    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing, scale):
        H = _H()
        lg = logits.contiguous()
        buf = torch.empty(2, dtype=torch.float32, device=logits.device)
        dlog = torch.empty(lg.shape, dtype=torch.float32, device=logits.device)
        dls = torch.empty_like(lg) if scale is not None else None
        H.ce_fwd(lg, target.contiguous(), buf, dlog, int(ignore_index), float(smoothing), scale, dls)
        ctx.save_for_backward(dlog)
        ctx.ldtype = lg.dtype
        ctx.token = _ScaledSeed(scale) if scale is not None else None
        ctx.dls = dls
        ctx.scaled = buf[1] if scale is not None else None
        return buf[0]

    @staticmethod
    def backward(ctx, grad):
        tok = ctx.token
        if tok is not None and tok.seeded:
            # grad is the scaler's scale tensor: the forward already wrote dlog * scale
            return ctx.dls, None, None, None, None
        (dlog,) = ctx.saved_tensors
        out = torch.empty(dlog.shape, dtype=ctx.ldtype, device=dlog.device)
        g = grad.reshape(1).to(torch.float32).contiguous()
        _H().ce_bwd(dlog, g, out)
        return out, None, None, None, None


class PrecomputedCEFn(torch.autograd.Function):
    """The loss a fused head launch already produced (ops/convnet_fused.py PreCE): no
    launch forward; backward as CrossEntropyFn (the scaled gradient when seeded)."""

    @staticmethod
    def forward(ctx, logits, pre):
        ctx.pre = pre
        ctx.ldtype = logits.dtype
        ctx.token = _ScaledSeed(pre.scale) if pre.scale is not None else None
        ctx.scaled = pre.loss[1] if pre.scale is not None else None
        return pre.loss[0]

    @staticmethod
    def backward(ctx, grad):
        tok = ctx.token
        if tok is not None and tok.seeded:
            return ctx.pre.dls, None
        dlog = ctx.pre.dlog
        out = torch.empty(dlog.shape, dtype=ctx.ldtype, device=dlog.device)
        _H().ce_bwd(dlog, grad.reshape(1).to(torch.float32).contiguous(), out)
        return out, None


_UNIT: dict = {}
_UNIT_SEED = os.environ.get("DPA_UNIT_SEED", "1") != "0"  # 0: no unit-seed speculation (A/B)


def unit_scale(device: torch.device) -> torch.Tensor:
    """A persistent device ``[1.0]``: the "scale" a loss is pre-differentiated with when no
    GradScaler is active (fp32 training, /root/reference/origin_main.py:57-66)."""
    t = _UNIT.get(device)
    if t is None:
        t = _UNIT[device] = torch.ones(1, dtype=torch.float32, device=device)
    return t


def seed_scale(device: torch.device):
    """The scale a native loss kernel pre-differentiates for: the active GradScaler's (its
    scaled backward seeds the loss with it), else -- on a HIP device -- the unit tensor,
    which the loss's own ``backward()`` then seeds with (no ones() fill, no CE backward
    launch; the fused ConvNet head also runs its backward rows in the forward launch).
    None on CPU or with DPA_UNIT_SEED=0."""
    from ..amp.grad_scaler import active_scale

    s = active_scale(device)
    if s is None and _UNIT_SEED and device.type == "cuda":
        s = unit_scale(device)
    return s


class _LossViewFn(torch.autograd.Function):
    """The loss as a view of itself (no launch): the tensor a unit-seeded loss is handed out
    as, so the ``backward`` override stored on it can hold the real loss strongly."""

    @staticmethod
    def forward(ctx, loss):
        return loss.view_as(loss)

    @staticmethod
    def backward(ctx, grad):
        return grad


def _unit_seeded(loss: torch.Tensor, node, unit: torch.Tensor) -> torch.Tensor:
    """``loss.backward()`` of an unscaled native CE loss: seed with the unit tensor the loss
    was pre-differentiated for (grad 1, as autograd's implicit seed) and let the CE node hand
    back the gradient its forward already wrote; any other call goes through torch.

    Returns the tensor to hand out.  The override lives on a view of the loss and holds the
    loss itself: ``f(x).backward()`` drops the last reference to the returned temporary
    before the bound call runs (so a weak reference would be dead), and a strong reference
    from the loss's own attribute would be a cycle keeping the step's autograd graph alive
    until the cyclic GC (as in amp/grad_scaler.py's scaled loss)."""
    from ..amp.grad_scaler import _seeded_backward

    seed = unit.view(())
    out = _LossViewFn.apply(loss)

    def _backward(gradient=None, retain_graph=None, create_graph=False, inputs=None):
        if gradient is None and not create_graph:
            node.token.seeded = True
            try:
                _seeded_backward(loss, seed, retain_graph, inputs)
            finally:
                node.token.seeded = False
        else:
            torch.Tensor.backward(loss, gradient, retain_graph, create_graph, inputs)

    out.backward = _backward
    return out


def cross_entropy(logits, target, ignore_index=-100, label_smoothing=0.0):
    if logits.dim() != 2:
        raise ValueError("native cross_entropy expects [B, C] logits")
    scale = seed_scale(logits.device) if logits.requires_grad else None
    pre = getattr(logits, "_dpa_pre_ce", None)
    if (pre is not None and pre.target is target and pre.ignore_index == ignore_index
            and pre.smoothing == label_smoothing and pre.scale is scale and logits.requires_grad):
        loss = PrecomputedCEFn.apply(logits, pre)
    else:
        loss = CrossEntropyFn.apply(logits, target, ignore_index, label_smoothing, scale)
    if scale is not None and loss.grad_fn is not None:
        node = loss.grad_fn
        if scale is _UNIT.get(logits.device):
            loss = _unit_seeded(loss, node, scale)
        else:
            # the token / pre-scaled value travel with the loss tensor to GradScaler.scale
            loss._dpa_ce = (node, scale)
    return loss


def accuracy_(logits, target, counters):
    """counters[0] += B; counters[1] += #correct  (device-side, no sync)."""
    _H().accuracy(logits.contiguous(), target.contiguous(), counters)
