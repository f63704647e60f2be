"""Fused Conv5x5 -> BatchNorm2d/SyncBatchNorm -> ReLU -> MaxPool2d(2,2) block.

Autograd wrapper around the HIP kernels in ``csrc/kernels/convblock.hip``.
One block = 2 launches forward (conv+partial stats, bn+relu+pool) and 5
backward (reduce, elemt, wgrad, slab-reduce, dgrad), no zero-fill launches,
instead of the ~12 ATen/MIOpen kernels plus host syncs of the reference
(/root/reference/ddp_main.py:16-27 under SyncBN, torch/nn/modules/_functions.py:10-205).

SyncBN: when ``comm`` is given and its world size is > 1 the per-workgroup
forward partial sums (sum, sum of squares, count per channel) and the
per-split backward sums are all-reduced through the communicator — one
collective each, no device->host mask (counts travel in the buffer).
"""
from __future__ import annotations

import torch

from .._ext import load as _load_ext


def _C():
    return _load_ext().convblock


def supported(x: torch.Tensor, conv: torch.nn.Conv2d) -> bool:
    if not x.is_cuda or x.dim() != 4:
        return False
    if conv.kernel_size != (5, 5) or conv.stride != (1, 1) or conv.padding != (2, 2) or conv.groups != 1 \
            or conv.dilation != (1, 1) or conv.bias is None:
        return False
    return _C().supported(int(x.shape[1]), int(conv.out_channels), int(x.shape[2]), int(x.shape[3]))


class ConvBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, gamma, beta, running_mean, running_var, nbt, training, momentum, eps, comm,
                cdtype):
        C = _C()
        x = x.to(cdtype).contiguous()
        B, cin, H, W = x.shape
        cout = w.shape[0]
        dev = x.device
        y = torch.empty((B, cout, H, W), dtype=cdtype, device=dev)
        p = torch.empty((B, cout, H // 2, W // 2), dtype=cdtype, device=dev)
        idx = torch.empty((B, cout, H // 2, W // 2), dtype=torch.uint8, device=dev)
        fstats = torch.empty(C.stats_len(cout), dtype=torch.float32, device=dev)
        mom = -1.0 if momentum is None else float(momentum)
        if training:
            fslab = torch.empty(C.fwd_rows(cin, cout, H, W, B) * C.fslab_row(cout), dtype=torch.float32, device=dev)
            C.conv_fwd(x, w, b, y, fslab, fstats, running_mean)
            if comm is not None and comm.active:
                comm.all_reduce_(fslab)
            C.bn_relu_pool(y, fslab, fstats, gamma, beta, running_mean, running_var, nbt, mom, float(eps), True, p,
                           idx)
        else:
            C.conv_fwd(x, w, b, y)
            C.bn_relu_pool(y, None, fstats, gamma, beta, running_mean, running_var, nbt, mom, float(eps), False, p,
                           idx)
        ctx.save_for_backward(x, w, gamma, y, p, idx, fstats)
        ctx.eps = float(eps)
        ctx.comm = comm
        ctx.training = training
        ctx.mark_non_differentiable(idx)
        return p

    @staticmethod
    def backward(ctx, dp):
        if not ctx.training:
            raise RuntimeError("ConvBlockFn backward in eval mode is not supported (use train() for training)")
        C = _C()
        x, w, gamma, y, p, idx, fstats = ctx.saved_tensors
        dp = dp.to(y.dtype).contiguous()
        B, cout, H, W = y.shape
        cin = w.shape[1]
        dev = y.device
        nw = w.numel()
        nsplit = C.bwd_split(B)
        bslab = torch.empty(nsplit * 2 * cout, dtype=torch.float32, device=dev)
        C.bwd_reduce(dp, p, idx, y, fstats, ctx.eps, bslab)
        comm = ctx.comm
        if comm is not None and comm.active:
            gslab = comm.all_reduce(bslab)  # out of place: local sums stay the BN param grads
        else:
            gslab = bslab
        dy = torch.empty_like(y)
        C.bwd_elemt(dp, p, idx, y, fstats, gslab, gamma, ctx.eps, dy)
        wslab = torch.empty(C.wgrad_rows(cin, cout, H, W, B) * (nw + cout), dtype=torch.float32, device=dev)
        C.conv_wgrad(x, dy, wslab)
        # one output buffer: dW | db | dbeta | dgamma (views handed to autograd)
        out = torch.empty(nw + cout + 2 * cout, dtype=torch.float32, device=dev)
        C.slab_reduce(wslab, nw + cout, out.narrow(0, 0, nw + cout), bslab, 2 * cout, out.narrow(0, nw + cout, 2 * cout))
        dw = out.narrow(0, 0, nw).view_as(w)
        db = out.narrow(0, nw, cout)
        dbeta = out.narrow(0, nw + cout, cout)
        dgamma = out.narrow(0, nw + 2 * cout, cout)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((B, cin, H, W), dtype=y.dtype, device=dev)
            C.conv_dgrad(dy, w, dx)
        return dx, dw, db, dgamma, dbeta, None, None, None, None, None, None, None, None


def conv_block(x, conv, bn, comm=None, cdtype=None):
    """Run conv -> bn -> relu -> maxpool with the fused kernels.

    ``conv``: nn.Conv2d(5x5, pad 2, bias), ``bn``: BatchNorm2d-like module
    (weight, bias, running_mean, running_var, num_batches_tracked, momentum, eps).
    """
    if cdtype is None:
        from ..amp import compute_dtype

        cdtype = compute_dtype(x)
    training = bn.training
    if training and not bn.track_running_stats:
        raise NotImplementedError("fused block needs track_running_stats=True")
    return ConvBlockFn.apply(x, conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                             bn.num_batches_tracked, training, bn.momentum, bn.eps, comm, cdtype)
