"""Fused Conv5x5 -> BatchNorm2d/SyncBatchNorm -> ReLU -> MaxPool2d(2,2) block.

Autograd wrapper around the HIP kernels in ``csrc/kernels/convblock.hip``.
One block = 2 launches forward (conv+stats, bn+relu+pool) and 4 backward
(reduce, elemt, wgrad, dgrad) + 1 zero-fill, instead of the ~12 ATen/MIOpen
kernels plus host syncs of the reference
(/root/reference/ddp_main.py:16-27 under SyncBN, torch/nn/modules/_functions.py:10-205).

SyncBN: when ``comm`` is given and its world size is > 1 the 2C+1 forward
statistics (sum, sum of squares, count) and the 2C backward sums are
all-reduced through the communicator — 1 collective each, no
device->host mask (the count is carried in the buffer).
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
        B, _, H, W = x.shape
        cout = w.shape[0]
        y = torch.empty((B, cout, H, W), dtype=cdtype, device=x.device)
        p = torch.empty((B, cout, H // 2, W // 2), dtype=cdtype, device=x.device)
        idx = torch.empty((B, cout, H // 2, W // 2), dtype=torch.uint8, device=x.device)
        if training:
            stats = torch.zeros(C.stats_len(cout), dtype=torch.float32, device=x.device)
            C.conv_fwd(x, w, b, y, stats, running_mean)
            if comm is not None and comm.world_size > 1:
                comm.all_reduce_(stats.narrow(0, 0, 2 * cout + 1))
        else:
            stats = torch.empty(0, dtype=torch.float32, device=x.device)
            C.conv_fwd(x, w, b, y)
        mom = -1.0 if momentum is None else float(momentum)
        C.bn_relu_pool(y, stats, gamma, beta, running_mean, running_var, nbt, mom, float(eps), bool(training), p,
                       idx)
        ctx.save_for_backward(x, w, gamma, y, p, idx, stats)
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
        x, w, gamma, y, p, idx, stats = ctx.saved_tensors
        dp = dp.to(y.dtype).contiguous()
        cout, cin = w.shape[0], w.shape[1]
        nw, nb = w.numel(), cout
        # one zero-filled buffer: dW | db | sum(dy) (=dbeta) | sum(dy*xhat) (=dgamma)
        buf = torch.zeros(nw + nb + 2 * cout, dtype=torch.float32, device=y.device)
        dw = buf.narrow(0, 0, nw).view_as(w)
        db = buf.narrow(0, nw, nb)
        sums = buf.narrow(0, nw + nb, 2 * cout)
        C.bwd_reduce(dp, p, idx, y, stats, ctx.eps, sums)
        comm = ctx.comm
        if comm is not None and comm.world_size > 1:
            gsums = comm.all_reduce(sums)  # out of place: local sums stay the BN param grads
        else:
            gsums = sums
        dy = torch.empty_like(y)
        C.bwd_elemt(dp, p, idx, y, stats, gsums, gamma, ctx.eps, dy)
        C.conv_wgrad(x, dy, dw, db)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((y.shape[0], cin, y.shape[2], y.shape[3]), dtype=y.dtype, device=y.device)
            C.conv_dgrad(dy, w, dx)
        dbeta = sums.narrow(0, 0, cout)
        dgamma = sums.narrow(0, cout, cout)
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


def conv_block_reference(x, conv, bn, comm=None):
    """Pure-PyTorch semantics of the block (CPU path / numerics oracle)."""
    import torch.nn.functional as F

    y = F.conv2d(x, conv.weight.to(x.dtype), conv.bias.to(x.dtype), stride=1, padding=2)
    y = bn(y) if comm is None else bn(y)
    return F.max_pool2d(F.relu(y), 2, 2)
