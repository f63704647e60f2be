"""SyncBatchNorm: batch statistics over all ranks.

Semantics of torch.nn.SyncBatchNorm (torch/nn/modules/batchnorm.py:790-901,
torch/nn/modules/_functions.py:10-205): training forward normalises with the
global mean / biased variance, updates running stats with the global unbiased
variance (momentum 0.1, eps 1e-5); backward all-reduces sum(dy) and
sum(dy*(x-mean)); eval (or world size 1) is plain BatchNorm.

Structure here: the statistics are plain sums (shifted by the running mean,
which is identical on every rank) so the forward needs ONE all-reduce of 2C+1
floats (sum, sum of squares, count) instead of all_gather(mean, invstd, count)
+ a device->host mask; ranks with an empty batch contribute count 0 without a
host sync.  Inside the fused ConvNet block (ops/convblock.py) the same
collectives run between the fused kernels; this module's own forward is the
generic path for any other network.

reference: /root/reference/ddp_main.py:120 (``nn.SyncBatchNorm.convert_sync_batchnorm``).
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn.modules.batchnorm import _BatchNorm

from . import comm as _comm


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, eps, comm):
        C = x.shape[1]
        xf = x.float()
        red = [0] + list(range(2, x.dim()))
        shift = running_mean.detach().float().view(1, C, *([1] * (x.dim() - 2)))
        d = xf - shift
        n_local = float(x.numel() // C)
        stats = torch.cat([d.sum(red), (d * d).sum(red), torch.full((1,), n_local, device=x.device)])
        if comm is not None and comm.active:
            comm.all_reduce_(stats)
        n = stats[2 * C]
        m1 = stats[:C] / n
        mean = running_mean.float() + m1
        var = (stats[C:2 * C] / n - m1 * m1).clamp_min(0)
        invstd = torch.rsqrt(var + eps)
        with torch.no_grad():
            nbt.add_(1)
            # cumulative average (momentum=None) stays on the device: no host sync
            mom = momentum if momentum is not None else nbt.reciprocal().float()
            running_mean.mul_(1 - mom).add_(mean * mom)
            running_var.mul_(1 - mom).add_(var * (n / (n - 1).clamp_min(1)) * mom)
        shp = (1, C) + (1,) * (x.dim() - 2)
        xhat = (xf - mean.view(shp)) * invstd.view(shp)
        w = weight.float().view(shp) if weight is not None else 1.0
        b = bias.float().view(shp) if bias is not None else 0.0
        y = (xhat * w + b).to(x.dtype)
        ctx.save_for_backward(xhat, invstd, weight, n.reshape(1))
        ctx.comm = comm
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        xhat, invstd, weight, n = ctx.saved_tensors
        C = xhat.shape[1]
        red = [0] + list(range(2, xhat.dim()))
        shp = (1, C) + (1,) * (xhat.dim() - 2)
        dyf = dy.float()
        s1 = dyf.sum(red)
        s2 = (dyf * xhat).sum(red)
        sums = torch.cat([s1, s2])
        comm = ctx.comm
        g = comm.all_reduce(sums) if (comm is not None and comm.active) else sums
        w = weight.float() if weight is not None else torch.ones(C, device=dy.device)
        k1 = (g[:C] / n).view(shp)
        k2 = (g[C:] / n).view(shp)
        dx = (w * invstd).view(shp) * (dyf - k1 - xhat * k2)
        return (dx.to(dy.dtype), s2 if ctx.has_w else None, s1 if ctx.has_b else None, None, None, None, None,
                None, None)


class _NativeBN:
    """bn_act(relu=False) with the module's buffers; gamma / beta passed explicitly so
    a non-affine module can use constant ones / zeros."""

    @staticmethod
    def apply(x, w, b, mod, comm):
        from ..ops.bn_nhwc import BNActFn

        return BNActFn.apply(x, w, b, None, mod.running_mean, mod.running_var, mod.num_batches_tracked,
                             mod.momentum, mod.eps, True, False, comm, None, None)


class SyncBatchNorm(_BatchNorm):
    """Drop-in for torch.nn.SyncBatchNorm (same parameters / buffers / state_dict)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device=device, dtype=dtype)
        self.process_group = process_group

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError(f"expected at least 2D input (got {input.dim()}D input)")

    @property
    def comm(self):
        pg = self.process_group
        if isinstance(pg, _comm.Communicator):
            return pg
        return _comm.default_comm()

    def _native(self, x) -> bool:
        """Device input in training: the channels_last kernels of ops/bn_nhwc.py
        (statistics, one all-reduce of 2C+1 floats, apply; backward sums, one all-reduce,
        elementwise) instead of the torch-op path below.  Any rank >= 2 (BatchNorm1d's
        [N, C] / [N, C, L], BatchNorm3d's [N, C, D, H, W]) runs as the 4-D view
        [N, C, prod(rest), 1]: the per-channel statistics are the same reduction."""
        return (x.is_cuda and x.dim() >= 2 and x.numel() > 0 and self.training and self.track_running_stats
                and x.dtype in (torch.float32, torch.float16, torch.bfloat16))

    def forward(self, x):
        self._check_input_dim(x)
        comm = self.comm
        if self._native(x):
            from ..ops.bn_nhwc import bn_act

            C = x.shape[1]
            if not self.affine:  # the kernels take gamma / beta: identity affine
                if getattr(self, "_ones", None) is None or self._ones.device != x.device:
                    self._ones = torch.ones(C, device=x.device)
                    self._zeros = torch.zeros(C, device=x.device)
            w = self.weight if self.affine else self._ones
            b = self.bias if self.affine else self._zeros
            if x.dim() != 4:
                x4 = x.reshape(x.shape[0], C, -1, 1)
                return _NativeBN.apply(x4, w, b, self, comm if comm.active else None).contiguous().view(x.shape)
            y = _NativeBN.apply(x, w, b, self, comm if comm.active else None)
            return y if x.is_contiguous(memory_format=torch.channels_last) else y.contiguous()
        if not self.training or not self.track_running_stats or not comm.active:
            if self.training and self.track_running_stats:
                # the same shifted-sum path, world of one
                return _SyncBNFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                                       self.num_batches_tracked, self.momentum, self.eps, None)
            return nn.functional.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias,
                                            self.training or not self.track_running_stats,
                                            0.0 if self.momentum is None else self.momentum, self.eps)
        return _SyncBNFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                               self.num_batches_tracked, self.momentum, self.eps, comm)


def convert_sync_batchnorm(module: nn.Module, process_group=None) -> nn.Module:
    """Replace every BatchNorm*D with SyncBatchNorm sharing its parameters and buffers
    (torch/nn/modules/batchnorm.py:842-901)."""
    out = module
    if isinstance(module, _BatchNorm) and not isinstance(module, SyncBatchNorm):
        out = SyncBatchNorm(module.num_features, module.eps, module.momentum, module.affine,
                            module.track_running_stats, process_group)
        if module.affine:
            with torch.no_grad():
                out.weight = module.weight
                out.bias = module.bias
        out.running_mean = module.running_mean
        out.running_var = module.running_var
        out.num_batches_tracked = module.num_batches_tracked
        out.training = module.training
        if hasattr(module, "qconfig"):
            out.qconfig = module.qconfig
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, process_group))
    del module
    return out
