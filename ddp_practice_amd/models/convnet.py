"""The reference ConvNet, with the same module tree / state_dict keys.

reference: /root/reference/origin_main.py:9-31 and ddp_main.py:13-36:
    layer1 = Conv2d(1,16,5,p=2) -> BatchNorm2d(16) -> ReLU -> MaxPool2d(2,2)
    layer2 = Conv2d(16,32,5,p=2) -> BatchNorm2d(32) -> ReLU -> MaxPool2d(2,2)
    fc     = Linear(7*7*32, num_classes)
29,034 parameters, 16 state_dict entries ("layer1.0.weight" ... "fc.bias").

On a HIP device the whole network runs as ONE fused op (3 launches forward,
7 backward: ops/convnet_fused.py); ``fused="layer"`` runs each ``layerN`` as
one op (2 launches forward, 4-5 backward: ops/convblock.py) and ``fc`` on the
MFMA head kernel; ``fused=False`` runs the torch modules.  When a
``SyncBatchNorm`` from this package replaces the BatchNorm (see
``parallel.sync_bn.convert_sync_batchnorm``) the fused op all-reduces its
statistics through that module's communicator.  On CPU the plain PyTorch
modules run (the reference's semantics; used by the plumbing config and the
CPU test tier).

``amp_dtype`` reproduces the reference's ``autocast`` *inside* ``forward``
(ddp_main.py:31): ``None`` = fp32 (origin_main.py), ``torch.float16`` = the
reference's AMP default, ``torch.bfloat16`` = this framework's AMP default.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from ..amp import autocast, compute_dtype


class ConvNet(nn.Module):
    def __init__(self, num_classes: int = 10, amp_dtype: torch.dtype | None = None, fused: bool | str = True):
        super().__init__()
        self.layer1 = nn.Sequential(
            nn.Conv2d(1, 16, kernel_size=5, stride=1, padding=2),
            nn.BatchNorm2d(16),
            nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2),
        )
        self.layer2 = nn.Sequential(
            nn.Conv2d(16, 32, kernel_size=5, stride=1, padding=2),
            nn.BatchNorm2d(32),
            nn.ReLU(),
            nn.MaxPool2d(kernel_size=2, stride=2),
        )
        self.fc = nn.Linear(7 * 7 * 32, num_classes)
        self.amp_dtype = amp_dtype
        self.fused = fused

    # ---------------------------------------------------------------- native
    def _native_ok(self, x: torch.Tensor) -> bool:
        if not (self.fused and x.is_cuda):
            return False
        from ..ops.convblock import supported

        return supported(x, self.layer1[0]) and self.layer1[1].track_running_stats \
            and self.layer2[1].track_running_stats

    @staticmethod
    def _comm_of(bn: nn.Module):
        if not bn.training:
            return None
        if isinstance(bn, nn.SyncBatchNorm):  # torch's SyncBN: use the package communicator
            from ..parallel.comm import default_comm

            return default_comm()
        return getattr(bn, "comm", None)

    @classmethod
    def _block(cls, seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
        from ..ops.convblock import conv_block

        return conv_block(x, seq[0], seq[1], comm=cls._comm_of(seq[1]))

    def _forward_native(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops import convnet_fused
        from ..ops.head import linear

        if self.fused != "layer" and convnet_fused.supported(self, x):
            c1, c2 = self._comm_of(self.layer1[1]), self._comm_of(self.layer2[1])
            if c1 is c2:
                return convnet_fused.convnet_forward(self, x, comm=c1)
        out = self._block(self.layer1, x)
        out = self._block(self.layer2, out)
        out = out.reshape(out.size(0), -1)
        return linear(out, self.fc.weight, self.fc.bias)

    def _forward_torch(self, x: torch.Tensor) -> torch.Tensor:
        out = self.layer1(x)
        out = self.layer2(out)
        out = out.reshape(out.size(0), -1)
        return self.fc(out)

    def accepts_deferred_batch(self, x: torch.Tensor) -> bool:
        """The fused forward performs a deferred batch gather (data/loader.py) itself:
        conv1 reads the HBM-resident dataset directly."""
        if not (self.fused is True and x.is_cuda):
            return False
        from ..ops import convnet_fused

        want = self.amp_dtype if self.amp_dtype is not None else torch.float32
        return x.dtype == want and x.is_contiguous() and self._native_ok(x) and convnet_fused.supported(self, x)

    def set_slab_sink(self, optimizer) -> bool:
        """Let ``optimizer`` (optim.SGD) sum the conv1 weight-gradient partial rows inside
        its fused AMP step instead of a separate column-sum launch (ops/convnet_fused.py).
        Under DDP only through ``DistributedDataParallel.set_slab_sink`` (a reducer that
        packs gradients reads ``.grad`` in its hooks); engine.TrainLoop enables it.
        Returns whether it was enabled."""
        if not hasattr(optimizer, "defer_slab") or os.environ.get("DPA_SLAB_SINK", "1") == "0":
            return False
        self._dpa_slab_sink = optimizer
        return True

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if getattr(x, "_dpa_gather", None) is not None and not (self.training and self.accepts_deferred_batch(x)):
            from ..data.loader import flush_pending

            flush_pending(x)
        native = self._native_ok(x)
        fwd = self._forward_native if native else self._forward_torch
        if self.amp_dtype is not None:
            with autocast(dtype=self.amp_dtype, device_type="cuda" if x.is_cuda else "cpu"):
                if native and x.dtype != compute_dtype(x):
                    x = x.to(compute_dtype(x))
                return fwd(x)
        return fwd(x)
