"""Layer modules with native HIP forward/backward on a GPU.

Drop-ins for the torch.nn modules the reference uses
(/root/reference/origin_main.py:12-24,86): same constructor arguments,
parameters and state_dict keys; on a HIP device ``forward`` runs this
package's kernels, on CPU the torch implementation.
"""
from __future__ import annotations

import torch
import torch.nn as _tnn

from ..parallel.sync_bn import SyncBatchNorm, convert_sync_batchnorm  # noqa: F401


class CrossEntropyLoss(_tnn.CrossEntropyLoss):
    """Mean-reduced CE over [B, C] logits on the fused HIP kernel (log-softmax +
    NLL + analytic gradient in one pass); other configurations use torch."""

    def forward(self, input, target):
        if (input.is_cuda and input.dim() == 2 and self.weight is None and self.reduction == "mean"
                and target.dtype == torch.int64 and target.dim() == 1):
            from ..ops.head import cross_entropy

            return cross_entropy(input, target, self.ignore_index, self.label_smoothing)
        return super().forward(input, target)


class Linear(_tnn.Linear):
    """y = x W^T + b on the MFMA head kernel (activations in the autocast dtype)."""

    def forward(self, input):
        if input.is_cuda and self.weight.dtype == torch.float32:
            from ..ops.head import linear

            return linear(input, self.weight, self.bias)
        return super().forward(input)
