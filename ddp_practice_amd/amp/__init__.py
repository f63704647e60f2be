"""Mixed precision: an explicit precision policy (autocast) and a device-resident GradScaler.

reference: /root/reference/ddp_main.py:31 (``torch.cuda.amp.autocast()`` inside
``ConvNet.forward``), :10,126,91-93 (``GradScaler``; scale / step / update).
"""
from .autocast import autocast, compute_dtype, is_enabled, current_dtype  # noqa: F401
from .grad_scaler import GradScaler  # noqa: F401
