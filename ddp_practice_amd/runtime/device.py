"""Device selection.

The reference maps ``--gpu "0,1"`` to ``CUDA_VISIBLE_DEVICES`` before any GPU
initialisation (/root/reference/ddp_main.py:63, ddp_main_torchrun.py:58).  On
ROCm the HIP runtime honours ``CUDA_VISIBLE_DEVICES`` as well; only that
variable is set (setting ``HIP_VISIBLE_DEVICES`` too would filter twice).  Must
run before the first HIP call in the process (``torch.cuda.device_count()``
does not initialise the runtime on this image).
"""
from __future__ import annotations

import os


def select_devices(gpu: str | None) -> None:
    if gpu is None or gpu == "":
        return
    os.environ["CUDA_VISIBLE_DEVICES"] = gpu


def local_device():
    import torch

    if not torch.cuda.is_available():
        return torch.device("cpu")
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()
    return torch.device("cuda", lr % max(n, 1))
