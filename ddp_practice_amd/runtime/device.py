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


def shared_gpu_env(world: int | None) -> None:
    """Environment of ranks that share one device (``--share-gpu`` rehearsals): the fused
    paths' gates (``DPA_SHARED_GPU``) and, for 3+ ranks, one HIP hardware queue per process.

    With HIP's default 4 queues per process, 4 processes on one MI355X stalled at the same
    point of the 3-epoch phase twice (every rank's host had issued the same collectives;
    their one-shot all-reduce kernels waited on a peer whose work never ran), and completed
    twice at 836-841k img/s with one queue each (``profiles/r5v_shared_gpu_hw_queues.txt``):
    more queues than the scheduler maps at once leave a rank unscheduled while its peers
    spin.  ``DPA_SHARED_HW_QUEUES`` overrides the count.  Before the first HIP call only.
    """
    os.environ["DPA_SHARED_GPU"] = "1"
    q = os.environ.get("DPA_SHARED_HW_QUEUES")
    if q is None and (world is None or world >= 3):
        q = "1"
    if q:
        os.environ["GPU_MAX_HW_QUEUES"] = q
