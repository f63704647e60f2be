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


def _loaded_hip():
    """The HIP runtime this process already loaded (torch's bundled libamdhip64), or None.  Opening
    another copy by name could bring up a second runtime whose settings torch never sees."""
    import ctypes

    try:
        with open("/proc/self/maps") as f:
            paths = {ln.split()[-1] for ln in f if "libamdhip64" in ln}
    except OSError:
        return None
    return ctypes.CDLL(sorted(paths)[0]) if paths else None


def spin_sync(device: int = 0) -> int | None:
    """Host waits on the GPU (``torch.cuda.synchronize``, event and stream waits) busy-poll:
    ``hipSetDeviceFlags(hipDeviceScheduleSpin)`` on ``device``.  HIP's default (Auto) yields
    the CPU whenever the host has more logical CPUs than HIP contexts -- always, here -- and a
    yielding wait notices completion later.  Call after ``import torch`` and before the
    device's first use (hipErrorSetOnActiveProcess after it).  Opt-in (``DPA_SPIN_SYNC=1``): on
    the driver's 20-step ConvNet window it measured no difference (0.0491-0.0518 vs
    0.0491-0.0504 ms, profiles/r6u_spin_sync_ab.txt).  Returns the hipError code, None when
    skipped (not opted in, or no HIP runtime loaded)."""
    if os.environ.get("DPA_SPIN_SYNC", "0") != "1":
        return None
    import ctypes

    lib = _loaded_hip()
    if lib is None:
        return None
    rc = lib.hipSetDevice(ctypes.c_int(device))
    if rc != 0:
        return int(rc)
    return int(lib.hipSetDeviceFlags(ctypes.c_uint(1)))  # hipDeviceScheduleSpin


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


def shared_cu_mask(world: int | None, rank: int) -> str | None:
    """Ranks sharing one device (``--share-gpu`` rehearsals), 3 or more: rank ``rank`` runs on
    its own 1/world of the compute units (``HSA_CU_MASK``, read by the HSA runtime when it
    creates the process's queues), and the residency checks of the fused kernels count only
    those (``DPA_RESIDENT_CUS``, csrc/common.h co_resident).

    Why: every rank's in-kernel exchanges and grid barriers spin until their peers / their
    own workgroups arrive.  With one rank per GPU (the driver's multi-GPU run) a rank's
    kernels always have a whole card; eight ranks on ONE card without masks let the spinning
    workgroups of seven ranks occupy the CUs a waiting eighth rank needs -- the world-8
    rehearsals stalled so (profiles/r6c_rehearse8_stall.txt).  Disjoint CU ranges make each
    rank a small "GPU" of its own.  ``DPA_SHARED_CUS`` is the device's CU count (MI355X: 256),
    ``DPA_SHARED_CU_MASK=0`` disables the masks.  Before the rank's first HIP call only."""
    if world is None or world < 3 or os.environ.get("DPA_SHARED_CU_MASK", "1") == "0":
        return None
    n = int(os.environ.get("DPA_SHARED_CUS", "256"))
    per = max(1, n // world)
    lo = (rank % world) * per
    mask = f"0:{lo}-{lo + per - 1}"
    os.environ["HSA_CU_MASK"] = mask
    os.environ["DPA_RESIDENT_CUS"] = str(per)
    return mask
