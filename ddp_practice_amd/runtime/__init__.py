"""Runtime: device selection, hipGraph step capture."""
from .graph import CapturedStep  # noqa: F401
from .device import select_devices, local_device  # noqa: F401
