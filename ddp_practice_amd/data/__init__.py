"""Data pipeline: MNIST IDX / synthetic datasets, DistributedSampler, device-resident loader."""
from .mnist import MNIST, ImageDataset, synthetic, read_idx, idx_available  # noqa: F401
from .imagenet import synthetic_imagenet  # noqa: F401
from .sampler import DistributedSampler  # noqa: F401
from .loader import DeviceLoader, accepts_deferred, flush_pending  # noqa: F401
