"""MNIST-shaped datasets: IDX reader (torchvision's on-disk layout) and a
deterministic synthetic generator for machines without the dataset.

reference: /root/reference/ddp_main.py:127-129,143-145 —
``torchvision.datasets.MNIST(root="./data", train=..., transform=ToTensor(),
download=True)``.  torchvision is not installed here and there is no network,
so: if ``<root>/MNIST/raw/{train,t10k}-{images-idx3,labels-idx1}-ubyte[.gz]``
exist they are read; otherwise (or with ``synthetic=True``) a synthetic set of
the same shape/dtype is generated: 60,000 train / 10,000 test uint8 1x28x28
images, 10 classes.  Samples are class prototypes (random strokes) with
random translation, intensity and pixel noise, so the task is learnable and
accuracy is meaningful.

Datasets keep the raw uint8 images; ``ToTensor`` semantics (x / 255, no
mean/std normalisation) are applied by the loader's gather kernel.
"""
from __future__ import annotations

import gzip
import os
import struct

import numpy as np
import torch


class ImageDataset:
    """uint8 images [N, H, W] (one channel, MNIST) or [N, C, H, W] + int64 labels [N];
    items are (float [C,H,W] in [0,1], int)."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, name: str = ""):
        assert images.dtype == torch.uint8 and images.dim() in (3, 4)
        assert labels.dtype == torch.int64 and labels.numel() == images.shape[0]
        self.images = images
        self.labels = labels
        self.name = name
        self._dev_cache: dict = {}

    @property
    def sample_shape(self) -> tuple:
        """(C, H, W) of one item (what ToTensor yields)."""
        s = tuple(self.images.shape[1:])
        return (1,) + s if len(s) == 2 else s

    def __len__(self):
        return self.images.shape[0]

    def __getitem__(self, i):
        return self.images[i].float().div_(255.0).reshape(self.sample_shape), int(self.labels[i])

    @property
    def num_classes(self) -> int:
        return int(self.labels.max().item()) + 1 if len(self) else 0

    def to_device(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        """The dataset resident in device memory (cached)."""
        key = str(device)
        if key not in self._dev_cache:
            self._dev_cache[key] = (self.images.to(device), self.labels.to(device))
        return self._dev_cache[key]


# --------------------------------------------------------------------- IDX
def _open(path):
    if os.path.exists(path):
        return open(path, "rb")
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    raise FileNotFoundError(path)


def read_idx(path: str) -> np.ndarray:
    with _open(path) as f:
        data = f.read()
    zero, dtype_code, ndim = struct.unpack(">HBB", data[:4])
    if zero != 0 or dtype_code != 0x08:
        raise ValueError(f"{path}: not an unsigned-byte IDX file")
    dims = struct.unpack(">" + "I" * ndim, data[4:4 + 4 * ndim])
    arr = np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim)
    return arr.reshape(dims)


def _idx_paths(root: str, train: bool):
    p = "train" if train else "t10k"
    raw = os.path.join(root, "MNIST", "raw")
    return os.path.join(raw, f"{p}-images-idx3-ubyte"), os.path.join(raw, f"{p}-labels-idx1-ubyte")


def idx_available(root: str) -> bool:
    for train in (True, False):
        for path in _idx_paths(root, train):
            if not (os.path.exists(path) or os.path.exists(path + ".gz")):
                return False
    return True


def load_idx(root: str, train: bool) -> ImageDataset:
    ip, lp = _idx_paths(root, train)
    imgs = torch.from_numpy(read_idx(ip).copy())
    labels = torch.from_numpy(read_idx(lp).astype(np.int64))
    return ImageDataset(imgs, labels, name=f"MNIST-{'train' if train else 'test'}")


# --------------------------------------------------------------- synthetic
def _prototypes(rng: np.random.Generator, classes: int, hw: int) -> np.ndarray:
    yy, xx = np.mgrid[0:hw, 0:hw].astype(np.float32)
    protos = np.zeros((classes, hw, hw), np.float32)
    for c in range(classes):
        img = np.zeros((hw, hw), np.float32)
        for _ in range(3):  # three random strokes per class
            p0 = rng.uniform(6, hw - 6, size=2)
            p1 = rng.uniform(6, hw - 6, size=2)
            for t in np.linspace(0.0, 1.0, 24):
                cy, cx = p0 * (1 - t) + p1 * t
                img += np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * 1.3 ** 2))
        protos[c] = np.clip(img / img.max() * 1.2, 0, 1)
    return protos


def synthetic(n: int, seed: int, classes: int = 10, hw: int = 28, proto_seed: int = 1234,
              name: str = "synthetic") -> ImageDataset:
    """Deterministic MNIST-shaped dataset (prototypes shared across splits via ``proto_seed``)."""
    prng = np.random.default_rng(proto_seed)
    protos = _prototypes(prng, classes, hw)
    shifts = [(dy, dx) for dy in range(-2, 3) for dx in range(-2, 3)]
    variants = np.stack([np.roll(protos, s, axis=(1, 2)) for s in shifts], 1)  # [C, 25, hw, hw]
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, size=n)
    which = rng.integers(0, len(shifts), size=n)
    amp = rng.uniform(0.6, 1.0, size=(n, 1, 1)).astype(np.float32)
    out = np.empty((n, hw, hw), np.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = variants[labels[s:e], which[s:e]] * amp[s:e]
        noise = rng.normal(0.0, 0.25, size=base.shape).astype(np.float32)
        out[s:e] = (np.clip(base + noise, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
    return ImageDataset(torch.from_numpy(out), torch.from_numpy(labels.astype(np.int64)), name=name)


def MNIST(root: str = "./data", train: bool = True, synthetic_fallback: bool = True, force_synthetic: bool = False,
          n: int | None = None) -> ImageDataset:
    """MNIST from IDX files if present under ``root``, else the synthetic stand-in."""
    if not force_synthetic and idx_available(root):
        return load_idx(root, train)
    if not synthetic_fallback and not force_synthetic:
        raise FileNotFoundError(f"MNIST IDX files not found under {root}/MNIST/raw")
    if n is None:
        n = 60000 if train else 10000
    return synthetic(n, seed=1 if train else 2, name=f"synthetic-MNIST-{'train' if train else 'test'}")
