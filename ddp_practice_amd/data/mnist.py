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
        """The dataset resident in device memory (cached; no copy if it was built there)."""
        key = str(device)
        if key not in self._dev_cache and self.images.device == torch.device(device):
            self._dev_cache[key] = (self.images, self.labels)
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


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _noise_np(seed: int, start: int, count: int) -> np.ndarray:
    """N(0,1) float32 for the flat pixel counters [start, start+count) -- the host twin of
    csrc/kernels/data.hip synth_kernel (splitmix64 + Box-Muller)."""
    with np.errstate(over="ignore"):
        z = _splitmix64((np.uint64(seed) << np.uint64(40)) + np.arange(start, start + count, dtype=np.uint64))
    u1 = ((z >> np.uint64(40)) + np.uint64(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    u2 = ((z >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return (np.sqrt(np.float32(-2.0) * np.log(u1)) * np.cos(np.float32(6.2831853071795864) * u2)).astype(np.float32)


def synthetic(n: int, seed: int, classes: int = 10, hw: int = 28, proto_seed: int = 1234,
              name: str = "synthetic", device=None) -> ImageDataset:
    """Deterministic MNIST-shaped dataset (prototypes shared across splits via ``proto_seed``).

    Per sample: a class prototype shifted by up to 2 pixels, scaled by U(0.6, 1), plus
    0.25 * N(0,1) pixel noise from a counter-based generator.  ``device`` = a HIP device:
    the images are generated in HBM by one kernel (csrc/kernels/data.hip synth) and never
    exist on the host; on the host the same formula runs in numpy (equal up to float
    rounding of the noise)."""
    prng = np.random.default_rng(proto_seed)
    protos = _prototypes(prng, classes, hw)
    shifts = [(dy, dx) for dy in range(-2, 3) for dx in range(-2, 3)]
    variants = np.stack([np.roll(protos, s, axis=(1, 2)) for s in shifts], 1)  # [C, 25, hw, hw]
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, size=n)
    which = rng.integers(0, len(shifts), size=n)
    amp = rng.uniform(0.6, 1.0, size=n).astype(np.float32)
    npix = hw * hw
    if device is not None and torch.device(device).type == "cuda":
        from .._ext import load as _load_ext

        dev = torch.device(device)
        out = torch.empty((n, hw, hw), dtype=torch.uint8, device=dev)
        lab = torch.from_numpy(labels.astype(np.int64)).to(dev)
        _load_ext().data.synth(torch.from_numpy(variants).to(dev), lab, torch.from_numpy(which.astype(np.int64)).to(dev),
                               torch.from_numpy(amp).to(dev), len(shifts), int(seed), out)
        return ImageDataset(out, lab, name=name)
    out = np.empty((n, hw, hw), np.uint8)
    chunk = 4096
    flat_var = variants.reshape(classes * len(shifts), npix)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = flat_var[labels[s:e] * len(shifts) + which[s:e]] * amp[s:e, None]
        noise = _noise_np(seed, s * npix, (e - s) * npix).reshape(e - s, npix)
        v = np.clip(base + np.float32(0.25) * noise, 0.0, 1.0) * np.float32(255.0) + np.float32(0.5)
        out[s:e] = v.astype(np.uint8).reshape(e - s, hw, hw)
    return ImageDataset(torch.from_numpy(out), torch.from_numpy(labels.astype(np.int64)), name=name)


def MNIST(root: str = "./data", train: bool = True, synthetic_fallback: bool = True, force_synthetic: bool = False,
          n: int | None = None, device=None) -> ImageDataset:
    """MNIST from IDX files if present under ``root``, else the synthetic stand-in."""
    if not force_synthetic and idx_available(root):
        return load_idx(root, train)
    if not synthetic_fallback and not force_synthetic:
        raise FileNotFoundError(f"MNIST IDX files not found under {root}/MNIST/raw")
    if n is None:
        n = 60000 if train else 10000
    return synthetic(n, seed=1 if train else 2, name=f"synthetic-MNIST-{'train' if train else 'test'}",
                     device=device)
