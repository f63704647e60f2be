"""Synthetic ImageNet-shaped dataset for the CLIs' ``--model resnet50`` runs
(BASELINE.json config 5: ResNet-50 on synthetic 3x224x224).

The reference trains only its MNIST ConvNet (/root/reference/ddp_main.py:127-145);
there is no ImageNet reader here and no network to fetch one, so the set is
generated: uint8 [N, 3, hw, hw] images, ``classes`` labels.  Each class has a
coarse 3x8x8 colour prototype; a sample is its class prototype upsampled to
hw x hw (nearest), scaled by a random intensity, plus uniform pixel noise, so the
task is learnable and accuracy moves.  Generation is chunked and cheap (uint8
noise), ~0.15 MB per 224x224 sample.
"""
from __future__ import annotations

import numpy as np
import torch

from .mnist import ImageDataset


def synthetic_imagenet(n: int, seed: int, classes: int = 1000, hw: int = 224, proto_seed: int = 4321,
                       name: str = "synthetic-imagenet") -> ImageDataset:
    g = 8
    prng = np.random.default_rng(proto_seed)
    protos = prng.uniform(0.0, 200.0, size=(classes, 3, g, g)).astype(np.float32)
    rep = -(-hw // g)  # ceil: nearest upsampling factor, cropped to hw
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, classes, size=n)
    amp = rng.uniform(0.6, 1.0, size=(n, 1, 1, 1)).astype(np.float32)
    out = np.empty((n, 3, hw, hw), np.uint8)
    chunk = 256
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = protos[labels[s:e]] * amp[s:e]                     # [b, 3, g, g]
        up = base.repeat(rep, axis=2).repeat(rep, axis=3)[:, :, :hw, :hw]
        noise = rng.integers(0, 56, size=up.shape, dtype=np.uint8)
        out[s:e] = up.astype(np.uint8) + noise                    # <= 200 + 55: no overflow
    return ImageDataset(torch.from_numpy(out), torch.from_numpy(labels.astype(np.int64)), name=name)
