"""Data pipeline semantics (CPU): DistributedSampler parity with torch, IDX reader,
synthetic determinism, DeviceLoader order/contents."""
import math
import os
import struct

import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler as TorchDS

from ddp_practice_amd.data import DeviceLoader, DistributedSampler, ImageDataset, MNIST, read_idx, synthetic


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [1, 7, 60000, 10000, 33])
@pytest.mark.parametrize("w", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("drop_last", [False, True])
@pytest.mark.parametrize("shuffle", [True, False])
def test_sampler_matches_torch(n, w, drop_last, shuffle):
    if drop_last and n < w:
        return
    for epoch in (0, 3):
        for rank in range(w):
            ours = DistributedSampler(_DS(n), num_replicas=w, rank=rank, shuffle=shuffle, seed=5, drop_last=drop_last)
            ref = TorchDS(_DS(n), num_replicas=w, rank=rank, shuffle=shuffle, seed=5, drop_last=drop_last)
            ours.set_epoch(epoch)
            ref.set_epoch(epoch)
            assert len(ours) == len(ref)
            assert list(iter(ours)) == list(iter(ref))


def test_sampler_padding_large_world():
    # padding larger than the dataset (repeat-then-truncate branch)
    for rank in range(8):
        ours = DistributedSampler(_DS(3), num_replicas=8, rank=rank)
        ref = TorchDS(_DS(3), num_replicas=8, rank=rank)
        assert list(iter(ours)) == list(iter(ref))


def _write_idx(path, arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(struct.pack(">HBB", 0, 0x08, arr.ndim))
        f.write(struct.pack(">" + "I" * arr.ndim, *arr.shape))
        f.write(arr.tobytes())


def test_idx_roundtrip(tmp_path):
    raw = tmp_path / "MNIST" / "raw"
    raw.mkdir(parents=True)
    rng = np.random.default_rng(0)
    for split, n in (("train", 50), ("t10k", 20)):
        _write_idx(raw / f"{split}-images-idx3-ubyte", rng.integers(0, 256, (n, 28, 28)))
        _write_idx(raw / f"{split}-labels-idx1-ubyte", rng.integers(0, 10, (n,)))
    ds = MNIST(root=str(tmp_path), train=True)
    assert len(ds) == 50 and ds.images.shape == (50, 28, 28)
    assert torch.equal(ds.images, torch.from_numpy(read_idx(str(raw / "train-images-idx3-ubyte")).copy()))
    x, y = ds[3]
    assert x.shape == (1, 28, 28) and 0.0 <= x.min() and x.max() <= 1.0 and isinstance(y, int)
    assert len(MNIST(root=str(tmp_path), train=False)) == 20


def test_synthetic_deterministic_and_learnable_shape():
    a = synthetic(512, seed=1)
    b = synthetic(512, seed=1)
    c = synthetic(512, seed=2)
    assert torch.equal(a.images, b.images) and torch.equal(a.labels, b.labels)
    assert not torch.equal(a.images, c.images)
    assert a.images.dtype == torch.uint8 and a.images.shape == (512, 28, 28)
    assert set(a.labels.tolist()) <= set(range(10))
    # class prototypes are shared across splits: per-class means correlate
    ma = torch.stack([a.images[a.labels == k].float().mean(0) for k in range(10)]).flatten(1)
    mc = torch.stack([c.images[c.labels == k].float().mean(0) for k in range(10)]).flatten(1)
    cos = torch.nn.functional.cosine_similarity(ma, mc)
    assert cos.min() > 0.9


def test_device_loader_cpu_matches_manual():
    ds = synthetic(100, seed=3)
    s = DistributedSampler(ds, num_replicas=2, rank=1, shuffle=True)
    s.set_epoch(2)
    ld = DeviceLoader(ds, batch_size=16, sampler=s, device="cpu")
    order = s.indices()
    batches = list(ld)
    assert [b[0].shape[0] for b in batches] == ld.batch_sizes() == [16, 16, 16, 2]
    assert len(ld) == math.ceil(50 / 16)
    for i, (x, y) in enumerate(batches):
        sel = order[i * 16:(i + 1) * 16]
        assert torch.allclose(x, ds.images[sel].float().unsqueeze(1) / 255.0)
        assert torch.equal(y, ds.labels[sel])


def test_device_loader_drop_last_and_shuffle_generator():
    ds = synthetic(50, seed=4)
    g1 = torch.Generator().manual_seed(7)
    g2 = torch.Generator().manual_seed(7)
    a = [y for _, y in DeviceLoader(ds, batch_size=8, shuffle=True, generator=g1, drop_last=True, device="cpu")]
    b = [y for _, y in DeviceLoader(ds, batch_size=8, shuffle=True, generator=g2, drop_last=True, device="cpu")]
    assert len(a) == 6 and all(torch.equal(u, v) for u, v in zip(a, b))


def test_image_dataset_getitem_totensor_semantics():
    imgs = torch.arange(0, 2 * 28 * 28, dtype=torch.int64).remainder(256).to(torch.uint8).view(2, 28, 28)
    ds = ImageDataset(imgs, torch.tensor([3, 4]))
    x, y = ds[1]
    assert y == 4 and torch.allclose(x[0], imgs[1].float() / 255.0)


def test_synthetic_imagenet_multichannel_loader():
    """[N, C, H, W] uint8 datasets (the CLIs' --model resnet50 set): ToTensor items are
    [C, H, W], and the loader's batches match a manual gather."""
    import torch

    from ddp_practice_amd.data import DeviceLoader, synthetic_imagenet

    ds = synthetic_imagenet(10, seed=3, classes=7, hw=20)
    assert ds.images.shape == (10, 3, 20, 20) and ds.sample_shape == (3, 20, 20)
    assert int(ds.labels.max()) < 7
    x, y = ds[4]
    assert x.shape == (3, 20, 20) and torch.equal(x, ds.images[4].float() / 255.0) and y == int(ds.labels[4])
    again = synthetic_imagenet(10, seed=3, classes=7, hw=20)
    assert torch.equal(again.images, ds.images)  # deterministic
    ld = DeviceLoader(ds, batch_size=4, device="cpu")
    seen = 0
    for imgs, labels in ld:
        assert imgs.shape[1:] == (3, 20, 20)
        for i in range(imgs.shape[0]):
            src = int(ld._order[seen + i])
            assert torch.equal(imgs[i], ds.images[src].float() / 255.0) and int(labels[i]) == int(ds.labels[src])
        seen += imgs.shape[0]
    assert seen == 10
