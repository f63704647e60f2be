"""Device-resident data loader.

Replaces ``DataLoader(dataset, batch_size, sampler=..., num_workers=4,
pin_memory=True, generator=g)`` (reference: /root/reference/ddp_main.py:133-142)
with zero worker processes and zero per-batch host->device copies: the
uint8 dataset is uploaded to HBM once, the epoch's index order (the
DistributedSampler output, or a RandomSampler-style permutation) is uploaded
once per epoch, and each batch is produced by one gather kernel that also
applies ``ToTensor`` (x/255) and casts to the compute dtype.

Two ways to consume it:
  * iteration: ``for images, labels in loader`` — same contract as the
    reference DataLoader (partial last batch kept unless drop_last);
  * static buffers for hipGraph capture: ``loader.static_batch(B)`` returns
    fixed (images, labels) tensors and ``loader.fill_(...)`` the capturable
    gather that advances a device-side step counter.
"""
from __future__ import annotations

import math

import os

import torch

from .._ext import load as _load_ext
from .mnist import ImageDataset


class DeviceLoader:
    def __init__(self, dataset: ImageDataset, batch_size: int = 1, shuffle: bool = False, sampler=None,
                 generator: torch.Generator | None = None, drop_last: bool = False, device=None,
                 dtype: torch.dtype = torch.float32, num_workers: int = 0, pin_memory: bool = False):
        if sampler is not None and shuffle:
            raise ValueError("sampler option is mutually exclusive with shuffle")
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.sampler = sampler
        self.generator = generator
        self.drop_last = drop_last
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.dtype = dtype
        # accepted for signature compatibility; there are no worker processes
        self.num_workers = num_workers
        self.pin_memory = pin_memory
        self._order: torch.Tensor | None = None
        self._ctr = None
        self._imgs, self._labels = dataset.to_device(self.device)
        self._chw = dataset.sample_shape

    # ----------------------------------------------------------- ordering
    def epoch_order(self) -> torch.Tensor:
        """This epoch's sample order (CPU int64)."""
        if self.sampler is not None:
            if hasattr(self.sampler, "indices"):
                return self.sampler.indices()
            return torch.tensor(list(iter(self.sampler)), dtype=torch.int64)
        n = len(self.dataset)
        if self.shuffle:
            if self.generator is None:
                seed = int(torch.empty((), dtype=torch.int64).random_().item())
                g = torch.Generator()
                g.manual_seed(seed)
            else:
                g = self.generator
            return torch.randperm(n, generator=g)
        return torch.arange(n)

    def num_samples(self) -> int:
        return len(self.sampler) if self.sampler is not None else len(self.dataset)

    def __len__(self) -> int:
        n = self.num_samples()
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def batch_sizes(self) -> list[int]:
        n, b = self.num_samples(), self.batch_size
        full = n // b
        out = [b] * full
        if not self.drop_last and n % b:
            out.append(n % b)
        return out

    # --------------------------------------------------------- device path
    def start_epoch(self) -> torch.Tensor:
        """Upload this epoch's order and reset the device step counter."""
        order = self.epoch_order()
        if self._order is None or self._order.shape != order.shape:
            self._order = order.to(self.device)
        else:
            # in place: captured hipGraphs hold this buffer's address
            self._order.copy_(order)
        order = self._order
        if self._ctr is None:
            self._ctr = torch.zeros(2, dtype=torch.int32, device=self.device)
        else:
            self._ctr.zero_()
        return order

    def static_batch(self, batch_size: int | None = None):
        b = batch_size or self.batch_size
        imgs = torch.empty((b,) + self._chw, dtype=self.dtype, device=self.device)
        labels = torch.empty((b,), dtype=torch.int64, device=self.device)
        return imgs, labels

    @staticmethod
    def pair(images: torch.Tensor, labels: torch.Tensor) -> None:
        """Record that ``labels`` are the targets of ``images``: a training forward of the
        fused ConvNet then computes the loss (and the head backward) in its head launch,
        and the loss call on the same ``labels`` launches nothing (ops/convnet_fused.py)."""
        images._dpa_labels = labels

    def fill_(self, images: torch.Tensor, labels: torch.Tensor, step: int = -1, defer: bool = False) -> None:
        """Gather batch ``step`` (or the device counter's step if -1, advancing it).

        ``defer=True`` (device counter only): launch nothing; the gather is recorded on
        ``images`` and performed by the first kernel of a model that consumes it
        (the fused ConvNet's conv1, csrc/kernels/convblock_impl.h PRO 3).  Any other
        reader must call ``flush_pending(images)`` first; ``accepts_deferred`` says
        whether a model does it itself.
        """
        self.pair(images, labels)
        if self._order is None:
            self.start_epoch()
        if defer and step < 0 and self.device.type == "cuda":
            images._dpa_gather = (self._imgs, self._labels, self._order, self._ctr, labels, 1.0 / 255.0, 0.0)
            return
        images._dpa_gather = None
        if self.device.type == "cuda":
            _load_ext().data.gather(self._imgs, self._labels, self._order, self._ctr, int(step), images, labels,
                                    1.0 / 255.0, 0.0)
        else:
            if step < 0:
                step = int(self._ctr[0])
                self._ctr[0] += 1
            b = images.shape[0]
            sel = self._order[step * self.batch_size: step * self.batch_size + b]
            images.copy_((self._imgs[sel].to(torch.float32) / 255.0).reshape(images.shape).to(images.dtype))
            labels.copy_(self._labels[sel])

    def set_step(self, step: int) -> None:
        if self._ctr is None:
            self._ctr = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._ctr[0] = step
        self._ctr[1] = 0

    def __iter__(self):
        self.start_epoch()
        for i, b in enumerate(self.batch_sizes()):
            imgs, labels = self.static_batch(b)
            self.fill_(imgs, labels, step=i) if b == self.batch_size else self._fill_tail(imgs, labels, i)
            yield imgs, labels

    def _fill_tail(self, imgs, labels, i):
        # partial last batch: explicit step index, batch_size stride
        self.pair(imgs, labels)
        if self.device.type == "cuda":
            sub = self._order[i * self.batch_size:]
            _load_ext().data.gather(self._imgs, self._labels, sub, self._ctr, 0, imgs, labels, 1.0 / 255.0, 0.0)
        else:
            self.fill_(imgs, labels, step=i)


def flush_pending(images: torch.Tensor) -> None:
    """Perform a deferred gather (``DeviceLoader.fill_(..., defer=True)``) now, if any."""
    g = getattr(images, "_dpa_gather", None)
    if g is None:
        return
    images._dpa_gather = None
    imgs, labels, order, ctr, lab_out, scale, shift = g
    _load_ext().data.gather(imgs, labels, order, ctr, -1, images, lab_out, scale, shift)


def accepts_deferred(model, images: torch.Tensor) -> bool:
    """Whether ``model(images)`` performs a deferred gather itself (so a training step
    may hand it the batch without the separate gather launch)."""
    if os.environ.get("DPA_DEFER_GATHER", "1") == "0":
        return False
    m = getattr(model, "module", model)
    f = getattr(m, "accepts_deferred_batch", None)
    return bool(f is not None and images.is_cuda and f(images))
