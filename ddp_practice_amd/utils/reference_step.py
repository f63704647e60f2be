"""The reference's training step on PyTorch's own stack: the same-node baseline.

This is what /root/reference/ddp_main.py:83-93 (``train``) and :117-126 run,
re-expressed for a device-resident batch so that only the framework differs:

    model = ConvNet()                                  torch nn modules (fused=False)
    model = nn.SyncBatchNorm.convert_sync_batchnorm(model)      W > 1  (:120)
    model = torch.nn.parallel.DistributedDataParallel(model)    W > 1  (:121-123)
    with torch.autocast("cuda", dtype): outputs = model(images)  (:31, autocast in forward)
    loss = nn.CrossEntropyLoss()(outputs, labels)                (:89, outside autocast)
    optimizer.zero_grad(); scaler.scale(loss).backward()         (:90-91)
    scaler.step(optimizer); scaler.update()                      (:92-93, torch.amp.GradScaler)

with ``torch.optim.SGD(lr=1e-4)`` and torch DDP over the default
``torch.distributed`` process group (RCCL).  Differences, all in torch's
favour: the uint8 dataset is resident on the device and a batch is an index
gather + ``/255`` (the reference's DataLoader workers and H2D copies are
gone), and at W = 1 the model is not wrapped in DDP.

Used by ``bench.py`` (``baseline_same_node_img_s`` and ``--impl torch``).
"""
from __future__ import annotations

import time

import torch
import torch.nn as nn


class TorchReferenceStep:
    def __init__(self, device: torch.device, amp_dtype: torch.dtype | None, world: int, images_u8: torch.Tensor,
                 labels: torch.Tensor, order: torch.Tensor, batch_size: int, local_rank: int | None = None,
                 seed: int = 0):
        from ..models import ConvNet

        torch.manual_seed(seed)
        model = ConvNet(amp_dtype=None, fused=False).to(device)
        if world > 1:
            model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
            model = nn.parallel.DistributedDataParallel(
                model, device_ids=[local_rank if local_rank is not None else device.index])
        self.model = model
        self.criterion = nn.CrossEntropyLoss().to(device)
        self.optimizer = torch.optim.SGD(model.parameters(), 1e-4)
        self.amp_dtype = amp_dtype
        self.scaler = torch.amp.GradScaler("cuda", enabled=amp_dtype is not None)
        self.images, self.labels, self.order = images_u8, labels, order
        self.B = batch_size
        self.nfull = order.numel() // batch_size
        self.pos = 0

    def _batch(self):
        if self.pos >= self.nfull:
            self.pos = 0
        idx = self.order[self.pos * self.B:(self.pos + 1) * self.B]
        self.pos += 1
        return self.images[idx].unsqueeze(1).float().div_(255.0), self.labels[idx]

    def step(self) -> None:
        images, labels = self._batch()
        with torch.autocast("cuda", dtype=self.amp_dtype or torch.float16, enabled=self.amp_dtype is not None):
            outputs = self.model(images)
        loss = self.criterion(outputs, labels)
        self.optimizer.zero_grad()
        self.scaler.scale(loss).backward()
        self.scaler.step(self.optimizer)
        self.scaler.update()

    def time_steps(self, steps: int, warmup: int, barrier) -> float:
        """Seconds for ``steps`` steps after ``warmup`` untimed ones (barrier + sync on both sides)."""
        self.model.train()
        for _ in range(warmup):
            self.step()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0
