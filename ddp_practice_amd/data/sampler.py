"""DistributedSampler with torch's exact index semantics, computed as tensors.

torch/utils/data/distributed.py:17,102,107-137,146: ``num_samples =
ceil(N/W)`` (or the drop_last variant), permutation ``randperm(N,
generator=manual_seed(seed + epoch))``, padding by wrapping from the front,
then rank ``r`` takes ``indices[r::W]``.  Every rank therefore sees the same
number of batches, which the per-step collectives (DDP all-reduce, SyncBN)
require.

reference: /root/reference/ddp_main.py:130-132,146-148,160
(``DistributedSampler(dataset)``, ``sampler.set_epoch(epoch)``).
"""
from __future__ import annotations

import math

import torch


class DistributedSampler:
    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            from ..parallel import comm as _comm

            num_replicas = _comm.get_world_size() if num_replicas is None else num_replicas
            rank = _comm.get_rank() if rank is None else rank
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def indices(self) -> torch.Tensor:
        """This rank's indices for the current epoch, as an int64 CPU tensor."""
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(n, generator=g)
        else:
            idx = torch.arange(n)
        if not self.drop_last:
            pad = self.total_size - n
            if pad > 0:
                if pad <= n:
                    idx = torch.cat([idx, idx[:pad]])
                else:
                    idx = torch.cat([idx.repeat(math.ceil(pad / n) + 1)])[: self.total_size]
        else:
            idx = idx[: self.total_size]
        assert idx.numel() == self.total_size
        out = idx[self.rank:self.total_size:self.num_replicas]
        assert out.numel() == self.num_samples
        return out

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
