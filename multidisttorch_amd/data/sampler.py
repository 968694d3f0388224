"""Epoch index lists with ``DistributedSampler`` parity.

The reference shards MNIST **across groups** with
``DistributedSampler(trainset, rank=group_id, num_replicas=world_size//local_size)``
(/root/reference/vae-hpo.py:146) — every member of a group sees the same
shard — and never calls ``set_epoch`` (same order every epoch).
``shard_indices`` reproduces torch's algorithm index-for-index
(torch/utils/data/distributed.py: randperm(generator seeded seed+epoch), pad by
wrap-around to a multiple of num_replicas, stride from rank) so trial g trains
on exactly the samples it would under the reference. The list is uploaded
once per epoch as int32 and consumed on the device by the fused kernels.
"""

from __future__ import annotations

import math

import torch

__all__ = ["shard_indices", "batch_count", "EpochIndexer", "reference_num_replicas"]


def reference_num_replicas(world_size: int, group_size: int) -> int:
    """``num_replicas`` exactly as /root/reference/vae-hpo.py:146 computes it:
    ``world_size // local_size`` with ``local_size`` the trial group's size.

    This is NOT always the trial count K: with leftover ranks (W % K != 0) the
    reference still divides the world by the group size, e.g. W=3, K=2 gives
    groups of 1 and ``num_replicas = 3`` (three shards of 20000, the third never
    trained), W=7, K=3 gives groups of 2 and ``num_replicas = 3``."""
    if group_size < 1 or world_size < group_size:
        raise ValueError(f"bad world/group sizes {world_size}/{group_size}")
    return world_size // group_size


def shard_indices(n: int, num_replicas: int, rank: int, shuffle: bool = True, seed: int = 0,
                  epoch: int = 0, drop_last: bool = False) -> torch.Tensor:
    if not 0 <= rank < num_replicas:
        raise ValueError(f"rank {rank} out of range for {num_replicas} replicas")
    if drop_last and n % num_replicas != 0:
        num_samples = math.ceil((n - num_replicas) / num_replicas)
    else:
        num_samples = math.ceil(n / num_replicas)
    total = num_samples * num_replicas
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g)
    else:
        idx = torch.arange(n)
    if not drop_last:
        pad = total - idx.numel()
        if pad > 0:
            if pad <= idx.numel():
                idx = torch.cat([idx, idx[:pad]])
            else:
                idx = torch.cat([idx, idx.repeat(math.ceil(pad / idx.numel()))[:pad]])
    else:
        idx = idx[:total]
    return idx[rank:total:num_replicas].contiguous()


def batch_count(n: int, batch: int) -> int:
    return -(-n // batch)


class EpochIndexer:
    """Caches the per-epoch device index list (constant when set_epoch is not used)."""

    def __init__(self, n: int, num_replicas: int, rank: int, seed: int = 0, shuffle: bool = True,
                 set_epoch: bool = False, device=None):
        self.n, self.num_replicas, self.rank = n, num_replicas, rank
        self.seed, self.shuffle, self.set_epoch = seed, shuffle, set_epoch
        self.device = device
        self._cache = {}

    def __call__(self, epoch: int) -> torch.Tensor:
        e = epoch if self.set_epoch else 0
        if e not in self._cache:
            idx = shard_indices(self.n, self.num_replicas, self.rank, self.shuffle, self.seed, e)
            self._cache = {e: idx.to(device=self.device, dtype=torch.int32)}
        return self._cache[e]

    def __len__(self):
        return math.ceil(self.n / self.num_replicas)
