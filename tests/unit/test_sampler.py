"""Index parity with torch DistributedSampler(rank=group_id, num_replicas=K)
(reference vae-hpo.py:146), including padding and drop_last."""
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from multidisttorch_amd.data.sampler import EpochIndexer, shard_indices


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,k", [(60000, 1), (60000, 2), (60000, 7), (101, 4), (5, 8)])
@pytest.mark.parametrize("drop_last", [False, True])
def test_parity(n, k, drop_last):
    for r in range(k):
        ref = list(DistributedSampler(_DS(n), num_replicas=k, rank=r, drop_last=drop_last))
        ours = shard_indices(n, k, r, drop_last=drop_last).tolist()
        assert ours == ref


def test_epoch_order_fixed_without_set_epoch():
    ix = EpochIndexer(1000, 2, 1)
    assert torch.equal(ix(0), ix(5))
    ix2 = EpochIndexer(1000, 2, 1, set_epoch=True)
    assert not torch.equal(ix2(0), ix2(1))


@pytest.mark.parametrize("w,k", [(3, 2), (7, 3), (8, 3), (5, 2), (8, 8), (8, 2)])
def test_reference_num_replicas_and_shards(w, k):
    """num_replicas = W // (W // K), as /root/reference/vae-hpo.py:146 computes
    it (world_size // local_size) -- not K when W % K leaves idle ranks."""
    from multidisttorch_amd.data.sampler import reference_num_replicas

    n = w // k
    nrep = reference_num_replicas(w, n)
    assert nrep == w // n
    if (w, k) == (3, 2):
        assert nrep == 3  # differs from K = 2
    if (w, k) == (7, 3):
        assert nrep == 3
    for g in range(k):  # every trial group's shard is DistributedSampler(rank=g, num_replicas=W//n)
        ref = list(DistributedSampler(_DS(60000), num_replicas=w // n, rank=g))
        assert shard_indices(60000, nrep, g).tolist() == ref
