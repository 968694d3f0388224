"""Carving the world into K disjoint trial groups.

Parity:
  * ``setup_ddp_groups`` <- /root/reference/utils.py:146-163
    (contiguous blocks ``[g*n, (g+1)*n)``, ``n = W // K``, leftover ranks idle,
    every rank enters every ``new_group`` in the same order, returns all K
    handles with ``GroupMember.NON_GROUP_MEMBER`` for non-members)
  * ``print0`` <- /root/reference/utils.py:165-174 (``"[W:G] msg"`` from group
    rank 0 only).

The rank arithmetic lives in :class:`GroupPlan` (pure, unit-testable, no
process group needed). On an 8xMI355X node with one process per GPU the plan
keeps each trial on contiguous GPUs; in a fully connected xGMI mesh any
contiguous block of size s has s-1 direct links per member, so contiguity is
free and matches the reference's mapping.
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch.distributed as dist

__all__ = ["GroupPlan", "TrialGroup", "setup_ddp_groups", "print0", "member_groups",
           "group_rank", "group_size"]


@dataclass(frozen=True)
class GroupPlan:
    """Pure rank math for a K-way contiguous carve of a world of size W."""

    world_size: int
    num_groups: int

    def __post_init__(self):
        if self.num_groups < 1:
            raise ValueError("num_groups must be >= 1")
        if self.world_size < self.num_groups:
            raise AssertionError(
                f"Number of groups {self.num_groups} requested exceeds number of total "
                f"processes {self.world_size} available")

    @property
    def ranks_per_group(self) -> int:
        return self.world_size // self.num_groups

    def ranks(self, g: int) -> List[int]:
        n = self.ranks_per_group
        return list(range(g * n, g * n + n))

    def all_ranks(self) -> List[List[int]]:
        return [self.ranks(g) for g in range(self.num_groups)]

    def group_of(self, world_rank: int) -> Optional[int]:
        g = world_rank // self.ranks_per_group
        return g if g < self.num_groups else None

    def group_rank_of(self, world_rank: int) -> int:
        g = self.group_of(world_rank)
        return -1 if g is None else world_rank - g * self.ranks_per_group

    @property
    def idle_ranks(self) -> List[int]:
        return list(range(self.num_groups * self.ranks_per_group, self.world_size))


@dataclass
class TrialGroup:
    """A group handle plus its plan coordinates (returned by ``member_groups``)."""

    group_id: int
    ranks: Sequence[int]
    pg: object
    world_rank: int = 0
    extra: dict = field(default_factory=dict)

    @property
    def size(self) -> int:
        return len(self.ranks)

    @property
    def rank(self) -> int:
        return self.world_rank - self.ranks[0] if self.world_rank in self.ranks else -1


def setup_ddp_groups(num_groups: int, verbose: bool = True, backend: Optional[str] = None):
    """Create all K trial groups (world collective); return the K handles.

    Every rank calls ``dist.new_group`` for every group in the same order:
    torch names process groups from a per-process counter, so skipping a call
    on non-members would make store keys collide (the anti-pattern commented
    out at /root/reference/example-subgroup.py:10-17).
    """
    from ..runtime.bootstrap import get_comm_size_and_rank

    world_size, world_rank = get_comm_size_and_rank()
    if verbose:
        print("world_size, world_rank:", world_size, world_rank)
    plan = GroupPlan(world_size, num_groups)
    handles = []
    import datetime as _dt

    from ..runtime.faults import group_timeout_s

    from ..runtime.bootstrap import bound_device, world_is_device_bound

    # On an eager, device-bound RCCL world, passing device_id makes torch
    # derive each trial communicator with ncclCommSplit from the world
    # communicator (every rank takes part; non-members split with NOCOLOR).
    split = backend in (None, "nccl") and world_is_device_bound()
    for g in range(num_groups):
        # bounded collective timeout: a dead replica fails its group fast
        kw = {"ranks": plan.ranks(g), "timeout": _dt.timedelta(seconds=group_timeout_s())}
        if backend is not None:
            kw["backend"] = backend
        if split:
            kw["device_id"] = bound_device()
        handles.append(dist.new_group(**kw))
    for g in range(num_groups):
        if dist.get_rank(handles[g]) >= 0:
            if verbose:
                print(f"Rank {world_rank} is in group {g}")
    return handles


def member_groups(handles) -> List[TrialGroup]:
    """The (usually single) groups this rank belongs to, as TrialGroup records."""
    world_size = dist.get_world_size()
    world_rank = dist.get_rank()
    plan = GroupPlan(world_size, len(handles))
    out = []
    for g, pg in enumerate(handles):
        if dist.get_rank(pg) >= 0:
            out.append(TrialGroup(g, plan.ranks(g), pg, world_rank))
    return out


def group_rank(pg=None) -> int:
    return dist.get_rank(pg) if dist.is_initialized() else 0


def group_size(pg=None) -> int:
    return dist.get_world_size(pg) if dist.is_initialized() else 1


def print0(*args, sep=" ", process_group=None):
    """Print ``"[world_rank:group_rank] msg"`` from rank 0 of ``process_group``."""
    if dist.is_initialized():
        rank = dist.get_rank(process_group)
        world_rank = dist.get_rank()
    else:
        rank, world_rank = 0, 0
    if rank == 0:
        print(f"[{world_rank}:{rank}]", sep.join(map(str, args)), flush=True)
