"""GroupPlan rank math (reference utils.py:146-163)."""
import pytest
from hypothesis import given, strategies as st

from multidisttorch_amd.parallel.groups import GroupPlan


def test_contiguous_blocks_and_idle():
    p = GroupPlan(8, 2)
    assert p.all_ranks() == [[0, 1, 2, 3], [4, 5, 6, 7]]
    assert p.idle_ranks == []
    p = GroupPlan(5, 2)
    assert p.all_ranks() == [[0, 1], [2, 3]]
    assert p.idle_ranks == [4]
    assert p.group_of(4) is None and p.group_rank_of(4) == -1
    assert p.group_of(3) == 1 and p.group_rank_of(3) == 1


def test_too_many_groups_asserts():
    with pytest.raises(AssertionError):
        GroupPlan(1, 2)


@given(st.integers(1, 64), st.integers(1, 64))
def test_partition_properties(w, k):
    if k > w:
        return
    p = GroupPlan(w, k)
    seen = [r for g in p.all_ranks() for r in g]
    assert seen == sorted(seen) == list(range(k * (w // k)))
    assert len(p.idle_ranks) == w % k
    for r in range(w):
        g = p.group_of(r)
        if g is not None:
            assert r in p.ranks(g) and p.group_rank_of(r) == r - p.ranks(g)[0]


def test_p2p_two_shot_rule(monkeypatch):
    """p2p reducer kinds: one-shot at s = 2 (equal bytes per link), two-shot
    for buckets >= MDT_P2P_TWO_SHOT_MB in groups of 3+; p2p1/p2p2 force a form."""
    from multidisttorch_amd.parallel.ddp import P2P_KINDS, two_shot_min_bytes

    monkeypatch.delenv("MDT_P2P_TWO_SHOT_MB", raising=False)
    assert two_shot_min_bytes(P2P_KINDS["p2p"], 2) == -1
    assert two_shot_min_bytes(P2P_KINDS["p2p"], 4) == 4 << 20
    assert two_shot_min_bytes(P2P_KINDS["p2p1"], 8) == -1
    assert two_shot_min_bytes(P2P_KINDS["p2p2"], 2) == 0
    monkeypatch.setenv("MDT_P2P_TWO_SHOT_MB", "0.5")
    assert two_shot_min_bytes(P2P_KINDS["p2p"], 3) == 1 << 19
