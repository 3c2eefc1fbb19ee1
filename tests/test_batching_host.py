"""CPU: the host logic of length-bucketed batching (attack-vc_amd/batching.py)."""
import pytest

import batching


def test_buckets_group_by_key_in_order():
    keys = [128, 96, 128, 300, 96, 128, 64]
    assert batching.buckets(keys, 2) == [[0, 2], [5], [1, 4], [3], [6]]
    assert batching.buckets(keys, 256) == [[0, 2, 5], [1, 4], [3], [6]]
    assert batching.buckets([(128, 100), (128, 128), (128, 100)], 8) == [[0, 2], [1]]
    with pytest.raises(ValueError):
        batching.buckets(keys, 0)


def test_assign_balances_and_covers():
    costs = [10, 1, 5, 5, 3]
    own = batching.assign(costs, 2)
    assert sorted(own[0] + own[1]) == [0, 1, 2, 3, 4]
    loads = sorted(sum(costs[j] for j in o) for o in own)
    assert loads == [11, 13]
    assert batching.assign(costs, 1) == [[0, 1, 2, 3, 4]]
    assert batching.assign([1], 3) == [[0], [], []]


def test_attack_many_validates_before_touching_a_device():
    import torch
    m = torch.nn.Linear(1, 1)
    with pytest.raises(ValueError):
        batching.attack_many("emb", [m], [torch.zeros(80, 10)], [], 0.1, 1)
    with pytest.raises(ValueError):
        batching.attack_many("e2e", [m], [torch.zeros(80, 10)], [torch.zeros(80, 10)], 0.1, 1)
    with pytest.raises(ValueError):
        batching.attack_many("pgd", [m], [], [], 0.1, 1)
    assert batching.attack_many("emb", [m], [], [], 0.1, 1) == []
