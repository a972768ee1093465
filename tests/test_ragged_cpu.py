"""Ragged plan builder (host C++, trex_ragged_plan_build): offsets, work-item
table and per-tree programs equal the uniform planner's per tree."""

from __future__ import annotations

import numpy as np
import pytest

from trex_amd import TreePlan, random_topologies
from trex_amd._lib import TREX_PLAN_HEADER_INTS, TrexError
from trex_amd.ragged import RaggedTreePlan, from_padded
from trex_amd.topology import create_balanced_binary_tree


def test_ragged_plan_layout_matches_uniform_plans():
    sizes = [(5, 100), (9, 64), (32, 130), (2, 1)]
    chs = [random_topologies(1, n, seed=n)[0] for n, _ in sizes]
    p = RaggedTreePlan(chs, [L for _, L in sizes])
    n_all = np.array([2 * n - 1 for n, _ in sizes])
    nl, ni = (n_all + 1) // 2, n_all - (n_all + 1) // 2
    Ls = np.array([L for _, L in sizes])
    assert p.items == int(((Ls + 63) // 64).sum())
    assert p.leaf_bytes == int((nl * Ls).sum()) and p.row_sites == int((ni * Ls).sum())
    assert p.sites == int(Ls.sum()) and p.steps == int(ni.sum())
    np.testing.assert_array_equal(p.leaf_offsets, np.concatenate([[0], np.cumsum(nl * Ls)[:-1]]))
    np.testing.assert_array_equal(p.row_offsets, np.concatenate([[0], np.cumsum(ni * Ls)[:-1]]))
    h = TREX_PLAN_HEADER_INTS
    meta = p.host[h:h + 12 * p.B].reshape(p.B, 12)
    ritem = p.host[h + 12 * p.B:h + 12 * p.B + p.items]
    steps = p.host[h + 12 * p.B + p.items:h + 12 * p.B + p.items + 4 * p.steps].reshape(-1, 4)
    np.testing.assert_array_equal(ritem, np.repeat(np.arange(p.B), (Ls + 63) // 64))
    for b, ch in enumerate(chs):
        u = TreePlan(ch[None])
        off = meta[b, 0]
        np.testing.assert_array_equal(steps[off:off + ni[b]], u.fwd_steps[0])
        assert meta[b, 1] == ni[b] and meta[b, 2] == nl[b] and meta[b, 3] == Ls[b]
    assert p.n_slots == max(TreePlan(c[None]).n_slots for c in chs)


def test_ragged_plan_rejects_bad_trees():
    with pytest.raises(ValueError):
        RaggedTreePlan([np.full((2, 2), -1, np.int32)], [10])  # n_all < 3
    bad = random_topologies(1, 4, seed=0)[0].copy()
    bad[-1, 0] = 99  # child id out of range
    with pytest.raises(TrexError):
        RaggedTreePlan([bad], [10])


def test_from_padded_shapes_and_leaf_conversion():
    Q, MAX, NB = 4, 63, 64
    A = np.zeros((2, MAX, MAX), np.float32)
    nm = np.zeros((2, MAX), bool)
    S = np.zeros((2, 8, NB), np.float32)
    sm = np.zeros((2, NB), bool)
    for b, (nl, L) in enumerate([(4, 10), (8, 64)]):
        A[b, :2 * nl - 1, :2 * nl - 1] = create_balanced_binary_tree(nl)
        nm[b, :2 * nl - 1] = True
        sm[b, :L] = True
    S[0, 0, :3] = [-1.0, 4.0, 2.7]  # wraps to 3, dropped (-1 code), truncates to 2
    plan, packed, shapes = from_padded(A, nm, S, sm, Q)
    assert shapes == [(7, 10), (15, 64)]
    assert list(packed[:3]) == [3, -1, 2]
    bad = nm.copy()
    bad[0, 2] = False
    with pytest.raises(ValueError):
        from_padded(A, bad, S, sm, Q)
