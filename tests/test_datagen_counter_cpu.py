"""Host checks of the device data generators' CPU restatement
(oracle/datagen_ref.py) against the invariants trex's generate_groundtruth
holds (src/trex/ground_truth.py:20-52, 112-197): zero root, every edge
changes exactly n_mutations distinct sites, states in [0, Q), balanced
numbering.  Random numbers differ from trex's threefry by design, so the
data are compared through these properties ("parity unpinned" for the raw
draws; the device generator is pinned to this restatement bit for bit in
tests/test_datagen_gpu.py)."""

from __future__ import annotations

import numpy as np
import pytest

from oracle.datagen_ref import draw, generate_groundtruth, mix64, uniform_states
from trex_amd.topology import create_balanced_binary_tree


def test_mix64_known_values():
    # splitmix64 from state 0: first outputs of the published generator
    # (state += golden gamma, then the finaliser) -- mix64 is that finaliser
    # with the increment folded in
    assert int(mix64(0)) == 0xE220A8397B1DCDAF
    assert int(mix64(0x9E3779B97F4A7C15)) == 0x6E789E6AA1B965F4


def test_draw_is_pure_function_of_indices():
    a = draw(7, np.arange(10), np.arange(10))
    b = np.array([int(draw(7, s, s)) for s in range(10)], dtype=np.uint64)
    np.testing.assert_array_equal(a, b)
    assert len(set(a.tolist())) == 10


@pytest.mark.parametrize("nl,L,Q,mut", [(2, 5, 4, 1), (8, 100, 4, 5), (16, 257, 20, 50),
                                        (4, 10, 4, 10), (8, 30, 2, 3), (4, 20, 61, 0)])
def test_groundtruth_invariants(nl, L, Q, mut):
    s = generate_groundtruth(3, nl, L, Q, mut).astype(np.int64)
    n_all = 2 * nl - 1
    assert s.shape == (n_all, L) and s.min() >= 0 and s.max() < Q
    assert not s[-1].any()
    adj = create_balanced_binary_tree(nl)
    for c in range(n_all - 1):
        p = int(np.argmax(adj[c]))
        assert p == nl + c // 2
        assert int((s[c] != s[p]).sum()) == mut
    again = generate_groundtruth(3, nl, L, Q, mut)
    np.testing.assert_array_equal(again, s.astype(np.int8))
    if mut:
        assert not np.array_equal(generate_groundtruth(4, nl, L, Q, mut), again)


def test_mutation_offsets_cover_all_nonzero_shifts():
    s = generate_groundtruth(11, 64, 400, 5, 40).astype(np.int64)
    nl = 64
    shifts = set()
    for c in range(2 * nl - 2):
        d = (s[c] - s[nl + c // 2]) % 5
        shifts |= set(d[d != 0].tolist())
    assert shifts == {1, 2, 3, 4}


def test_uniform_states_range_and_balance():
    x = uniform_states(5, 200000, 4).astype(np.int64)
    assert x.min() == 0 and x.max() == 3
    frac = np.bincount(x, minlength=4) / x.size
    assert np.all(np.abs(frac - 0.25) < 0.01)
