"""Device data generators (trex_amd/csrc/datagen.hip) vs their CPU
restatement (oracle/datagen_ref.py), bit for bit at small sizes, and trex's
generate_groundtruth invariants (src/trex/ground_truth.py:20-52, 112-197)
at C5 size (256 leaves x 10 000 sites): zero root, exactly n_mutations
changed sites on every edge, states in [0, Q)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle.datagen_ref import generate_groundtruth as gt_ref
from oracle.datagen_ref import uniform_states as us_ref
from trex_amd.datagen import generate_groundtruth_device, uniform_states_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nl,L,Q,mut", [(2, 5, 4, 1), (8, 100, 4, 5), (16, 257, 20, 50),
                                        (4, 10, 4, 10), (32, 1000, 61, 7), (4, 20, 4, 0)])
def test_groundtruth_device_matches_restatement(device, nl, L, Q, mut):
    s, adj = generate_groundtruth_device(nl, Q, mut, L, seed=9, device=device)
    np.testing.assert_array_equal(s.cpu().numpy(), gt_ref(9, nl, L, Q, mut))
    assert adj.shape == (2 * nl - 1, 2 * nl - 1) and adj.sum() == 2 * nl - 2


def test_groundtruth_device_invariants_c5_size(device):
    nl, L, Q, mut = 256, 10000, 4, 5
    s, _ = generate_groundtruth_device(nl, Q, mut, L, seed=6, device=device)
    s2, _ = generate_groundtruth_device(nl, Q, mut, L, seed=6, device=device)
    assert torch.equal(s, s2)
    s = s.long()
    assert int(s.min()) >= 0 and int(s.max()) < Q and not bool(s[-1].any())
    parent = nl + torch.arange(2 * nl - 2, device=device) // 2
    changed = (s[:-1] != s[parent]).sum(1)
    assert bool((changed == mut).all())


@pytest.mark.parametrize("n,Q", [(1, 4), (1000, 4), (65537, 20), (300000, 61)])
def test_uniform_states_device_matches_restatement(device, n, Q):
    x = uniform_states_device((n,), Q, seed=3, device=device)
    np.testing.assert_array_equal(x.cpu().numpy(), us_ref(3, n, Q))


def test_uniform_states_device_c4_size(device):
    x = uniform_states_device((1024, 32, 5000), 4, seed=4, device=device)
    frac = torch.bincount(x.view(-1).long(), minlength=4).double() / x.numel()
    assert float((frac - 0.25).abs().max()) < 1e-3
    tail = x.view(-1)[-4096:].cpu().numpy()
    np.testing.assert_array_equal(tail, us_ref(4, x.numel(), 4, start=x.numel() - 4096))
