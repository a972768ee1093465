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


def _adjacency(nl, kind):
    """"root0": balanced tree relabelled so the self-parented root is node 0
    (the reference's BFS then reaches every node); "last": root n - 1 with a
    self-loop (the reference's 0-padded child lists overflow its queue, some
    nodes are never evolved, the -1 slots re-evolve the root); "none": no
    self-parented node (BFS rooted at node 0 by the jnp.where fill)."""
    from trex_amd.topology import create_balanced_binary_tree

    adj = create_balanced_binary_tree(nl).copy()
    n = adj.shape[0]
    if kind == "root0":
        perm = np.arange(n)
        perm[[0, n - 1]] = [n - 1, 0]
        adj = adj[np.ix_(perm, perm)]
        adj[0, 0] = 1
    elif kind == "last":
        adj[-1, -1] = 1
    return adj


@pytest.mark.parametrize("nl,L,Q,K,rate,std,cp,bl,kind", [
    (8, 64, 4, 2, 0.1, 0.0, 0.5, 1, "root0"),
    (16, 300, 4, 4, 0.05, 0.3, 0.5, 3, "root0"),
    (8, 50, 20, 2, 0.2, 0.0, 0.0, 2, "root0"),
    (4, 40, 2, 3, 0.1, 0.0, 1.0, 5, "root0"),
    (8, 64, 4, 2, 0.1, 0.0, 0.5, 1, "none"),   # the reference's -1 slot quirk
    (8, 64, 4, 2, 0.3, 0.0, 0.5, 2, "last"),   # queue overflow, root re-evolved
    (32, 2000, 4, 4, 0.02, 0.5, 0.5, 2, "root0"),
])
def test_nk_tree_device_matches_restatement(device, nl, L, Q, K, rate, std, cp, bl, kind):
    """trex_datagen_nk_tree (generate_tree_data's process, nk_model.py:
    116-278) equals its CPU restatement bit for bit: same draws, fixed-point
    fitness sums, the reference's traversal (oracle.datagen_ref.
    evolve_order_ref, independent of the device's level planner) incl. the
    -1 tail and the dropped enqueues."""
    from oracle.datagen_ref import evolve_order_ref
    from oracle.datagen_ref import generate_tree_data as nk_ref
    from trex_amd.datagen import create_nk_model_landscape, generate_tree_data_device

    ls = create_nk_model_landscape(L, K, seed=nl + L, n_states=Q)
    adj = _adjacency(nl, kind)
    rs = np.random.default_rng(L).integers(0, Q, L)
    got = generate_tree_data_device(ls, adj, rs, rate, seed=21, coupled_mutation_prob=cp,
                                    mutation_rate_noise_std=std, branch_length=bl,
                                    device=device).cpu().numpy()
    _, parent, order = evolve_order_ref(adj)
    ref = nk_ref(21, ls["interactions"], ls["fitness_tables"], parent, order, rs, Q, rate, std, cp,
                 bl)
    np.testing.assert_array_equal(got, ref)
    assert got.min() >= 0 and got.max() < Q
