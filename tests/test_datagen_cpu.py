"""Host data generators (trex_amd.datagen) against the reference's own test
assertions (tests/test_ground_truth.py:15-68, tests/test_nk_model_new.py:36-87)
-- values differ from trex (numpy PCG64 instead of JAX threefry), the
processes and invariants are the reference's."""

from __future__ import annotations

import numpy as np
import pytest

from oracle.sankoff_ref import run_sankoff_ref
from trex_amd import datagen as D
from trex_amd.topology import create_balanced_binary_tree


@pytest.mark.parametrize("n_states,n_mutations,batch,seq_length", [(10, 5, 5, 8), (4, 2, 8, 4)])
def test_mutate(n_states, n_mutations, batch, seq_length):
    rng = np.random.default_rng(0)
    seq = rng.integers(0, n_states, size=(batch, seq_length))
    mutated = np.stack([D.mutate(rng, s, n_states, n_mutations) for s in seq])
    assert mutated.shape == (batch, seq_length)
    assert np.all((mutated >= 0) & (mutated < n_states))
    assert np.sum(mutated != seq) == n_mutations * batch


@pytest.mark.parametrize("n_leaves,seq_length,n_states,n_mutations",
                         [(4, 100, 20, 10), (8, 50, 4, 5)])
def test_generate_groundtruth(n_leaves, seq_length, n_states, n_mutations):
    t = D.generate_groundtruth(n_leaves, n_states, n_mutations, seq_length, seed=1)
    n_all = 2 * n_leaves - 1
    assert t.masked_sequences.shape == (n_all, seq_length)
    assert t.all_sequences.shape == (n_all, seq_length) and t.adjacency.shape == (n_all, n_all)
    assert np.all((t.adjacency == 0) | (t.adjacency == 1))
    assert np.all(t.adjacency[:, -1][-3:-1] == 1)
    assert np.any(t.masked_sequences[:n_leaves] != 0)
    assert np.all(t.masked_sequences[n_leaves:] == 0)
    assert np.sum(t.adjacency[:, -1]) == 2 and t.adjacency[-1, -1] == 0
    # every edge carries exactly n_mutations substitutions
    par = np.argmax(t.adjacency[:-1], axis=1)
    d = (t.all_sequences[:-1] != t.all_sequences[par]).sum(1)
    assert np.all(d == n_mutations)
    with pytest.raises(ValueError):
        D.generate_groundtruth(6, n_states, n_mutations, seq_length)


def test_groundtruth_feeds_sankoff_lower_bound():
    """The Sankoff score of the generated leaves is at most the cost of the
    true ancestral labelling (unit costs: n_mutations per edge)."""
    n_leaves, L, Q, m = 16, 200, 4, 5
    t = D.generate_groundtruth(n_leaves, Q, m, L, seed=3)
    n_all = 2 * n_leaves - 1
    cost = (np.ones((Q, Q)) - np.eye(Q)).astype(np.float32)
    _, _, total = run_sankoff_ref(t.adjacency, cost, t.masked_sequences[:n_leaves], n_all, Q,
                                  n_leaves)
    assert 0 < total <= m * (n_all - 1)


def test_nk_landscape_and_fitness():
    land = D.create_nk_model_landscape(20, 2, seed=0, n_states=4)
    assert land["interactions"].shape == (20, 2) and land["fitness_tables"].shape == (20, 64)
    seq = np.random.default_rng(1).integers(0, 4, size=20)
    f = D.get_fitness(seq, land)
    idx = seq + 4 * seq[land["interactions"][:, 0]] + 16 * seq[land["interactions"][:, 1]]
    assert f == pytest.approx(float(land["fitness_tables"][np.arange(20), idx].mean()), rel=1e-6)


def test_generate_tree_data_branch_length_and_defaults():
    land = D.create_nk_model_landscape(20, 2, seed=42, n_states=4)
    adj = create_balanced_binary_tree(16)
    root = np.random.default_rng(5).integers(0, 4, size=20)

    def mean_dist(bl):
        t = D.generate_tree_data(land, adj, root[:, None], 0.05, seed=101, branch_length=bl)
        return float(np.mean(t.all_sequences != root[None, :]))

    assert mean_dist(10) > mean_dist(1)
    a = D.generate_tree_data(land, adj, root[:, None], 0.05, seed=7)
    b = D.generate_tree_data(land, adj, root[:, None], 0.05, seed=7, mutation_rate_noise_std=0.0,
                             branch_length=1)
    assert np.array_equal(a.all_sequences, b.all_sequences)
