"""Host checks of the NK tree-evolution restatement behind the device
generator (oracle/datagen_ref.generate_tree_data, trex_datagen_nk_tree):
the traversal of trex's generate_tree_data (src/trex/nk_model.py:149-190,
including its -1 BFS-slot quirk on adjacencies without a self-parented
root) and the process invariants.  The random numbers are the device's
counter-based draws, not JAX's, so values are compared only with the device
(tests/test_datagen_gpu.py)."""

from __future__ import annotations

import numpy as np

import pytest

from oracle.datagen_ref import evolve_order_ref, generate_tree_data, sorted_nodes_ref
from trex_amd import datagen as D
from trex_amd.datagen import bfs_levels, create_nk_model_landscape, get_fitness
from trex_amd.topology import create_balanced_binary_tree


def _rooted_balanced(nl):
    """Balanced tree with its root relabelled 0 and self-parented: the
    reference's BFS pads child lists with node 0 (nk_model.py:170), which is
    then already visited, so the traversal is a plain BFS over every node."""
    adj = create_balanced_binary_tree(nl).copy()
    n = adj.shape[0]
    perm = np.arange(n)
    perm[[0, n - 1]] = [n - 1, 0]
    adj = adj[np.ix_(perm, perm)]
    adj[0, 0] = 1
    return adj


def _self_looped_last_root(nl):
    """The root at n - 1 with a self-loop (advisor's case): the 0 pads
    enqueue node 0 repeatedly, the fixed queue overflows, later children
    are dropped."""
    adj = create_balanced_binary_tree(nl).copy()
    adj[-1, -1] = 1
    return adj


def test_bfs_levels_rooted_tree():
    root, parent, order, offs = bfs_levels(_rooted_balanced(8))
    assert root == 0 and order[0] == 0 and sorted(order.tolist()) == list(range(15))
    assert offs.tolist() == [0, 1, 3, 7, 15]
    pos = {int(v): i for i, v in enumerate(order)}
    for v in range(1, 15):
        assert pos[int(parent[v])] < pos[v]


def test_reference_bfs_self_looped_last_root():
    """7-node balanced tree, adj[6, 6] = 1: the reference's traversal is
    [6, 4, 5, 0, 1, 2, -1] -- node 3's enqueue falls past the full queue and
    is dropped, the -1 slot re-evolves row 6 (the root) from itself."""
    adj = _self_looped_last_root(4)
    root, parent, sn = sorted_nodes_ref(adj)
    assert root == 6 and sn.tolist() == [6, 4, 5, 0, 1, 2, -1]
    r2, p2, sn2 = D.reference_sorted_nodes(adj)
    assert r2 == root and np.array_equal(p2, parent) and np.array_equal(sn2, sn)
    root, parent, order, offs = bfs_levels(adj)
    assert order.tolist() == [6, 4, 5, 0, 1, 2, 6] and offs.tolist() == [0, 1, 3, 7]
    # host generator: node 3 never evolves (stays 0), the root is re-evolved
    ls = create_nk_model_landscape(20, 2, seed=3, n_states=4)
    rs = np.full((20, 1), 3)
    t = D.generate_tree_data(ls, adj, rs, 0.9, seed=5, coupled_mutation_prob=0.0, n_states=4)
    seqs = t.all_sequences
    assert np.all(seqs[3] == 0) and np.any(seqs[0] != 0)


def _random_adjacency(rng, n):
    """Random parent pointers (some nodes self-parented, some rows empty,
    occasional extra edges): every reference BFS path gets exercised."""
    A = np.zeros((n, n), np.float32)
    for v in range(n):
        u = rng.random()
        if u < 0.1:
            A[v, v] = 1
        elif u < 0.9:
            A[v, rng.integers(0, n)] = 1
    for _ in range(rng.integers(0, 3)):
        A[rng.integers(0, n), rng.integers(0, n)] = 1
    return A


@pytest.mark.parametrize("seed", range(40))
def test_reference_bfs_restatements_agree_and_levels_are_sequential(seed):
    """trex_amd.datagen.reference_sorted_nodes == the oracle's independent
    restatement, and bfs_levels' parallel levels reproduce sequential slot
    order: each slot writes f(its parent's current row, slot)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 40))
    A = _random_adjacency(rng, n)
    root, parent, sn = sorted_nodes_ref(A)
    r2, p2, sn2 = D.reference_sorted_nodes(A)
    assert r2 == root and np.array_equal(p2, parent) and np.array_equal(sn2, sn)
    root, parent, order, offs = bfs_levels(A)
    _, _, order_ref = evolve_order_ref(A)
    assert np.array_equal(order, order_ref) and order[0] == root
    seq = [("root" if v == root else 0) for v in range(n)]
    for slot in range(1, n):
        v = int(order[slot])
        seq[v] = (seq[int(parent[v])], slot)
    lvl = [("root" if v == root else 0) for v in range(n)]
    assert offs[0] == 0 and offs[1] == 1 and offs[-1] == n and np.all(np.diff(offs) > 0)
    for lo, hi in zip(offs[1:-1], offs[2:]):
        reads = {slot: lvl[int(parent[order[slot]])] for slot in range(lo, hi)}
        for slot in range(lo, hi):
            lvl[int(order[slot])] = (reads[slot], slot)
    assert lvl == seq


def test_bfs_levels_reference_quirk_without_root():
    """create_balanced_binary_tree has no self-parented node: the reference
    roots the BFS at node 0 (the jnp.where fill), reaches nothing, and its
    -1 slots re-evolve the last node n_nodes - 1 from its argmax parent."""
    root, parent, order, offs = bfs_levels(create_balanced_binary_tree(4))
    assert root == 0 and order.tolist() == [0] + [6] * 6
    assert offs.tolist() == list(range(8)) and parent[6] == 0


def test_rate_zero_independent_mutations_copy_the_parent():
    ls = create_nk_model_landscape(30, 2, seed=3, n_states=4)
    root, parent, order, _ = bfs_levels(_rooted_balanced(8))
    rs = np.random.default_rng(0).integers(0, 4, 30)
    s = generate_tree_data(7, ls["interactions"], ls["fitness_tables"], parent, order, rs, 4, 0.0,
                           0.0, 0.0, 3)
    assert np.all(s == rs.astype(np.int8))


def test_coupled_mutations_touch_only_a_site_and_its_interactions():
    ls = create_nk_model_landscape(40, 3, seed=4, n_states=4)
    root, parent, order, _ = bfs_levels(_rooted_balanced(16))
    rs = np.random.default_rng(1).integers(0, 4, 40)
    s = generate_tree_data(9, ls["interactions"], ls["fitness_tables"], parent, order, rs, 4, 0.3,
                           0.0, 1.0, 1).astype(np.int64)
    assert np.all(s[root] == rs) and s.min() >= 0 and s.max() < 4
    inter = np.asarray(ls["interactions"])
    for v in order[1:]:
        d = np.nonzero(s[v] != s[parent[v]])[0]
        if d.size:  # accepted: the changed sites lie in one {site} + interactions set
            assert any(set(d.tolist()) <= {i, *inter[i].tolist()} for i in range(40))


def test_metropolis_prefers_fitter_sequences():
    """Long branches drift uphill: mean child fitness exceeds the root's."""
    ls = create_nk_model_landscape(50, 2, seed=5, n_states=4)
    root, parent, order, _ = bfs_levels(_rooted_balanced(16))
    rs = np.random.default_rng(2).integers(0, 4, 50)
    s = generate_tree_data(11, ls["interactions"], ls["fitness_tables"], parent, order, rs, 4, 0.1,
                           0.3, 0.5, 20)
    f_root = get_fitness(rs, ls)
    f_leaves = np.mean([get_fitness(s[v], ls) for v in range(16)])
    assert f_leaves > f_root


def test_device_generator_validates_indices_on_the_host():
    """trex_datagen_nk_tree indexes LDS and the fitness table with the
    interactions and states: out-of-range input is refused before any
    device work (no GPU needed to reach the check)."""
    ls = create_nk_model_landscape(10, 2, seed=1, n_states=4)
    adj = _rooted_balanced(4)
    bad = dict(ls, interactions=np.where(ls["interactions"] == 0, 10, ls["interactions"]))
    bad["interactions"][0, 0] = 10
    with pytest.raises(ValueError, match="interactions"):
        D.generate_tree_data_device(bad, adj, np.zeros(10, np.int64), 0.1, device="cpu")
    with pytest.raises(ValueError, match="root_sequence"):
        D.generate_tree_data_device(ls, adj, np.full(10, 4), 0.1, device="cpu")
    with pytest.raises(ValueError, match="fitness_tables"):
        D.generate_tree_data_device(dict(ls, fitness_tables=ls["fitness_tables"][:, :5]), adj,
                                    np.zeros(10, np.int64), 0.1, device="cpu")
