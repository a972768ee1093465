"""Host checks of the NK tree-evolution restatement behind the device
generator (oracle/datagen_ref.generate_tree_data, trex_datagen_nk_tree):
the traversal of trex's generate_tree_data (src/trex/nk_model.py:149-190,
including its -1 BFS-slot quirk on adjacencies without a self-parented
root) and the process invariants.  The random numbers are the device's
counter-based draws, not JAX's, so values are compared only with the device
(tests/test_datagen_gpu.py)."""

from __future__ import annotations

import numpy as np

from oracle.datagen_ref import generate_tree_data
from trex_amd.datagen import bfs_levels, create_nk_model_landscape, get_fitness
from trex_amd.topology import create_balanced_binary_tree


def _rooted_balanced(nl):
    adj = create_balanced_binary_tree(nl).copy()
    adj[-1, -1] = 1  # self-parented root: the BFS reaches every node
    return adj


def test_bfs_levels_rooted_tree():
    root, parent, order, offs = bfs_levels(_rooted_balanced(8))
    assert root == 14 and order[0] == 14 and sorted(order.tolist()) == list(range(15))
    assert offs.tolist() == [0, 1, 3, 7, 15]
    pos = {int(v): i for i, v in enumerate(order)}
    for v in range(14):
        assert pos[int(parent[v])] < pos[v]


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
