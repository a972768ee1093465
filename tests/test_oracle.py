"""CPU tests: the oracle against the reference's fixtures, known answers,
finite differences and the committed golden vectors."""

from __future__ import annotations

import json
import os

import numpy as np
import pytest

from _cases import hamming, int_cost, random_leaves, random_topologies, simulate_leaves, weird_children
from oracle.sankoff_ref import normalize_leaves, run_dp_ref, run_sankoff_ref, trex_children_table
from oracle.softmin_ref import batched_fwd_bwd_ref, sankoff_fwd_bwd_ref
from trex_amd.topology import adjacency_from_children

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _kat():
    with open(os.path.join(GOLDEN, "kat_sankoff.json")) as f:
        return json.load(f)


def test_kat_run_sankoff():
    k = _kat()
    adj = np.zeros((5, 5))
    for c, p in k["adjacency_edges"]:
        adj[c, p] = 1
    seqs = np.array(k["leaf_sequences"], dtype=np.float32)
    recon, dp, total = run_sankoff_ref(adj, np.array(k["cost"]), seqs, 5, 2, 3, return_path=True)
    assert total == np.float32(k["total"])
    np.testing.assert_array_equal(dp, np.array(k["dp"], dtype=np.float32))
    np.testing.assert_array_equal(recon, np.array(k["reconstructed"], dtype=np.float32))
    # reference assertions (tests/test_sankoff.py:68-72)
    assert recon.shape == (5, 2) and dp.shape == (2, 5, 2) and total >= 0
    o = sankoff_fwd_bwd_ref(trex_children_table(adj), normalize_leaves(seqs, 2),
                            np.array(k["cost"]), 0.0)
    np.testing.assert_array_equal(o["d_cost"], np.array(k["d_cost"]))


def test_kat_run_dp_fixture():
    k = _kat()["run_dp_fixture"]
    adj = np.array(k["adjacency"], dtype=np.float32)
    dp0 = np.full((1, 3, 2), 1e5, np.float32)
    bt0 = np.zeros((1, 3, 2, 4), np.float32)
    seqs = np.array(k["sequences"], dtype=np.float32)
    dp, bt = run_dp_ref(adj, dp0, bt0, seqs, np.array([[0, 1], [1, 0]], np.float32))
    assert dp[0, 0, 0] == 0 and dp[0, 1, 1] == 0  # tests/test_sankoff.py:35-36
    np.testing.assert_array_equal(dp[0], np.array(k["dp"], np.float32))
    np.testing.assert_array_equal(bt[0, 2], np.array(k["bt_row2"], np.float32))


def test_convergence_invariant_oracle():
    """tests/test_convergence.py:69-73 on a numpy-simulated 4x20x4 case."""
    seqs, adj = simulate_leaves(4, 20, 4, 3, seed=42)
    cost = hamming(4)
    recon, _, total = run_sankoff_ref(adj, cost, seqs[:4], 7, 4, 4, return_path=True)
    r = recon.astype(np.int64)
    parent = adj.argmax(axis=1)
    assert abs(total - cost[r[parent], r][:-1].sum()) < 1e-3


@pytest.mark.parametrize("case", ["random", "fwdref", "dag"])
def test_batched_oracle_equals_trex_mirror(case):
    if case == "random":
        ch = random_topologies(1, 16, seed=3)
    else:
        ch = weird_children(case)[None]
    n_all = ch.shape[1]
    nl = (n_all + 1) // 2
    leaves = random_leaves(1, nl, 33, 4, seed=1, missing=0.1)
    cost = int_cost(4, seed=2)
    o = batched_fwd_bwd_ref(ch, leaves, cost, 0.0)
    adj = adjacency_from_children(ch)[0]
    seqs = np.where(leaves[0] < 0, 99, leaves[0]).astype(np.float32)
    _, dp, total = run_sankoff_ref(adj, cost, seqs, n_all, 4, nl)
    np.testing.assert_array_equal(o["dp"][0].transpose(2, 0, 1).astype(np.float32), dp[:, nl:])
    assert np.float32(o["tree_score"][0]) == total


def _num_grad(fn, c, eps):
    g = np.zeros_like(c)
    for i in range(c.shape[0]):
        for j in range(c.shape[1]):
            cp = c.copy()
            cm = c.copy()
            cp[i, j] += eps
            cm[i, j] -= eps
            g[i, j] = (fn(cp) - fn(cm)) / (2 * eps)
    return g


@pytest.mark.parametrize("tau", [1.0, 0.2])
def test_softmin_gradient_finite_difference(tau):
    ch = random_topologies(1, 8, seed=4)[0]
    leaves = random_leaves(1, 8, 25, 4, seed=5)[0]
    rng = np.random.default_rng(6)
    cost = rng.uniform(0.2, 2.0, size=(4, 4))
    o = sankoff_fwd_bwd_ref(ch, leaves, cost, tau)
    num = _num_grad(lambda c: sankoff_fwd_bwd_ref(ch, leaves, c, tau)["tree_score"], cost, 1e-5)
    np.testing.assert_allclose(o["d_cost"], num, rtol=1e-6, atol=1e-8)


def test_hard_gradient_finite_difference_without_ties():
    ch = random_topologies(1, 8, seed=7)[0]
    leaves = random_leaves(1, 8, 25, 4, seed=8)[0]
    rng = np.random.default_rng(9)
    cost = rng.uniform(0.2, 2.0, size=(4, 4))  # generic: no ties
    o = sankoff_fwd_bwd_ref(ch, leaves, cost, 0.0)
    num = _num_grad(lambda c: sankoff_fwd_bwd_ref(ch, leaves, c, 0.0)["tree_score"], cost, 1e-7)
    np.testing.assert_allclose(o["d_cost"], num, rtol=1e-6, atol=1e-6)


def test_softmin_tends_to_hard():
    ch = random_topologies(1, 8, seed=10)[0]
    leaves = random_leaves(1, 8, 40, 4, seed=11)[0]
    rng = np.random.default_rng(12)
    cost = rng.uniform(0.2, 2.0, size=(4, 4))
    hard = sankoff_fwd_bwd_ref(ch, leaves, cost, 0.0)
    soft = sankoff_fwd_bwd_ref(ch, leaves, cost, 1e-4)
    assert abs(soft["tree_score"] - hard["tree_score"]) < 1e-2
    np.testing.assert_allclose(soft["d_cost"], hard["d_cost"], atol=1e-3)
    np.testing.assert_allclose(soft["marginals"], hard["marginals"], atol=1e-3)


def test_marginals_are_distributions():
    ch = random_topologies(1, 16, seed=13)[0]
    leaves = random_leaves(1, 16, 30, 4, seed=14)[0]
    o = sankoff_fwd_bwd_ref(ch, leaves, hamming(4), 0.5)
    np.testing.assert_allclose(o["marginals"].sum(axis=1), 1.0, rtol=1e-12)


def test_golden_fixtures_reproduce():
    import sys

    sys.path.insert(0, GOLDEN)
    import make_golden

    data = np.load(os.path.join(GOLDEN, "sankoff_cases.npz"))
    names = sorted(set(k.split("/")[0] for k in data.files))
    assert names
    for name in names:
        res = make_golden.compute(data[f"{name}/children"], data[f"{name}/leaves"],
                                  data[f"{name}/cost"])
        for key, val in res.items():
            np.testing.assert_array_equal(val, data[f"{name}/{key}"], err_msg=f"{name}/{key}")


@pytest.mark.parametrize("n_leaves", [8, 6, 10])
def test_exact_backtrack_restatement_agrees_with_topology_simulation(n_leaves):
    """oracle.backtrack_site_exact (the reference's stack machine step by
    step, sankoff.py:212-265) == backtrack_ref (DFS simulated once on the
    topology) on run_dp's tables, including n_leaves != (n_all+1)//2."""
    from oracle.sankoff_ref import backtrack_ref, backtrack_site_exact

    ch = random_topologies(1, 8, seed=n_leaves)[0]
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(n_leaves)
    L, Q = 40, 4
    seqs = rng.integers(0, Q, size=(8, L)).astype(np.float32)
    dp0 = np.full((L, 15, Q), 1e5, np.float32)
    bt0 = np.zeros((L, 15, Q, 4), np.float32)
    dp, bt = run_dp_ref(adj, dp0, bt0, seqs, int_cost(Q, seed=1))
    roots = dp[:, -1].argmin(axis=1).astype(np.int32)
    want = backtrack_ref(14, roots, bt, 15, n_leaves)
    for l in range(L):
        np.testing.assert_array_equal(backtrack_site_exact(14, roots[l], bt[l], 15, n_leaves),
                                      want[:, l])
