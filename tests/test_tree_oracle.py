"""CPU tests of the tree-cost oracle: the reference's own assertions
(tests/test_tree.py:18-87), hand identities, and finite-difference checks of
every analytic gradient the GPU path reproduces."""

from __future__ import annotations

import numpy as np
import pytest

from oracle import tree_ref as T


def test_reference_tree_fixtures():
    # tests/test_tree.py:18-25
    soft = np.array([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.3, 0.3, 0.4]])
    oh = T.discretize_tree_topology(soft, 3)
    assert oh.shape == (3, 3) and np.all(oh.sum(1) == 1)
    np.testing.assert_array_equal(oh.argmax(1), [1, 0, 2])
    # :28-32 update_tree rows sum to 1
    out = T.update_tree(np.ones((2, 1)), noise=np.zeros((2, 1)))
    assert out.shape == (3, 3) and np.allclose(out.sum(1), 1)
    # :35-38 no ancestors -> identity
    assert T.update_tree(np.ones((1, 0))).shape == (2, 2)
    # :48-51 constraint on eye(5) is non-negative
    assert T.enforce_graph_constraints(np.eye(5), 10.0) >= 0
    # :54-61 surrogate on one-hot, eye(2): self edges -> 0
    seqs = np.eye(4)[np.array([[0, 1, 2], [3, 2, 1]])]
    assert T.compute_surrogate_cost(seqs, np.eye(2)) == 0.0
    # :64-70 compute_cost, eye(3) parents = self -> 0
    s3 = np.eye(2)[np.array([[0, 1], [1, 0], [0, 0]])]
    assert T.compute_cost(s3, np.eye(3), np.ones((2, 2)) - np.eye(2)) == 0.0


def test_constraint_value_eye5():
    # n=5 -> n_anc=2: columns 3, 4 over rows 0..3 of eye(5) sum to 1 and 0
    assert T.enforce_graph_constraints(np.eye(5), 10.0) == 10.0 * ((1 - 2) ** 2 + (0 - 2) ** 2)


def test_surrogate_equals_edge_hamming_for_onehot():
    rng = np.random.default_rng(0)
    n, L, Q = 7, 30, 4
    seq = rng.integers(0, Q, size=(n, L))
    S = np.eye(Q)[seq]
    parent = np.array([4, 4, 5, 5, 6, 6, 6])
    A = np.eye(n)[parent]
    A[-1] = 0
    ham = sum((seq[i] != seq[parent[i]]).sum() for i in range(n - 1))
    assert T.compute_surrogate_cost(S, A) == ham
    C = np.ones((Q, Q)) - np.eye(Q)
    A2 = np.eye(n)[parent]
    assert T.compute_cost(S, A2, C) == ham


def _fd(f, x, eps=1e-6):
    g = np.zeros_like(x)
    it = np.nditer(x, flags=["multi_index"])
    for _ in it:
        idx = it.multi_index
        xp = x.copy()
        xm = x.copy()
        xp[idx] += eps
        xm[idx] -= eps
        g[idx] = (f(xp) - f(xm)) / (2 * eps)
    return g


def test_surrogate_grads_finite_difference():
    rng = np.random.default_rng(1)
    n, L, Q = 5, 3, 4
    S = rng.random((n, L, Q))
    A = rng.random((n, n))
    _, dS, dA = T.compute_surrogate_cost_grads(S, A)
    np.testing.assert_allclose(dS, _fd(lambda s: T.compute_surrogate_cost(s, A), S), rtol=1e-6,
                               atol=1e-8)
    np.testing.assert_allclose(dA, _fd(lambda a: T.compute_surrogate_cost(S, a), A), rtol=1e-6,
                               atol=1e-8)


@pytest.mark.parametrize("fix", ["none", "seqs", "tree"])
def test_compute_loss_grads_finite_difference(fix):
    rng = np.random.default_rng(2)
    nl, L, Q = 4, 3, 4
    n = 2 * nl - 1
    n_anc = nl - 1
    params = {"tree_params": rng.normal(size=(n - 1, n_anc)),
              "ancestors": rng.normal(size=(n_anc, L, Q))}
    noise = rng.gumbel(size=(n - 1, n_anc))
    seqs = np.zeros((n, L, Q))
    seqs[:nl] = np.eye(Q)[rng.integers(0, Q, size=(nl, L))]
    adj = np.eye(n)[np.array([4, 4, 5, 5, 6, 6, 6])]
    kw = dict(fix_seqs=fix == "seqs", fix_tree=fix == "tree")
    if fix == "seqs":
        seqs = T.update_seq(params["ancestors"], seqs, 0.7)
    T_ = 0.7
    _, g = T.compute_loss(noise, params, seqs, T_, adj, **kw)
    for key in ("tree_params", "ancestors"):
        def f(x, key=key):
            p = dict(params)
            p[key] = x
            return T.compute_loss(noise, p, seqs, T_, adj, **kw)[0]

        np.testing.assert_allclose(g[key], _fd(f, params[key]), rtol=1e-5, atol=1e-7)


def test_adam_matches_closed_form_first_steps():
    p = {"x": np.array([1.0, -2.0])}
    st = T.adam_init(p)
    g = {"x": np.array([0.5, -0.25])}
    upd, st = T.adam_update(g, st, lr=0.01)
    # first Adam step: mu_hat = g, nu_hat = g^2 -> -lr * sign(g) (up to eps)
    np.testing.assert_allclose(upd["x"], -0.01 * np.sign(g["x"]), rtol=1e-7)
    upd2, _ = T.adam_update(g, st, lr=0.01)
    np.testing.assert_allclose(upd2["x"], -0.01 * np.sign(g["x"]), rtol=1e-7)
    # clipping
    big = {"x": np.array([30.0, 40.0])}
    u, _ = T.adam_update(big, T.adam_init(p), lr=1.0, clip_norm=1.0)
    np.testing.assert_allclose(u["x"], [-1.0, -1.0], rtol=1e-7)


def test_optax_oracle_adam_matches_adam_update():
    """The generic optax restatement reduces to adam_update for "adam"."""
    rng = np.random.default_rng(0)
    p = {"a": rng.normal(size=(3, 4))}
    st1, st2 = T.adam_init(p), T.optax_init(p)
    for _ in range(3):
        g = {"a": rng.normal(size=(3, 4))}
        u1, st1 = T.adam_update(g, st1, 0.01, clip_norm=1.0)
        u2, st2 = T.optax_update("adam", g, st2, p, 0.01, clip_norm=1.0)
        np.testing.assert_allclose(u1["a"], u2["a"], rtol=1e-12)
