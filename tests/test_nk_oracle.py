"""CPU checks of the NK landscape-aware oracle (oracle/nk_ref.py) and the
host planner (trex_nk_plan_build).

Pinning: the reference has no test of compute_parental_logits or the
landscape-aware loss (tests/test_nk_model_new.py covers the data generator
only), so the oracle is pinned by (i) a known-answer check derived from the
reference's definition -- for one-hot parents the logits are the fitness
table entries at index s * Q^k + sum_j c_j Q^(k-1-j) (benchmark.py:637-650),
(ii) the K = 0 broadcast (:616-620), (iii) central differences for the
gradient.  Beyond that, parity is unpinned (no JAX here).
"""

from __future__ import annotations

import numpy as np
import pytest

from oracle import nk_ref as nk


def _case(n_leaves, L, Q, k, seed, mask=False):
    rng = np.random.default_rng(seed)
    n_all = 2 * n_leaves - 1
    inter, F = nk.random_landscape(L, k, Q, seed=seed + 1)
    leaves = rng.integers(0, Q, size=(n_leaves, L))
    S0 = np.zeros((n_all, L, Q))
    S0[np.arange(n_leaves)[:, None], np.arange(L)[None, :], leaves] = 1.0
    A = np.zeros((n_all, n_all))
    par = n_leaves + np.arange(n_all - 1) // 2  # create_balanced_binary_tree numbering
    A[np.arange(n_all - 1), par] = 1.0
    anc = rng.normal(size=(n_all - n_leaves, L, Q))
    m = (rng.random(L) > 0.25) if mask else None
    return dict(S0=S0, A=A, inter=inter, F=F, anc=anc, mask=m, n_leaves=n_leaves)


@pytest.mark.parametrize("Q,k", [(2, 3), (4, 2), (3, 1)])
def test_parental_logits_one_hot_known_answer(Q, k):
    L, P = 7, 5
    rng = np.random.default_rng(Q * 10 + k)
    inter, F = nk.random_landscape(L, k, Q, seed=3)
    states = rng.integers(0, Q, size=(P, L))
    seqs = np.eye(Q)[states]
    out = nk.compute_parental_logits(seqs, inter, F, real_k=k)
    for p in range(P):
        for i in range(L):
            idx = 0
            for j in range(k):
                idx = idx * Q + states[p, inter[i, j]]
            for s in range(Q):
                assert out[p, i, s] == F[i, s * Q ** k + idx]


def test_parental_logits_k0_broadcast():
    L, Q = 6, 4
    F = np.random.default_rng(0).uniform(size=(L, Q))
    seqs = np.random.default_rng(1).dirichlet(np.ones(Q), size=(3, L))
    out = nk.compute_parental_logits(seqs, np.zeros((L, 0), np.int32), F, real_k=0)
    np.testing.assert_array_equal(out, np.broadcast_to(F, (3, L, Q)))


@pytest.mark.parametrize("Q,k,mask", [(3, 2, False), (4, 1, True), (2, 3, True)])
def test_landscape_loss_grad_central_differences(Q, k, mask):
    c = _case(4, 5, Q, k, seed=Q + k, mask=mask)
    args = (c["S0"], c["n_leaves"], c["inter"], c["F"], c["A"], 0.7, k, 1.3, c["mask"])
    loss, g = nk.landscape_loss_grad(c["anc"], *args)
    fd = np.zeros_like(c["anc"])
    eps = 1e-6
    for idx in np.ndindex(c["anc"].shape):
        a = c["anc"].copy()
        a[idx] += eps
        lp = nk.landscape_loss(a, *args)[0]
        a[idx] -= 2 * eps
        lm = nk.landscape_loss(a, *args)[0]
        fd[idx] = (lp - lm) / (2 * eps)
    np.testing.assert_allclose(g, fd, rtol=1e-6, atol=1e-8)


def test_lambda_zero_is_surrogate():
    c = _case(4, 5, 4, 2, seed=9)
    S = nk.update_seq_stacked(c["anc"], c["S0"], 4)
    loss, parts = nk.landscape_loss(c["anc"], c["S0"], 4, c["inter"], c["F"], c["A"], 0.0, 2)
    assert loss == nk.surrogate_cost(S, c["A"]) and parts["fitness"] == 0.0


def test_nk_plan_build_layout():
    """trex_nk_plan_build (host C++): distinct parents, child CSR, inverse
    interaction CSR in ascending (site, j) order."""
    from trex_amd._lib import lib, ptr

    L_ = lib()
    rng = np.random.default_rng(5)
    N, L, k = 9, 11, 3
    parent = np.array([5, 5, 6, 6, 7, 7, 8, 8, 0], np.int32)  # root row all-zero -> argmax 0
    inter = rng.integers(0, L, size=(L, k)).astype(np.int32)
    plan = np.zeros(int(L_.trex_nk_plan_ints(N, L, k)), np.int32)
    info = np.zeros(2, np.int32)
    assert L_.trex_nk_plan_build(ptr(parent), N, ptr(inter), L, k, ptr(plan), ptr(info)) == 0
    nP, nonroot = info
    assert nP == 5 and nonroot == 9
    h = 16
    prow = plan[h:h + N][:nP]
    cofs = plan[h + N:h + 2 * N + 1][:nP + 1]
    cidx = plan[h + 2 * N + 1:h + 3 * N + 1]
    rowmap = plan[h + 3 * N + 1:h + 4 * N + 1]
    iofs = plan[h + 4 * N + 1:h + 4 * N + 1 + L + 1]
    ient = plan[h + 4 * N + 1 + L + 1:]
    assert list(prow) == [0, 5, 6, 7, 8]
    for pc, p in enumerate(prow):
        assert list(cidx[cofs[pc]:cofs[pc + 1]]) == [n for n in range(N) if parent[n] == p]
        assert rowmap[p] == pc
    assert all(rowmap[r] == -1 for r in range(N) if r not in prow)
    flat = inter.reshape(-1)
    for m in range(L):
        assert list(ient[iofs[m]:iofs[m + 1]]) == [t for t in range(L * k) if flat[t] == m]


def test_nk_plan_build_rejects_bad_input():
    from trex_amd._lib import lib, ptr

    L_ = lib()
    plan = np.zeros(int(L_.trex_nk_plan_ints(3, 4, 1)), np.int32)
    bad_parent = np.array([1, 2, 3], np.int32)
    inter = np.zeros((4, 1), np.int32)
    assert L_.trex_nk_plan_build(ptr(bad_parent), 3, ptr(inter), 4, 1, ptr(plan), None) < 0
    parent = np.array([2, 2, 0], np.int32)
    bad_inter = np.full((4, 1), 4, np.int32)
    assert L_.trex_nk_plan_build(ptr(parent), 3, ptr(bad_inter), 4, 1, ptr(plan), None) < 0
