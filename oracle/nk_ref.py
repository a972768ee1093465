"""CPU oracle (numpy fp64): trex's NK landscape-aware loss and its gradient.

TEST INFRASTRUCTURE ONLY (import rule: see oracle/sankoff_ref.py header).

Restates maraxen/trex:
  compute_parental_logits               src/trex/evals/benchmark.py:586-663
  _update_seq_stacked                   src/trex/evals/benchmark.py:210-232
  _compute_loss_landscape_aware_stacked src/trex/evals/benchmark.py:235-306
  create_nk_model_landscape (shapes)    src/trex/nk_model.py:17-43
  pad_interactions / pad_fitness_table  src/trex/padding.py:144-216

compute_parental_logits follows the reference operation for operation: the
joint neighbour distribution is built by successive outer products
(einsum "pc,ps->pcs" then reshape, :637-642), so neighbour 0 is the MOST
significant digit of the joint index; the site's fitness table is reshaped
to (Q, Q**k) (:647), so the site's own state is the most significant digit of
the table index (note: get_fitness, nk_model.py:98-107, uses the opposite,
least-significant-first order; the reference's parental logits do not, and
neither does this restatement).  k is interactions.shape[1] (the padded k,
:619), so padded landscapes behave as in the reference.

The gradient is analytic reverse mode (checked against central differences in
tests/test_nk_oracle.py).  The reference has no test of this path
(tests/test_nk_model_new.py covers only the data generator): parity beyond
this restatement is unpinned.
"""

from __future__ import annotations

import numpy as np


def _softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def _log_softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    return x - m - np.log(np.exp(x - m).sum(axis=axis, keepdims=True))


def compute_parental_logits(parent_sequences, interactions, fitness_tables, real_k=None):
    """(n_parents, L, Q) logits (benchmark.py:586-663).

    parent_sequences (P, L, Q); interactions (L, k) int; fitness_tables
    (L, Q**(k+1)).  real_k == 0 returns the fitness table broadcast
    (:616-620, fitness_tables is (L, Q) then)."""
    P = np.asarray(parent_sequences, dtype=np.float64)
    n_p, L, Q = P.shape
    F = np.asarray(fitness_tables, dtype=np.float64)
    inter = np.asarray(interactions)
    if real_k == 0:
        return np.broadcast_to(F[None, :, :], (n_p, L, Q)).copy()
    k = inter.shape[1]
    out = np.empty((n_p, L, Q))
    for i in range(L):
        nb = inter[i, :k]
        probs = P[:, nb, :]  # (P, k, Q)
        joint = probs[:, 0, :]
        for j in range(1, k):
            joint = np.einsum("pc,ps->pcs", joint, probs[:, j, :]).reshape(n_p, -1)
        table = F[i].reshape(Q, -1)
        out[:, i, :] = np.einsum("si,pi->ps", table, joint)
    return out


def parental_logits_vjp(parent_sequences, interactions, fitness_tables, d_logits):
    """d/dP of sum(d_logits * compute_parental_logits(P)) for k >= 1."""
    P = np.asarray(parent_sequences, dtype=np.float64)
    n_p, L, Q = P.shape
    F = np.asarray(fitness_tables, dtype=np.float64)
    inter = np.asarray(interactions)
    k = inter.shape[1]
    g = np.asarray(d_logits, dtype=np.float64)
    dP = np.zeros_like(P)
    for i in range(L):
        nb = inter[i, :k]
        probs = P[:, nb, :]  # (P, k, Q)
        table = F[i].reshape((Q,) + (Q,) * k)  # [s, c0, ..., c_{k-1}]
        # dJ[p, c0..] = sum_s g[p, i, s] F[s, c0..]
        dJ = np.tensordot(g[:, i, :], table, axes=([1], [0]))  # (P, Q, ..., Q)
        letters = "abcdefghijklmnopqrstuvw"[:k]
        for j in range(k):
            # contract every other neighbour's probabilities, keep axis j
            operands = [dJ]
            subs = ["z" + letters]
            for jj in range(k):
                if jj != j:
                    operands.append(probs[:, jj, :])
                    subs.append("z" + letters[jj])
            expr = ",".join(subs) + "->z" + letters[j]
            dP[:, nb[j], :] += np.einsum(expr, *operands)
    return dP


def update_seq_stacked(ancestors, sequences, n_leaves, temperature=1.0):
    """sequences.at[n_leaves:].set(softmax(ancestors * T)) (benchmark.py:210-232)."""
    S = np.array(sequences, dtype=np.float64)
    S[n_leaves:] = _softmax(np.asarray(ancestors, dtype=np.float64) * temperature)
    return S


def surrogate_cost(S, A):
    """0.5 * sum_ij A_ij ||S_i - S_j||^2 (tree.py:163-209)."""
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    X = S.reshape(S.shape[0], -1)
    E = (X * X).sum(1)
    G = X @ X.T
    return 0.5 * float((A * (E[:, None] + E[None, :] - 2.0 * G)).sum())


def landscape_loss(ancestors, masked_sequences, n_leaves, interactions, fitness_tables,
                   adj_matrix, lambda_val, real_k, temperature=1.0, seq_mask=None):
    """_compute_loss_landscape_aware_stacked (benchmark.py:235-306), fp64.

    Returns (loss, parts) with parts = {surrogate, fitness, logits, S}."""
    S = update_seq_stacked(ancestors, masked_sequences, n_leaves, temperature)
    A = np.asarray(adj_matrix, dtype=np.float64)
    n_all, L, _ = S.shape
    mask = np.ones(L) if seq_mask is None else np.asarray(seq_mask, dtype=np.float64)
    sur = surrogate_cost(S, A)
    fit = 0.0
    logits = None
    if lambda_val > 0.0 and real_k > 0:
        parent = np.argmax(A, axis=1)  # first index of the max (:286)
        logits = compute_parental_logits(S[parent], interactions, fitness_tables, real_k)
        logp = _log_softmax(logits)
        ce = -(S * logp).sum(-1)  # (n_all, L)
        n_nonroot = float((np.arange(n_all) != parent).sum())
        fit = float((ce * mask[None, :]).sum()) / (n_nonroot * float(mask.sum()))
    return sur + lambda_val * fit, {"surrogate": sur, "fitness": fit, "logits": logits, "S": S}


def landscape_loss_grad(ancestors, masked_sequences, n_leaves, interactions, fitness_tables,
                        adj_matrix, lambda_val, real_k, temperature=1.0, seq_mask=None):
    """(loss, d loss / d ancestors) of landscape_loss (analytic, fp64)."""
    loss, parts = landscape_loss(ancestors, masked_sequences, n_leaves, interactions,
                                 fitness_tables, adj_matrix, lambda_val, real_k, temperature,
                                 seq_mask)
    S = parts["S"]
    A = np.asarray(adj_matrix, dtype=np.float64)
    n_all, L, Q = S.shape
    mask = np.ones(L) if seq_mask is None else np.asarray(seq_mask, dtype=np.float64)
    X = S.reshape(n_all, -1)
    r = A.sum(1)
    c = A.sum(0)
    dS = ((np.diag(r + c) - (A + A.T)) @ X).reshape(S.shape)
    if lambda_val > 0.0 and real_k > 0:
        parent = np.argmax(A, axis=1)
        n_nonroot = float((np.arange(n_all) != parent).sum())
        scale = lambda_val / (n_nonroot * float(mask.sum()))
        logits = parts["logits"]
        logp = _log_softmax(logits)
        w = mask[None, :, None] * scale
        dS += -logp * w  # child role
        # d ce / d logits = softmax * sum_s S - S
        dlog = (np.exp(logp) * S.sum(-1, keepdims=True) - S) * w
        dPar = parental_logits_vjp(S[parent], interactions, fitness_tables, dlog)
        np.add.at(dS, parent, dPar)
    anc = np.asarray(ancestors, dtype=np.float64)
    p = _softmax(anc * temperature)
    g = dS[n_leaves:]
    d_anc = temperature * p * (g - (g * p).sum(-1, keepdims=True))
    return loss, d_anc


def random_landscape(L, k, Q, seed=0):
    """create_nk_model_landscape's shapes (nk_model.py:31-43) from numpy: the
    reference draws with JAX's PRNG, which cannot run here."""
    rng = np.random.default_rng(seed)
    inter = rng.integers(0, L, size=(L, k)).astype(np.int32)
    F = rng.uniform(size=(L, Q ** (k + 1))).astype(np.float32)
    return inter, F


def pad_landscape(interactions, fitness_tables, target_k, Q):
    """pad_interactions / pad_fitness_table (padding.py:144-216), K axis only."""
    inter = np.asarray(interactions)
    F = np.asarray(fitness_tables)
    k = inter.shape[1]
    if target_k > k:
        inter = np.pad(inter, ((0, 0), (0, target_k - k)), constant_values=0)
        F = np.pad(F, ((0, 0), (0, Q ** (target_k + 1) - Q ** (k + 1))), constant_values=0.0)
    return inter, F
