"""CPU oracle (numpy fp64): trex's tree-cost functions, their gradients, Adam.

TEST INFRASTRUCTURE ONLY (import rule: see oracle/sankoff_ref.py header).

Restates maraxen/trex src/trex/tree.py:
  discretize_tree_topology :31-47, update_tree :50-107, update_seq :110-130,
  enforce_graph_constraints :133-160, compute_surrogate_cost :163-209,
  compute_soft_cost :212-266, compute_cost :269-296, compute_loss :299-342
and optax 0.2.6's adam / clip_by_global_norm (third-party, uv.lock:1728-1729,
not vendored; used at tests/test_convergence.py:103,227 and
src/trex/evals/benchmark.py:41-72) from their published definitions
(scale_by_adam with eps_root = 0, bias correction 1 - b**count,
clip: t / ||g|| * max_norm when ||g|| >= max_norm).  "parity unpinned" at the
optax boundary: no reference test checks optimiser arithmetic.

The Gumbel draw of update_tree (tree.py:71, JAX threefry PRNG) cannot be
reproduced without JAX, so the noise is an explicit input here and in the
build.  Gradients are analytic (reverse-mode by hand) and checked against
central differences in tests/test_tree_oracle.py.
"""

from __future__ import annotations

import numpy as np


def _softmax(x, axis=-1):
    m = np.max(x, axis=axis, keepdims=True)
    m = np.where(np.isfinite(m), m, 0.0)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def discretize_tree_topology(adjacency, n_nodes):
    """one_hot(argmax(adj, 1), n_nodes) (tree.py:46-47; first index on ties)."""
    idx = np.argmax(np.asarray(adjacency), axis=1)
    return np.eye(n_nodes)[idx]


def tree_logits(tree_params, noise=None, temperature=1.0, gates=None):
    """Masked logit matrix of update_tree (tree.py:63-105), before the softmax."""
    theta = np.asarray(tree_params, dtype=np.float64)
    n_m1, n_anc = theta.shape
    n = n_m1 + 1
    nl = n - n_anc
    p = theta + (0.0 if noise is None else np.asarray(noise, dtype=np.float64))
    if gates is not None:
        p = p * gates
    p = p / temperature
    z = np.full((n, n), -np.inf)
    z[:nl, nl:] = p[:nl]
    i = np.arange(n_anc - 1)[:, None]
    j = np.arange(n_anc)[None, :]
    z[nl:-1, nl:] = np.where(j > i, p[nl:], -np.inf)
    z[-1, -1] = 1.0
    return z


def update_tree(tree_params, noise=None, temperature=1.0, gates=None):
    theta = np.asarray(tree_params)
    n_m1, n_anc = theta.shape
    if n_anc == 0:
        return np.eye(n_m1 + 1)
    return _softmax(tree_logits(theta, noise, temperature, gates), axis=1)


def update_tree_vjp(tree_params, noise, temperature, gates, A, dA):
    """d loss / d tree_params given dA = d loss / d A (A = update_tree(...))."""
    n_m1, n_anc = np.asarray(tree_params).shape
    n = n_m1 + 1
    nl = n - n_anc
    dz = A * (dA - np.sum(A * dA, axis=1, keepdims=True))  # row-softmax VJP
    dp = np.zeros((n_m1, n_anc))
    dp[:nl] = dz[:nl, nl:]
    i = np.arange(n_anc - 1)[:, None]
    j = np.arange(n_anc)[None, :]
    dp[nl:] = np.where(j > i, dz[nl:-1, nl:], 0.0)
    dp = dp / temperature
    if gates is not None:
        dp = dp * gates
    return dp


def update_seq(ancestors, sequences, temperature=1.0):
    """S[n_leaf:] = softmax(ancestors * T) (tree.py:127-130; note * T)."""
    seq = np.array(sequences, dtype=np.float64, copy=True)
    n_leaf = (seq.shape[0] + 1) // 2
    seq[n_leaf:] = _softmax(np.asarray(ancestors, dtype=np.float64) * temperature, axis=-1)
    return seq


def update_seq_vjp(ancestors, temperature, S_anc, dS_anc):
    return temperature * S_anc * (dS_anc - np.sum(S_anc * dS_anc, axis=-1, keepdims=True))


def enforce_graph_constraints(adjacency, scaling_factor):
    """scale * sum_cols (sum_rows A[:-1, -n_anc:] - 2)^2 (tree.py:156-160)."""
    A = np.asarray(adjacency, dtype=np.float64)
    n = A.shape[0]
    n_anc = (n - 1) // 2
    cols = A[:-1, n - n_anc:].sum(axis=0) if n_anc > 0 else np.zeros(0)
    return scaling_factor * np.sum((cols - 2.0) ** 2)


def enforce_graph_constraints_grad(adjacency, scaling_factor):
    A = np.asarray(adjacency, dtype=np.float64)
    n = A.shape[0]
    n_anc = (n - 1) // 2
    g = np.zeros_like(A)
    if n_anc > 0:
        cols = A[:-1, n - n_anc:].sum(axis=0)
        g[:-1, n - n_anc:] = 2.0 * scaling_factor * (cols - 2.0)[None, :]
    return g


def compute_surrogate_cost(S, A):
    """(sum A*E[:,None] + sum A*E[None,:] - 2 sum A*G) / 2 (tree.py:199-209)."""
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    E = np.sum(S ** 2, axis=(-1, -2))
    F = S.reshape(S.shape[0], -1)
    G = F @ F.T
    return (np.sum(A * E[:, None]) + np.sum(A * E[None, :]) - 2 * np.sum(A * G)) / 2


def compute_surrogate_cost_grads(S, A):
    """(value, dS, dA): dS_k = ((r+c)_k S_k - ((A+A^T) S)_k), dA = (E_i+E_j)/2 - G."""
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    F = S.reshape(S.shape[0], -1)
    G = F @ F.T
    E = np.diag(G).copy()
    val = (np.sum(A * E[:, None]) + np.sum(A * E[None, :]) - 2 * np.sum(A * G)) / 2
    rc = A.sum(axis=1) + A.sum(axis=0)
    dF = rc[:, None] * F - (A + A.T) @ F
    dA = 0.5 * (E[:, None] + E[None, :]) - G
    return val, dF.reshape(S.shape), dA


def compute_soft_cost(S, A, C=None):
    """Weighted variant (tree.py:248-266); C None, (Q,) diagonal or (Q, Q)."""
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    if C is None:
        W = S
    else:
        C = np.asarray(C, dtype=np.float64)
        W = S * C if C.ndim == 1 else S @ C
    E = np.sum(S * W, axis=(-1, -2))
    F = S.reshape(S.shape[0], -1)
    H = W.reshape(S.shape[0], -1)
    G = F @ H.T
    return (np.sum(A * E[:, None]) + np.sum(A * E[None, :]) - 2 * np.sum(A * G)) / 2


def compute_cost(S, A, subst):
    """Exact cost of a labelled tree (tree.py:286-296)."""
    seq = np.argmax(np.asarray(S), axis=2)
    parent = np.argmax(discretize_tree_topology(A, np.asarray(A).shape[0]), axis=1)
    subst = np.asarray(subst, dtype=np.float64)
    return subst[seq[parent], seq][:-1, :].sum()


def compute_loss(noise, params, sequences, temperature, adjacency=None, *,
                 graph_constraint_scale=10.0, fix_seqs=False, fix_tree=False):
    """compute_loss (tree.py:336-342) with explicit Gumbel noise.

    Returns (loss, grads dict {tree_params, ancestors}).  update_tree is called
    without a temperature (tree.py:338), i.e. at 1.0.
    """
    anc = np.asarray(params["ancestors"], dtype=np.float64)
    theta = np.asarray(params["tree_params"], dtype=np.float64)
    S = sequences if fix_seqs else update_seq(anc, sequences, temperature)
    A = adjacency if fix_tree else update_tree(theta, noise, 1.0)
    val, dS, dA = compute_surrogate_cost_grads(S, A)
    con = enforce_graph_constraints(A, graph_constraint_scale)
    dA = dA + temperature * enforce_graph_constraints_grad(A, graph_constraint_scale)
    loss = val + temperature * con
    grads = {"tree_params": np.zeros_like(theta), "ancestors": np.zeros_like(anc)}
    if not fix_tree:
        grads["tree_params"] = update_tree_vjp(theta, noise, 1.0, None, A, dA)
    if not fix_seqs:
        n_leaf = (S.shape[0] + 1) // 2
        grads["ancestors"] = update_seq_vjp(anc, temperature, S[n_leaf:], dS[n_leaf:])
    return loss, grads


def adam_init(params):
    return {"count": 0, "mu": {k: np.zeros_like(v, dtype=np.float64) for k, v in params.items()},
            "nu": {k: np.zeros_like(v, dtype=np.float64) for k, v in params.items()}}


def adam_update(grads, state, lr, b1=0.9, b2=0.999, eps=1e-8, clip_norm=None):
    """optax.[chain(clip_by_global_norm(clip_norm),)] adam(lr): returns (updates, state)."""
    g = {k: np.asarray(v, dtype=np.float64) for k, v in grads.items()}
    if clip_norm is not None:
        norm = np.sqrt(sum(np.sum(v ** 2) for v in g.values()))
        if not norm < clip_norm:
            g = {k: v / norm * clip_norm for k, v in g.items()}
    count = state["count"] + 1
    mu = {k: (1 - b1) * g[k] + b1 * state["mu"][k] for k in g}
    nu = {k: (1 - b2) * g[k] ** 2 + b2 * state["nu"][k] for k in g}
    upd = {}
    for k in g:
        mh = mu[k] / (1 - b1 ** count)
        nh = nu[k] / (1 - b2 ** count)
        upd[k] = -lr * mh / (np.sqrt(nh) + eps)
    return upd, {"count": count, "mu": mu, "nu": nu}


# ---------------------------------------------------------------------------
# create_optimizer (src/trex/evals/benchmark.py:41-72): optax 0.2.6 adam /
# adamw / sgd(momentum) / rmsprop, optionally chained after
# clip_by_global_norm(1.0) -- restated from optax's published definitions
# (third-party, not vendored: "parity unpinned", no reference test checks it)
# ---------------------------------------------------------------------------
def optax_init(params):
    z = {k: np.zeros_like(v, dtype=np.float64) for k, v in params.items()}
    return {"count": 0, "s1": dict(z), "s2": {k: v.copy() for k, v in z.items()}}


def optax_update(name, grads, state, params, lr, clip_norm=1.0, b1=0.9, b2=0.999, eps=1e-8,
                 weight_decay=0.01, momentum=0.9, decay=0.9):
    """Returns (updates, state) for name in adam / adamw / sgd / rmsprop."""
    g = {k: np.asarray(v, dtype=np.float64) for k, v in grads.items()}
    if clip_norm is not None:
        norm = np.sqrt(sum(np.sum(v ** 2) for v in g.values()))
        if not norm < clip_norm:
            g = {k: v / norm * clip_norm for k, v in g.items()}
    count = state["count"] + 1
    s1, s2, upd = {}, {}, {}
    for k in g:
        if name in ("adam", "adamw"):
            m = (1 - b1) * g[k] + b1 * state["s1"][k]
            v = (1 - b2) * g[k] ** 2 + b2 * state["s2"][k]
            u = (m / (1 - b1 ** count)) / (np.sqrt(v / (1 - b2 ** count)) + eps)
            if name == "adamw":
                u = u + weight_decay * np.asarray(params[k], dtype=np.float64)
            s1[k], s2[k] = m, v
        elif name == "sgd":
            u = g[k] + momentum * state["s1"][k]
            s1[k], s2[k] = u, state["s2"][k]
        elif name == "rmsprop":
            v = decay * state["s2"][k] + (1 - decay) * g[k] ** 2
            u = g[k] / np.sqrt(v + eps)
            s1[k], s2[k] = state["s1"][k], v
        else:
            raise ValueError(name)
        upd[k] = -lr * u
    return upd, {"count": count, "s1": s1, "s2": s2}


def fixed_tree_loss_grad(ancestors, masked_sequences, n_leaves, adjacency):
    """run_trex_optimization_configurable's loss (benchmark.py:158-165):
    surrogate(update_seq_stacked(ancestors, T=1), A) and d / d ancestors."""
    anc = np.asarray(ancestors, dtype=np.float64)
    S = np.array(masked_sequences, dtype=np.float64)
    P = _softmax(anc)
    S[n_leaves:] = P
    A = np.asarray(adjacency, dtype=np.float64)
    loss, dS, _ = compute_surrogate_cost_grads(S, A)
    g = dS[n_leaves:]
    return loss, P * (g - (g * P).sum(-1, keepdims=True))
