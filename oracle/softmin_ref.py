"""CPU oracle (fp64): batched Sankoff forward + adjoint, hard and softmin.

TEST INFRASTRUCTURE ONLY (see oracle/sankoff_ref.py header for the import rule).

The hard (tau == 0) forward is trex's ``run_dp`` recurrence
(src/trex/sankoff.py:55-85) with trex's child rules (sankoff.py:60,67):

* a child index c < n_leaves is a leaf row (0 at the observed state, 1e5 else);
* n_leaves <= c < node is an already computed internal row;
* c == -1 (fill value) or c >= node reads a row still holding the 1e5 init
  (row -1 is the root row, written last; rows >= node are written later).

Its gradient is JAX's reverse-mode derivative of ``dp[:, -1].min(1).sum()``
(sankoff.py:187) w.r.t. ``cost_matrix``: ``jnp.min``'s JVP
(``_reduce_chooser_jvp_rule``, jax 0.7.2 pinned at uv.lock:857-858, not
vendored) spreads the cotangent evenly over tied minima.

The softmin relaxation (tau > 0) is BUILD-DEFINED -- trex has none
(sankoff.py:67-69 uses the hard min; readme.md:15 only claims
differentiability):

    smin_tau(x) = -tau * log(sum_j exp(-x_j / tau))
    M_c[i]      = smin_tau_j(C[i, j] + D_c[j]);  D_v[i] = sum_c M_c[i]
    site score  = smin_tau(D_root)   (or min(D_root) with hard_root=True)

and its adjoint (pre-order), with w_c[i, j] = softmax_j(-(C[i, j] + D_c[j]) / tau):

    gbar_root = softmax(-D_root / tau) * d_tree_score
    gbar_c[j] = sum_i gbar_v[i] w_c[i, j];  dC[i, j] += gbar_v[i] w_c[i, j]

tau -> 0 recovers the hard recurrence and the tie-averaged subgradient.
Everything here is float64 (the kernel is checked against it with a stated
tolerance); the hard forward is exact for integer costs.
"""

from __future__ import annotations

import numpy as np

from .sankoff_ref import SENTINEL, leaf_dp


def classify_children(children: np.ndarray, n_all: int):
    """children: (n_all, 2) trex child ids (rows < n_leaves unused).

    Returns list over internal rows r of [(kind, index), (kind, index)] with
    kind in {"leaf", "int", "sent"}; for "int" index = internal row.
    """
    n_leaves = (n_all + 1) // 2
    out = []
    for node in range(n_leaves, n_all):
        pair = []
        for c in children[node]:
            c = int(c)
            if c == -1 or c >= node:
                pair.append(("sent", -1))
            elif c < n_leaves:
                pair.append(("leaf", c))
            else:
                pair.append(("int", c - n_leaves))
        out.append(pair)
    return out


def _child_x(kind, idx, cost, leafD, D):
    if kind == "leaf":
        Dc = leafD[idx]
    elif kind == "int":
        Dc = D[idx]
    else:
        Dc = np.full(leafD.shape[1:], SENTINEL)
    return cost[None, :, :] + Dc[:, None, :]  # (L, Qi, Qj)


def _smin(x, tau):
    """Reduce the last axis; returns (value, weights) with weights summing to 1."""
    m = x.min(axis=-1)
    if tau == 0.0:
        ind = (x == m[..., None]).astype(np.float64)
        w = ind / ind.sum(axis=-1, keepdims=True)
        return m, w
    e = np.exp(-(x - m[..., None]) / tau)
    s = e.sum(axis=-1)
    return m - tau * np.log(s), e / s[..., None]


def sankoff_fwd_bwd_ref(children, leaves, cost, tau, d_tree_score=1.0,
                        hard_root=False):
    """One tree.

    children (n_all, 2) int; leaves (n_leaves, L) int8 codes (-1 = missing);
    cost (Q, Q).  Returns dict with dp (n_int, Q, L), site_score (L,),
    tree_score, d_cost (Q, Q), marginals (n_int, Q, L), and dp_mag
    (n_int, Q, L), each D entry's error scale for an fp32 evaluation:

        Dmag_v[i] = sum_c (|C_ij*| + tau (log s_c[i] + 1) + Dmag_c*),

    j* = argmin_j (C_ij + D_c[j]), s_c[i] = sum_j exp(-(x_j - min x) / tau),
    Dmag_c* = sum_j w_c[i, j] Dmag_c[j] for an internal child, |D_c[j*]| for
    a leaf / 1e5 row (exact inputs; 1e5 for a missing state).  This is the
    running error bound of the recursion -- D evaluated with every term's
    magnitude (M_c[i] = C_ij* + D_c[j*] - tau log s_c[i]; s >= 1 is a sum
    rounded relative to itself, so tau log s carries an absolute error of
    order tau eps even where log s ~ 0: hence tau (log s + 1); a softmin is
    1-Lipschitz, so the child's error arrives weighted by w).  A D entry that
    sums messages of either sign to ~0 keeps the absolute scale of its terms.
    """
    cost = np.asarray(cost, dtype=np.float64)
    Q = cost.shape[0]
    n_all = children.shape[0]
    n_leaves = (n_all + 1) // 2
    n_int = n_all - n_leaves
    L = leaves.shape[1]
    leafD = leaf_dp(leaves[:n_leaves], Q)  # (n_leaves, L, Q)
    kinds = classify_children(children, n_all)
    D = np.zeros((n_int, L, Q))
    Dmag = np.zeros((n_int, L, Q))  # error scale of D (docstring)
    for r in range(n_int):
        acc = np.zeros((L, Q))
        mag = np.zeros((L, Q))
        for kind, idx in kinds[r]:
            x = _child_x(kind, idx, cost, leafD, D)
            M, w = _smin(x, tau)
            acc = acc + M
            js = np.argmin(x, axis=-1)  # (L, Qi)
            xm = np.take_along_axis(x, js[..., None], axis=-1)[..., 0]
            # xm - M = tau log s; + tau: s >= 1 carries a relative rounding,
            # i.e. tau log s an absolute one of ~tau eps (log s ~ 0 included)
            mag = mag + np.abs(cost[np.arange(Q)[None, :], js]) + (xm - M) + tau
            if kind == "int":
                mag = mag + np.einsum("lij,lj->li", w, Dmag[idx])
            else:
                dcs = np.take_along_axis(x - cost[None, :, :], js[..., None], axis=-1)[..., 0]
                mag = mag + np.abs(dcs)
        D[r] = acc
        Dmag[r] = mag
    Droot = D[n_int - 1]
    site, groot = _smin(Droot, 0.0 if hard_root else tau)
    # adjoint, reverse node order (children have lower indices)
    G = np.zeros((n_int, L, Q))
    G[n_int - 1] = groot * d_tree_score
    dC = np.zeros((Q, Q))
    for r in range(n_int - 1, -1, -1):
        g = G[r]
        if not g.any():
            continue
        for kind, idx in kinds[r]:
            x = _child_x(kind, idx, cost, leafD, D)
            _, w = _smin(x, tau)
            contrib = g[:, :, None] * w  # (L, Qi, Qj)
            dC += contrib.sum(axis=0)
            if kind == "int":
                G[idx] += contrib.sum(axis=1)
    return {
        "dp": D.transpose(0, 2, 1).copy(),
        "dp_mag": Dmag.transpose(0, 2, 1).copy(),
        "site_score": site,
        "tree_score": site.sum(),
        "d_cost": dC,
        "marginals": G.transpose(0, 2, 1).copy(),
    }


def batched_fwd_bwd_ref(children, leaves, cost, tau, d_tree_score=None,
                        hard_root=False):
    """children (B, n_all, 2); leaves (B, n_leaves, L).  Sums d_cost over trees."""
    B = children.shape[0]
    if d_tree_score is None:
        d_tree_score = np.ones(B)
    outs = [sankoff_fwd_bwd_ref(children[b], leaves[b], cost, tau,
                                float(d_tree_score[b]), hard_root) for b in range(B)]
    return {
        "dp": np.stack([o["dp"] for o in outs]),
        "dp_mag": np.stack([o["dp_mag"] for o in outs]),
        "site_score": np.stack([o["site_score"] for o in outs]),
        "tree_score": np.array([o["tree_score"] for o in outs]),
        "d_cost": sum(o["d_cost"] for o in outs),
        "marginals": np.stack([o["marginals"] for o in outs]),
    }
