"""Seeded test inputs shared by CPU and GPU tests (numpy only)."""

from __future__ import annotations

import numpy as np

from trex_amd.topology import create_balanced_binary_tree, random_topologies


def simulate_leaves(n_leaves, seq_len, n_states, n_mutations, seed):
    """numpy restatement of trex's ground-truth simulation.

    src/trex/ground_truth.py:20-52 (mutate: exactly n_mutations sites get a
    random non-zero offset mod n_states) and :112-197 (root = zeros; node
    numbering leaves 0..n-1, parent of 2i, 2i+1 is n+i).  JAX's PRNG stream is
    not reproducible, so only the process is restated.  Returns
    (all_sequences (n_all, L) int8, adjacency (n_all, n_all) float32).
    """
    rng = np.random.default_rng(seed)
    n_anc = n_leaves - 1
    n_all = n_leaves + n_anc
    seqs = np.zeros((n_all, seq_len), dtype=np.int8)

    def mutate(parent):
        child = parent.copy()
        if n_mutations > 0:
            pos = rng.choice(seq_len, size=n_mutations, replace=False)
            off = rng.integers(1, n_states, size=n_mutations)
            child[pos] = (child[pos] + off) % n_states
        return child

    for i in range(n_anc):
        parent_idx = n_all - 1 - i
        p_i = parent_idx - n_leaves
        seqs[2 * p_i] = mutate(seqs[parent_idx])
        seqs[2 * p_i + 1] = mutate(seqs[parent_idx])
    adj = np.zeros((n_all, n_all), dtype=np.float32)
    for i in range(n_anc):
        adj[2 * i, n_leaves + i] = 1
        adj[2 * i + 1, n_leaves + i] = 1
    return seqs, adj


def hamming(n_states):
    return (np.ones((n_states, n_states)) - np.eye(n_states)).astype(np.float32)


def int_cost(n_states, seed, lo=1, hi=4):
    rng = np.random.default_rng(seed)
    c = rng.integers(lo, hi + 1, size=(n_states, n_states)).astype(np.float32)
    c = np.triu(c, 1)
    c = c + c.T
    return c


def random_leaves(B, n_leaves, L, n_states, seed, missing=0.0):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, n_states, size=(B, n_leaves, L)).astype(np.int8)
    if missing > 0:
        m = rng.random((B, n_leaves, L)) < missing
        x[m] = -1
    return x


def balanced_children(n_leaves, B=1):
    from trex_amd.topology import children_from_adjacency

    ch = children_from_adjacency(create_balanced_binary_tree(n_leaves))
    return np.repeat(ch, B, axis=0)


def weird_children(case):
    """Balanced 8-leaf child lists exercising trex's quirks (sankoff.py:60,67).

    "fwdref": node 8 lists internal node 10 (> 8) -> 1e5 row in the DP, but the
              backtrack still visits 10 from 8 (last visit wins); node 9 has
              a -1 fill (second child missing).
    "dag":    node 9 is a child of both 12 and 13; node 10 is an orphan.
    "cycle":  node 8 lists its ancestor 12 -> the reference backtrack never
              terminates (forward DP is still defined).
    """
    ch = balanced_children(8)[0].copy()
    if case == "fwdref":
        ch[8] = (0, 10)
        ch[9, 1] = -1
    elif case == "dag":
        ch[13] = (9, 11)
    elif case == "cycle":
        ch[8] = (0, 12)
    else:
        raise ValueError(case)
    return ch


def assert_grad_close(got, ref, rtol=1e-5, what="dC"):
    """Elementwise gradient bar: |got - ref| <= rtol * |ref| for EVERY entry
    (north_star: "grads within 1e-5 for the softmin relaxation").

    No matrix-max atol: a softmin dC entry is a sum of non-negative terms
    (softmax weight x cotangent), so each entry carries its own relative
    error; a normwise bar would let the small entries drift.  The only
    absolute slack is 1e-30, below fp32's normal range (1.2e-38) times the
    ~1e8 terms an entry sums -- entries the fp64 oracle holds at < 1e-30 are
    underflow in any fp32 arithmetic, the reference's included.  Returns the
    max elementwise relative error (the message reports it on failure)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    err = np.abs(got - ref)
    bound = rtol * np.abs(ref) + 1e-30
    rel = err / np.maximum(np.abs(ref), 1e-30)
    bad = ~(err <= bound)
    k = np.unravel_index(int(np.argmax(np.where(np.isfinite(rel), rel, np.inf))), rel.shape)
    assert not bad.any(), (f"{what}: max elementwise rel err {rel[k]:.3e} at {k} "
                           f"(got {got[k]!r}, ref {ref[k]!r}); {int(bad.sum())} of {bad.size} "
                           f"entries above rtol {rtol:g}")
    return float(rel[k])


def cond_rtol(dp_ref, tau, rtol=1e-5):
    """Per-entry relative bound set by fp32 D itself, for the cases where it
    exceeds 1e-5: the DP table is fp32 (as trex returns it), so each D value
    is rounded to half an ulp of |D|; a softmin weight
    w = exp((M_c[i] - C_ij - D_c[j]) / tau) has relative error equal to the
    absolute error of its exponent, ~ 2 * 2^-24 * max|D| / tau (the errors
    of the two D-like terms; normalisation keeps the dominant weights far
    more accurate, the tiny ones -- e^-40-class at tau = 0.05 -- carry the
    full amount).  Each dC entry is a non-negative combination of such
    weights, so this bounds it elementwise.  Used where the bound exceeds
    1e-5: leaves with out-of-range states (trex's all-1e5 row,
    sankoff.py:49-52,152, puts a 1e5 offset into every D) and tau = 0.05
    with costs up to 9 (|D| / tau ~ 2 000).  Never below rtol."""
    return max(rtol, 2.0 * 2.0 ** -24 * float(np.abs(dp_ref).max()) / tau)


def assert_bound_close(got, ref, bound, what="value"):
    """Elementwise |got - ref| <= bound (an array of per-entry bounds, e.g.
    1e-5 * (|M| @ |S|) for a product with mixed signs).  Returns the max of
    |got - ref| / bound; the message names the worst entry."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    bound = np.broadcast_to(np.asarray(bound, dtype=np.float64), ref.shape)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    err = np.abs(got - ref)
    ratio = err / np.maximum(bound, 1e-300)
    k = np.unravel_index(int(np.argmax(np.where(np.isfinite(ratio), ratio, np.inf))), ratio.shape)
    bad = ~(err <= bound)
    assert not bad.any(), (f"{what}: max err / bound {ratio[k]:.3e} at {k} (got {got[k]!r}, "
                           f"ref {ref[k]!r}, bound {bound[k]:.3e}); {int(bad.sum())} of "
                           f"{bad.size} entries out of bound")
    return float(ratio[k])


def assert_dp_close(got, ref, rtol=1e-5, what="dp"):
    """Softmin DP table vs the fp64 oracle, per entry: |got - ref| <= rtol *
    dp_mag (oracle/softmin_ref.py: the running error bound of the recursion,
    every term of every message at its magnitude -- a D entry summing
    messages of either sign keeps their absolute scale) + 1e-30.  got / ref in
    the oracle's (B, n_int, Q, L) order.  Returns the max err / bound."""
    return assert_bound_close(got, ref["dp"], rtol * ref["dp_mag"] + 1e-30, what=what)


def path_dmax(children, dp_ref):
    """Per (tree, internal row, site): the sum over the row and its ancestors
    (root included) of max_state |D|.  children (B, n_all, 2) trex child ids;
    dp_ref (B, n_int, Q, L) the oracle's table.  A marginal is a product of
    softmin weights along the path from the root, each weight's exponent
    (D_j - min D) / tau carrying fp32 D's rounding, ~eps |D| / tau, so the
    relative error of a marginal entry is bounded by ~eps * path_dmax / tau
    (shared children of trex's DAG quirk: the larger path)."""
    B, n_int, _, L = dp_ref.shape
    n_all = children.shape[1]
    nl = n_all - n_int
    dm = np.abs(dp_ref).max(axis=2)  # (B, n_int, L)
    out = np.zeros_like(dm)
    for b in range(B):
        parents = [[] for _ in range(n_int)]
        for node in range(nl, n_all):
            for c in children[b, node]:
                c = int(c)
                if nl <= c < node:
                    parents[c - nl].append(node - nl)
        for r in range(n_int - 1, -1, -1):
            up = 0.0
            for p in parents[r]:
                up = np.maximum(up, out[b, p])
            out[b, r] = dm[b, r] + up
    return out


def marginal_rtol(children, dp_ref, tau, rtol=1e-5, c=8.0):
    """Per-entry relative bound for softmin marginals vs the fp64 oracle,
    (B, n_int, 1, L): max(rtol, c * 2^-24 * path_dmax / tau) -- fp32 D's
    conditioning along the root path (see path_dmax), never below 1e-5.

    c from the adjoint's rounding steps.  A marginal is a product of softmin
    weights along its root path; each weight is exp((md - D_j) / tau) / s
    with |md|, |D_j| <= dmax (the row's max |D|), so its relative error is
    the absolute error of (md - D_j) / tau.  Per level, in units of
    2^-24 dmax / tau (half an ulp of dmax):
      * D_j as the kernel holds it: two messages, each rounded once after
        its own log / fma (1 + 1), and their sum rounded (1)          -> 3
      * md = min_j D_j: the same value, the same 3                     -> 3
      * the subtraction md - D_j, rounded                               -> 1
      * the scale by a = log2(e) / tau (1) and exp2's result (1 ulp of a
        value <= 1: below the unit of the others)                      -> 1
    c = 3 + 3 + 1 + 1 = 8 per level, summed over the path (path_dmax sums
    each level's dmax).  The normalisations 1/s (s a sum of <= Q terms in
    [0, 1]) add ~Q 2^-24 relative per level, independent of |D| / tau: that
    is what the rtol floor 1e-5 covers.  Measured on MI355X over every
    kernel and the tests' shapes (Q 4 .. 61, tau 0.02 .. 1, 8 .. 64 taxa, C3
    at full size): worst entry 5.0 (tools/parity_probe.py marg,
    profiles/r04_parity_probe.log), entries with the 1e-5 floor below 3e-6
    -- inside the derived bound."""
    return np.maximum(rtol, c * 2.0 ** -24 * path_dmax(children, dp_ref) / tau)[:, :, None, :]


def assert_marginals_close(got, ref, children, dp_ref, tau, c=8.0, what="marginals"):
    """Elementwise marginal bar: |got - ref| <= marginal_rtol * |ref| + 1e-30
    (1e-30: entries fp32 cannot hold near its underflow).  Returns the max
    relative error over entries with |ref| > 1e-30 and the bound used."""
    rt = marginal_rtol(children, dp_ref, tau, c=c)
    ref = np.asarray(ref, dtype=np.float64)
    assert_bound_close(got, ref, rt * np.abs(ref) + 1e-30, what=what)
    m = np.abs(ref) > 1e-30
    rel = np.abs(np.asarray(got, np.float64) - ref)[m] / np.abs(ref)[m]
    return float(rel.max()) if rel.size else 0.0, rt


def clear_argmax_mask(ref, rt, slack=4.0):
    """Sites / rows where the fp64 marginals' top two states differ by more
    than `slack` times their per-entry bounds: the soft ancestral state there
    is the fp64 argmax (elsewhere a tie within fp32 conditioning).
    ref (B, n_int, Q, L), rt (B, n_int, 1, L)."""
    top2 = np.sort(ref, axis=2)[:, :, -2:, :]
    return (top2[:, :, 1] - top2[:, :, 0]) > slack * rt[:, :, 0] * top2[:, :, 1] + 1e-30


def surrogate_grad_bounds(S, A, rtol=1e-5, constraint_grad=None):
    """Per-entry bounds for the surrogate's gradients (tree.py:163-209), fp64:
    dS = (r + c) S - (A + A^T) S  ->  rtol (|r + c| |S| + |A + A^T| |S|);
    dA = (E_i + E_j) / 2 - G_ij (+ T * constraint)  ->  rtol ((E_i + E_j) / 2
    + |G_ij| + |constraint term|): the sum of the magnitudes of each entry's
    terms, the rounding bound of any fp32 evaluation (entries that cancel to
    ~0 keep an absolute bound from their terms)."""
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    F = S.reshape(S.shape[0], -1)
    G = F @ F.T
    E = np.diag(G)
    rc = A.sum(axis=1) + A.sum(axis=0)
    AA = np.abs(A + A.T)
    bS = rtol * (np.abs(rc)[:, None] * np.abs(F) + AA @ np.abs(F))
    bA = 0.5 * (E[:, None] + E[None, :]) + np.abs(G)
    if constraint_grad is not None:
        bA = bA + np.abs(constraint_grad)
    return bS.reshape(S.shape), rtol * bA


def softmax_vjp_bound(P, M, axis=-1):
    """Magnitude bound of a softmax VJP P (g - sum(P g)) for |g| <= M
    (elementwise): P (M + sum(P M))."""
    return P * (M + np.sum(P * M, axis=axis, keepdims=True))


EPS_VJP = 8 * 2.0 ** -24  # a few fp32 roundings of the VJP's own arithmetic


def tree_param_select(dz, n_anc):
    """update_tree_vjp's map from the (n, n) logit cotangent to tree_params
    (oracle/tree_ref.py:73-78; tree.py:63-105 masking), temperature 1."""
    n = dz.shape[0]
    nl = n - n_anc
    dp = np.zeros((n - 1, n_anc))
    dp[:nl] = dz[:nl, nl:]
    i = np.arange(n_anc - 1)[:, None]
    j = np.arange(n_anc)[None, :]
    dp[nl:] = np.where(j > i, dz[nl:-1, nl:], 0.0)
    return dp


def loss_grad_bounds(noise, params, sequences, temperature, adjacency=None, *, rtol=1e-5,
                     fix_seqs=False, fix_tree=False, scale=10.0):
    """Per-entry bounds for compute_loss's gradients (tree.py:299-342; the
    oracle's compute_loss): dA / dS at rtol times their terms' magnitudes
    (surrogate_grad_bounds), carried through each softmax VJP (update_tree's
    rows, update_seq's states: softmax_vjp_bound) plus that VJP's own
    rounding at the magnitude of the exact cotangent.  Returns
    {tree_params, ancestors} bound arrays."""
    from oracle import tree_ref as T

    anc = np.asarray(params["ancestors"], dtype=np.float64)
    theta = np.asarray(params["tree_params"], dtype=np.float64)
    S = sequences if fix_seqs else T.update_seq(anc, sequences, temperature)
    A = adjacency if fix_tree else T.update_tree(theta, noise, 1.0)
    S = np.asarray(S, dtype=np.float64)
    A = np.asarray(A, dtype=np.float64)
    _, dS, dA = T.compute_surrogate_cost_grads(S, A)
    cg = temperature * T.enforce_graph_constraints_grad(A, scale)
    dA = dA + cg
    bS, bA = surrogate_grad_bounds(S, A, rtol, constraint_grad=cg)
    out = {"tree_params": np.zeros_like(theta), "ancestors": np.zeros_like(anc)}
    if not fix_tree:
        dz = softmax_vjp_bound(A, bA, axis=1) + EPS_VJP * softmax_vjp_bound(A, np.abs(dA), axis=1)
        out["tree_params"] = tree_param_select(dz, theta.shape[1])
    if not fix_seqs:
        nl = (S.shape[0] + 1) // 2
        Sa = S[nl:]
        out["ancestors"] = temperature * (softmax_vjp_bound(Sa, bS[nl:])
                                          + EPS_VJP * softmax_vjp_bound(Sa, np.abs(dS[nl:])))
    return out


def landscape_grad_bound(ancestors, masked_sequences, n_leaves, interactions, fitness, adj,
                         lambda_val, real_k, temperature=1.0, seq_mask=None, rtol=1e-5):
    """Per-entry bound for d loss / d ancestors of the NK landscape-aware
    loss (benchmark.py:235-306; oracle/nk_ref.py): every term of d loss / dS
    at its magnitude -- the surrogate's (surrogate_grad_bounds), the child
    cross-entropy's -log p (|logits| + |lse|, plus the logits' own error
    scale carried through log_softmax), d CE / d logits (p sum S + S, plus
    p's error scale) pushed through the parental-logits VJP with |F| (the
    parent distributions are >= 0, so that VJP of magnitudes sums the terms'
    magnitudes) -- times rtol, through update_seq's softmax VJP."""
    from oracle import nk_ref as nk

    _, parts = nk.landscape_loss(ancestors, masked_sequences, n_leaves, interactions, fitness,
                                 adj, lambda_val, real_k, temperature, seq_mask)
    S = parts["S"]
    A = np.asarray(adj, dtype=np.float64)
    n_all, L, Q = S.shape
    X = S.reshape(n_all, -1)
    rc = A.sum(1) + A.sum(0)
    mag = (np.abs(rc)[:, None] * np.abs(X) + np.abs(A + A.T) @ np.abs(X)).reshape(S.shape)
    if lambda_val > 0.0 and real_k > 0:
        mask = np.ones(L) if seq_mask is None else np.asarray(seq_mask, dtype=np.float64)
        parent = np.argmax(A, axis=1)
        n_nonroot = float((np.arange(n_all) != parent).sum())
        w = mask[None, :, None] * (lambda_val / (n_nonroot * float(mask.sum())))
        logits = parts["logits"]
        Fa = np.abs(np.asarray(fitness, dtype=np.float64))
        Lmag = nk.compute_parental_logits(S[parent], interactions, Fa, real_k)
        m = logits.max(-1, keepdims=True)
        lse = m + np.log(np.exp(logits - m).sum(-1, keepdims=True))
        p = np.exp(logits - lse)
        Lp = Lmag + (p * Lmag).sum(-1, keepdims=True)  # log_softmax of the logits' error
        mag = mag + (np.abs(logits) + np.abs(lse) + Lp) * w
        sumS = S.sum(-1, keepdims=True)
        dlog_mag = (p * sumS + S + p * Lp * sumS) * w
        np.add.at(mag, parent, nk.parental_logits_vjp(S[parent], interactions, Fa, dlog_mag))
    pa = S[n_leaves:]
    return rtol * temperature * softmax_vjp_bound(pa, mag[n_leaves:])


__all__ = ["simulate_leaves", "hamming", "int_cost", "random_leaves", "balanced_children",
           "weird_children", "random_topologies", "create_balanced_binary_tree",
           "assert_grad_close", "cond_rtol", "assert_bound_close", "assert_dp_close", "path_dmax", "marginal_rtol",
           "assert_marginals_close", "clear_argmax_mask", "surrogate_grad_bounds", "softmax_vjp_bound",
           "tree_param_select", "loss_grad_bounds", "landscape_grad_bound"]
