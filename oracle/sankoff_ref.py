"""CPU oracle: numpy restatement of trex's Sankoff hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker (or the timed CPU baseline) -- never as the thing measured or shipped.
The product path (``trex_amd``) never imports it and fails loudly when the HIP
library is missing.

What it restates (reference = maraxen/trex, read as text; JAX is not importable
in this image, see DESIGN.md "Oracle"):

* ``run_dp``                 src/trex/sankoff.py:24-94
* ``vectorized_dp``          src/trex/sankoff.py:97   (vmap over the site axis)
* ``run_sankoff``            src/trex/sankoff.py:114-188
* ``backtrack_sankoff_jit``  src/trex/sankoff.py:191-267

The hard-min path is restated in the reference's own arithmetic type (fp32 by
default, ``src/trex/types.py:13``) with the reference's operation order, so its
DP table, backtracking table, reconstruction and total are reproduced bit for
bit (the total is an fp32 sum whose order XLA does not fix; it is exact while
the integer total is < 2**24).  JAX indexing semantics that matter here are
restated explicitly:

* gather with a negative index wraps (``dp[-1]`` = last row), used by the
  ``fill_value=-1`` child of ``jnp.where(..., size=2)`` (sankoff.py:60,67);
* scatter ``.at[i, s].set(0)`` wraps negative ``s`` once and DROPS indices still
  out of range (sankoff.py:50, JAX "promise_in_bounds" scatter = drop);
* ``jnp.argmin`` returns the FIRST minimal index (sankoff.py:69,172).

Parity pin: the reference's own fixtures (tests/test_sankoff.py:9-72,
tests/test_convergence.py:42-85) with the hand-derived known answers recorded
in tests/golden/kat_sankoff.json, plus the invariant
``total == compute_cost(onehot(recon))`` (tests/test_convergence.py:69-73).
No reference-executed outputs exist (JAX absent), so this is a restatement
pinned by known answers, not by a reference run.
"""

from __future__ import annotations

import numpy as np

SENTINEL = 1e5  # src/trex/sankoff.py:152


# ---------------------------------------------------------------------------
# topology helpers
# ---------------------------------------------------------------------------
def trex_children(adj: np.ndarray, node: int) -> tuple[int, int]:
    """``jnp.where(adj[:, node] == 1, size=2, fill_value=-1)[0]`` (sankoff.py:60)."""
    rows = np.nonzero(adj[:, node] == 1)[0]
    out = [-1, -1]
    for k, r in enumerate(rows[:2]):
        out[k] = int(r)
    return out[0], out[1]


def trex_children_table(adj: np.ndarray) -> np.ndarray:
    """children[node] for every node, as trex's body_fun sees them.

    Applies run_sankoff's root self-loop removal (sankoff.py:141) first.
    Returns int32 (n_all, 2) with -1 fill.
    """
    a = np.array(adj, dtype=np.float64, copy=True)
    a[-1, -1] = 0
    n_all = a.shape[0]
    ch = np.full((n_all, 2), -1, dtype=np.int32)
    for v in range(n_all):
        ch[v] = trex_children(a, v)
    return ch


def _wrap_gather(idx: int, size: int) -> int:
    return idx + size if idx < 0 else idx


# ---------------------------------------------------------------------------
# hard Sankoff, exact restatement
# ---------------------------------------------------------------------------
def run_dp_ref(adj, dp, bt, seqs, cost, dtype=np.float32):
    """Vectorised ``run_dp`` over sites (== ``vectorized_dp``, sankoff.py:97).

    adj  (n_all, n_all); dp (L, n_all, Q); bt (L, n_all, Q, 4);
    seqs (n, L)  [site axis 1, as vmap in_axes=1]; cost (Q, Q).
    Returns (dp, bt) with the reference's dtype.
    """
    adj = np.asarray(adj)
    dp = np.array(dp, dtype=dtype, copy=True)
    bt = np.array(bt, dtype=dtype, copy=True)
    cost = np.asarray(cost, dtype=dtype)
    seqs = np.asarray(seqs, dtype=dtype)
    n_all = adj.shape[0]
    n_leaves = (n_all + 1) // 2
    L, _, Q = dp.shape
    sites = np.arange(L)
    # leaf init (sankoff.py:49-52): dp[i, int(seq[i])] = 0, negative wraps, OOB dropped;
    # int(.) is XLA's convert (_f2i: truncation, saturation, NaN -> 0), not numpy's astype
    f2i = np.vectorize(_f2i, otypes=[np.int64])
    for i in range(n_leaves):
        s = f2i(seqs[i])
        s = np.where(s < 0, s + Q, s)
        ok = (s >= 0) & (s < Q)
        dp[sites[ok], i, s[ok]] = 0
    # post-order over node index (sankoff.py:87-92)
    for node in range(n_leaves, n_all):
        c = trex_children(adj, node)
        total = np.zeros((L, Q), dtype=dtype)
        chars = []
        for k in range(2):
            ci = _wrap_gather(c[k], n_all)
            cost_array = cost[None, :, :] + dp[:, ci, None, :]  # (L, Q_i, Q_j)
            total = total + cost_array.min(axis=2)
            chars.append(cost_array.argmin(axis=2))
        dp[:, node, :] = total
        bt[:, node, :, 0] = c[0]
        bt[:, node, :, 1] = chars[0]
        bt[:, node, :, 2] = c[1]
        bt[:, node, :, 3] = chars[1]
    return dp, bt


def backtrack_ref(root_node, root_states, bt, n_all, n_leaves):
    """``vmap(backtrack_sankoff_jit)`` over sites (sankoff.py:166-180,191-267).

    The stack's node sequence depends on the topology only (bt[...,0] and
    bt[...,2] are the same for every state), so the DFS is simulated once with
    per-site state vectors.  Returns int32 (n_all, L).
    """
    L = bt.shape[0]
    sites = np.arange(L)
    recon = np.zeros((n_all, L), dtype=np.int32)
    stack = [(int(root_node), np.asarray(root_states, dtype=np.int32))]
    steps = 0
    while stack:
        steps += 1
        if steps > 10_000_000:
            raise RuntimeError("backtrack does not terminate (cyclic topology)")
        node, state = stack.pop()
        if node >= n_leaves:
            recon[node] = state
            info = bt[sites, node, state]  # (L, 4)
            c1 = int(info[0, 0])
            c2 = int(info[0, 2])
            stack.append((c1, info[:, 1].astype(np.int32)))
            stack.append((c2, info[:, 3].astype(np.int32)))
    return recon


def _f2i(x) -> int:
    """float -> int32 as XLA's convert: truncation, NaN -> 0, saturating."""
    x = float(x)
    if x != x:
        return 0
    if x >= 2147483647.0:
        return 2147483647
    if x <= -2147483648.0:
        return -2147483648
    return int(x)


def backtrack_site_exact(root_node, root_state, bt_site, n_all, n_leaves, max_steps=1 << 22):
    """One site of ``backtrack_sankoff_jit`` (sankoff.py:191-267), restated
    step by step for ANY backtracking table (per-state child ids allowed):

    * stack = zeros((n_all, 2), int32); stack[0] = (root_node, root_state);
      ptr = 1 (:212-214); loop while ptr > 0 (:220-223);
    * pop: (node, state) = stack[ptr-1] -- a traced gather, index clamped to
      n_all-1 (:232-233);
    * node >= n_leaves (:257-262): recon[node] = state (scatter, dropped when
      node >= n_all); child_info = bt[node, state] (gather: negative state
      wraps once, both indices clamped); the float entries are cast to int32
      when stored into the int32 stack; stack[ptr-1] and stack[ptr] are
      overwritten (scatters past n_all dropped); ptr += 1 (:236-251);
    * otherwise ptr -= 1 (:253-254).

    Returns int32 (n_all,), or raises RuntimeError after max_steps pops (the
    reference would not terminate).
    """
    bt_site = np.asarray(bt_site, dtype=np.float32)
    Q = bt_site.shape[1]
    stack = np.zeros((n_all, 2), dtype=np.int64)
    stack[0] = (root_node, root_state)
    ptr = 1
    recon = np.zeros(n_all, dtype=np.int64)
    steps = 0
    while ptr > 0:
        steps += 1
        if steps > max_steps:
            raise RuntimeError("backtrack does not terminate")
        cur = ptr - 1
        node, state = (int(v) for v in stack[min(cur, n_all - 1)])
        if node >= n_leaves:
            if node < n_all:
                recon[node] = state
            s = state + Q if state < 0 else state
            s = min(max(s, 0), Q - 1)
            info = bt_site[min(node, n_all - 1), s]
            if cur < n_all:
                stack[cur] = (_f2i(info[0]), _f2i(info[1]))
            if cur + 1 < n_all:
                stack[cur + 1] = (_f2i(info[2]), _f2i(info[3]))
            ptr = cur + 2
        else:
            ptr = cur
    return recon.astype(np.int32)


def run_sankoff_ref(adj, cost, seqs, n_all, n_states, n_leaves, return_path=False,
                    dtype=np.float32):
    """``run_sankoff`` (sankoff.py:114-188).  Returns (recon, dp, total)."""
    adj = np.array(adj, copy=True)
    adj[-1, -1] = 0
    adj = adj.astype(dtype)
    seqs = np.asarray(seqs).astype(dtype)
    cost = np.asarray(cost).astype(dtype)
    L = seqs.shape[1]
    bt = np.zeros((L, n_all, n_states, 4), dtype=dtype)
    dp = np.full((L, n_all, n_states), SENTINEL, dtype=dtype)
    dp, bt = run_dp_ref(adj, dp, bt, seqs, cost, dtype=dtype)
    recon = np.zeros((n_all, L), dtype=dtype)
    recon[:n_leaves] = seqs[:n_leaves]
    if return_path:
        root = adj.shape[0] - 1
        root_states = dp[:, root, :].argmin(axis=1).astype(np.int32)
        chars = backtrack_ref(root, root_states, bt, n_all, n_leaves)
        recon[n_leaves:] = chars[n_leaves:]
    total = dp[:, -1].min(axis=1).astype(np.float64).sum().astype(dtype)
    return recon, dp, total


# ---------------------------------------------------------------------------
# batched helpers used by the kernel parity tests
# ---------------------------------------------------------------------------
def normalize_leaves(seqs: np.ndarray, n_states: int) -> np.ndarray:
    """trex leaf-state semantics as int8 codes: [0,Q) observed, -1 = all-1e5 row.

    ``seq.astype(int32)`` is XLA's convert (truncation toward zero,
    saturation, NaN -> 0, as ``_f2i``); negative states wrap once; anything
    still out of range is dropped by the scatter (sankoff.py:50).
    """
    s = np.trunc(np.asarray(seqs, dtype=np.float64))
    s = np.where(np.isnan(s), 0.0, s)
    s = np.where(s < 0, s + n_states, s)
    ok = (s >= 0) & (s < n_states)
    return np.where(ok, s, -1).astype(np.int8)


def leaf_dp(leaf_codes: np.ndarray, n_states: int, dtype=np.float64) -> np.ndarray:
    """(..., L) int8 codes -> (..., L, Q) leaf DP rows (0 at state, 1e5 elsewhere)."""
    q = np.arange(n_states)
    return np.where(leaf_codes[..., None] == q, 0.0, SENTINEL).astype(dtype)
