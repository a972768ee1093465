"""GPU parity of the raw-table entry points (rundp.hip) vs the CPU oracle.

trex_amd.run_dp / vectorized_dp / backtrack_sankoff_jit / vmapped_backtrack
take and return the reference's own tables (sankoff.py:24-97, 191-267):
DP (L, n_all, Q) and BacktrackingTable (L, n_all, Q, 4).  Bars: bit-exact
(min-plus on floats is exact arithmetic per operation, argmins are indices),
including caller-initialised tables, NaN entries, forward references, a
root self-loop (run_dp does not drop it) and hostile backtracking tables.
The first test is the reference's own tests/test_sankoff.py:9-36 run through
trex_amd.
"""

from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from _cases import balanced_children, int_cost, random_topologies, weird_children
from oracle.sankoff_ref import backtrack_ref, backtrack_site_exact, run_dp_ref, run_sankoff_ref
from trex_amd import (TrexError, backtrack_sankoff_jit, run_dp, run_sankoff, vectorized_dp,
                      vmapped_backtrack)
from trex_amd.topology import adjacency_from_children

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _np(t):
    return t.cpu().numpy()


def test_reference_test_run_dp_basic(device):
    """tests/test_sankoff.py:9-36 verbatim in meaning (run_dp on a caller's
    3-node table), plus the hand-derived table of tests/golden/kat_sankoff.json."""
    adj = np.array([[0, 1, 0], [0, 1, 0], [0, 0, 0]], dtype=np.float32)
    n_states = 2
    seqs = np.array([[0], [1], [0]], dtype=np.float32)
    cost_matrix = np.array([[0, 1], [1, 0]], dtype=np.float32)
    dp = np.full((3, n_states), 1e5, dtype=np.float32)
    back = np.zeros((3, n_states, 4), dtype=np.float32)
    dp_out, back_out = run_dp(adj, dp, back, seqs, cost_matrix, device=device)
    assert tuple(dp_out.shape) == (3, n_states)
    assert tuple(back_out.shape) == (3, n_states, 4)
    assert dp_out[0, 0] == 0
    assert dp_out[1, 1] == 0
    with open(os.path.join(GOLDEN, "kat_sankoff.json")) as f:
        k = json.load(f)["run_dp_fixture"]
    np.testing.assert_array_equal(_np(dp_out), np.array(k["dp"], np.float32))
    np.testing.assert_array_equal(_np(back_out)[2], np.array(k["bt_row2"], np.float32))
    # inputs are not modified (functional API, .at[].set copies)
    assert dp[0, 0] == 1e5 and not back.any()


def _random_tables(rng, L, n_all, Q, *, init="sentinel"):
    if init == "sentinel":
        dp = np.full((L, n_all, Q), 1e5, np.float32)
    else:  # caller-chosen values, some NaN / inf, small integers
        dp = rng.integers(0, 9, size=(L, n_all, Q)).astype(np.float32)
        dp[rng.random((L, n_all, Q)) < 0.02] = np.nan
        dp[rng.random((L, n_all, Q)) < 0.02] = np.inf
    bt = rng.integers(-3, 5, size=(L, n_all, Q, 4)).astype(np.float32)
    return dp, bt


@pytest.mark.parametrize("Q", [2, 4, 5, 20, 33, 40])
@pytest.mark.parametrize("init", ["sentinel", "caller"])
@pytest.mark.parametrize("topo", ["random", "fwdref", "dag", "rootloop"])
def test_vectorized_dp_matches_restatement(device, Q, init, topo):
    """vmap(run_dp) over 300 sites on caller tables: dp and bt bit-exact vs
    the restatement.  Q = 33 / 40 run the any-Q kernel (rows re-read from the
    table).  "rootloop" keeps adj[-1, -1] = 1, which run_dp (unlike
    run_sankoff) does not remove: the root lists itself and reads its own
    still-initial row."""
    rng = np.random.default_rng(Q * 7 + len(init) + len(topo))
    if topo == "random":
        ch = random_topologies(1, 12, seed=Q)[0]
    elif topo == "rootloop":
        ch = balanced_children(8)[0].copy()
    else:
        ch = weird_children(topo)
    adj = adjacency_from_children(ch)[0]
    if topo == "rootloop":
        adj[13, 14] = 0.0  # the root keeps one real child (12) ...
        adj[-1, -1] = 1.0  # ... and lists itself second: (12, 14)
    n_all = adj.shape[0]
    L = 300
    dp0, bt0 = _random_tables(rng, L, n_all, Q, init=init)
    seqs = rng.integers(-Q, Q + 2, size=((n_all + 1) // 2 + 1, L)).astype(np.float32)
    # truncation, wrap, NaN -> state 0 (XLA's convert), saturated -> dropped
    seqs[0, :5] = [0.7, -0.2, np.nan, 1e12, -1.5]
    cost = int_cost(Q, seed=Q).astype(np.float32)
    with np.errstate(invalid="ignore"):
        r_dp, r_bt = run_dp_ref(adj, dp0, bt0, seqs, cost)
    dp, bt = vectorized_dp(adj, dp0, bt0, seqs, cost, device=device)
    np.testing.assert_array_equal(_np(dp), r_dp)
    np.testing.assert_array_equal(_np(bt), r_bt)


def test_run_dp_multi_state_sequences(device):
    """Unmapped run_dp with an (n, k) sequence array: ``.at[i, seq[i]]``
    zeroes all k listed states of leaf i (sankoff.py:50 with an index array)."""
    ch = balanced_children(4)[0]
    adj = adjacency_from_children(ch)[0]
    Q = 5
    seqs = np.array([[0, 3], [1, 1], [4, -1], [2, 0]], np.float32)
    dp0 = np.full((7, Q), 1e5, np.float32)
    bt0 = np.zeros((7, Q, 4), np.float32)
    cost = int_cost(Q, seed=2)
    dp, _ = run_dp(adj, dp0, bt0, seqs, cost, device=device)
    d = _np(dp)
    for i in range(4):
        want = np.full(Q, 1e5, np.float32)
        for s in seqs[i].astype(np.int64):
            want[s % Q] = 0.0
        np.testing.assert_array_equal(d[i], want)
    # ancestors follow from those rows exactly as the restatement computes them
    ref = dp0.copy()
    ref[:4] = d[:4]
    r_dp, _ = run_dp_ref(adj, ref[None], bt0[None], np.full((4, 1), -99, np.float32), cost)
    np.testing.assert_array_equal(d[4:], r_dp[0, 4:])


@pytest.mark.parametrize("Q", [4, 20])
def test_backtrack_from_run_dp_table(device, Q):
    """run_sankoff's pipeline on raw tables: vectorized_dp -> root argmin ->
    vmapped backtrack equals the restatement and the engine's reconstruction."""
    rng = np.random.default_rng(Q)
    n = 16
    ch = random_topologies(1, n, seed=3)[0]
    adj = adjacency_from_children(ch)[0]
    n_all = 2 * n - 1
    L = 700
    seqs = rng.integers(0, Q, size=(n, L)).astype(np.float32)
    cost = int_cost(Q, seed=4)
    dp0 = np.full((L, n_all, Q), 1e5, np.float32)
    bt0 = np.zeros((L, n_all, Q, 4), np.float32)
    dp, bt = vectorized_dp(adj, dp0, bt0, seqs, cost, device=device)
    r_dp, r_bt = run_dp_ref(adj, dp0, bt0, seqs, cost)
    roots = r_dp[:, -1, :].argmin(axis=1).astype(np.int32)
    out = vmapped_backtrack(n_all - 1, None, bt, n_all, n, dp=dp)
    want = backtrack_ref(n_all - 1, roots, r_bt, n_all, n)
    np.testing.assert_array_equal(_np(out), want)
    out2 = vmapped_backtrack(n_all - 1, torch.as_tensor(roots), bt, n_all, n)
    assert torch.equal(out, out2)
    recon, _, _ = run_sankoff(adj, cost, seqs, n_all, Q, n, return_path=True, device=device)
    np.testing.assert_array_equal(_np(recon)[n:], _np(out)[n:].astype(np.float32))
    # the unmapped single-site form
    s0 = backtrack_sankoff_jit(n_all - 1, int(roots[5]), bt[5], n_all, n, device=device)
    np.testing.assert_array_equal(_np(s0), want[:, 5])


@pytest.mark.parametrize("n_leaves", [5, 1])
def test_backtrack_hostile_tables(device, n_leaves):
    """Arbitrary tables: per-state child ids, out-of-range / negative states
    and node ids, stack overflow past n_all (n_leaves = 1: eight nested
    ancestors on a 9-entry stack) -- the reference's clamped gathers and
    dropped scatters, site by site (oracle backtrack_site_exact)."""
    rng = np.random.default_rng(11 + n_leaves)
    n_all, Q, L = 9, 3, 257
    bt = np.empty((L, n_all, Q, 4), np.float32)
    # child ids mostly below the parent (so the DFS ends), some junk
    for v in range(n_all):
        bt[:, v, :, 0] = rng.integers(-2, max(v, 1), size=(L, Q))
        bt[:, v, :, 2] = rng.integers(-2, max(v, 1), size=(L, Q))
    bt[:, :, :, 1] = rng.integers(-4, Q + 3, size=(L, n_all, Q))
    bt[:, :, :, 3] = rng.integers(-4, Q + 3, size=(L, n_all, Q)) + 0.7
    roots = rng.integers(-1, Q + 1, size=L).astype(np.int32)
    out = _np(vmapped_backtrack(n_all - 1, torch.as_tensor(roots), bt, n_all, n_leaves,
                                device=device))
    for l in range(L):
        np.testing.assert_array_equal(
            out[:, l], backtrack_site_exact(n_all - 1, int(roots[l]), bt[l], n_all, n_leaves))


def test_backtrack_cyclic_table_raises(device):
    """A table whose DFS never ends (node 8 lists itself): the reference's
    while_loop would not return; the build stops and raises."""
    n_all, Q, L = 9, 2, 64
    bt = np.zeros((L, n_all, Q, 4), np.float32)
    bt[:, 8, :, 0] = 8
    bt[:, 8, :, 2] = 0
    with pytest.raises(TrexError):
        vmapped_backtrack(8, np.zeros(L, np.int32), bt, n_all, 5, device=device)


@pytest.mark.parametrize("n_leaves", [6, 7, 9, 10])
def test_run_sankoff_n_leaves_quirk(device, n_leaves):
    """run_sankoff with n_leaves != (n_all+1)//2: the DP still initialises
    (n_all+1)//2 = 8 leaf rows (sankoff.py:46) while the reconstruction and
    the backtrack use the argument (:161-185) -- bit-exact vs the restatement."""
    ch = balanced_children(8)[0]
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(n_leaves)
    seqs = rng.integers(0, 4, size=(max(8, n_leaves), 120)).astype(np.float32)
    cost = int_cost(4, seed=n_leaves)
    recon, dp, total = run_sankoff(adj, cost, seqs, 15, 4, n_leaves, return_path=True,
                                   device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 15, 4, n_leaves, return_path=True)
    np.testing.assert_array_equal(_np(dp), r_dp)
    np.testing.assert_array_equal(_np(recon), r_recon)
    assert float(total) == float(r_total)
