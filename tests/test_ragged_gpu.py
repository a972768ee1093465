"""Ragged tree batches (mixed n_all_b / L_b in one launch) vs the oracle and
vs the uniform engine run tree by tree.

Q <= 4 runs the lane-per-site kernel, Q = 5 / 20 / 61 the state-parallel
one (each 64-site item split over ceil(64 / sites-per-wave) waves), Q = 100
the large-alphabet one (a 128-thread workgroup walks the item's 64 sites).

Bars: hard path bit-exact (dp, per-tree / per-site scores, trex backtrack);
per-tree scores and dp also bitwise equal to a uniform SankoffEngine on the
same tree (same kernel arithmetic); d_cost rtol 1e-6 (hard) / 1e-5 (softmin)
vs the fp64 oracle summed over trees (the batch sums in a different order).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import assert_bound_close, assert_grad_close, int_cost, random_leaves
from oracle.sankoff_ref import run_sankoff_ref
from oracle.softmin_ref import sankoff_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, random_topologies
from trex_amd.ragged import RaggedSankoffEngine, RaggedTreePlan, from_padded
from trex_amd.topology import adjacency_from_children, create_balanced_binary_tree

pytestmark = pytest.mark.gpu

SIZES = [(5, 100), (9, 64), (32, 130), (2, 1), (17, 1000), (3, 65)]


def _batch(Q, seed, missing=0.0):
    chs, leaves = [], []
    for i, (n, L) in enumerate(SIZES):
        chs.append(random_topologies(1, n, seed=seed + i)[0])
        leaves.append(random_leaves(1, n, L, Q, seed=seed + 10 + i, missing=missing)[0])
    return chs, leaves


def _ref(chs, leaves, cost, tau, dts):
    return [sankoff_fwd_bwd_ref(c, lv, cost, tau, float(dts[b]))
            for b, (c, lv) in enumerate(zip(chs, leaves))]


@pytest.mark.parametrize("Q", [2, 3, 4, 5, 20, 61, 100])
def test_ragged_hard_matches_oracle_and_uniform(device, Q):
    chs, leaves = _batch(Q, seed=Q, missing=0.05)
    plan = RaggedTreePlan(chs, [L for _, L in SIZES])
    eng = RaggedSankoffEngine(plan, Q, device)
    cost = int_cost(Q, seed=7)
    lv = torch.as_tensor(plan.pack_leaves(leaves), device=device)
    c = torch.as_tensor(cost, device=device)
    dts = np.arange(1, plan.B + 1) / plan.B
    ts, dp, ss = eng.forward(lv, c, 0.0, site_score=True)
    refs = _ref(chs, leaves, cost, 0.0, dts)
    dpn, ssn = dp.cpu().numpy(), ss.cpu().numpy()
    for b, r in enumerate(refs):
        np.testing.assert_array_equal(plan.tree_rows(dpn, b).transpose(0, 2, 1),
                                      r["dp"].astype(np.float32))
        np.testing.assert_array_equal(plan.tree_sites(ssn, b), r["site_score"].astype(np.float32))
        assert ts[b].item() == np.float32(r["tree_score"])
        # uniform engine on the same tree: bitwise identical
        u = SankoffEngine(TreePlan(chs[b][None]), SIZES[b][1], Q, device)
        f = u.forward(torch.as_tensor(leaves[b][None], device=device), c, 0.0)
        assert torch.equal(f.tree_score[0], ts[b])
        assert torch.equal(f.dp[0].reshape(-1, Q), torch.as_tensor(plan.tree_rows(dpn, b),
                                                                   device=device).reshape(-1, Q))
    dc, mg, an = eng.backward(lv, c, 0.0, dp, torch.as_tensor(dts, dtype=torch.float32),
                              marginals=True, anc_states=True)
    np.testing.assert_allclose(dc.cpu().numpy(), sum(r["d_cost"] for r in refs), rtol=1e-6,
                               atol=1e-6)
    mgn = mg.cpu().numpy()
    for b, r in enumerate(refs):
        np.testing.assert_allclose(plan.tree_rows(mgn, b).transpose(0, 2, 1), r["marginals"],
                                   rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("Q", [4, 20, 100])
@pytest.mark.parametrize("tau", [0.3, 1.0])
def test_ragged_softmin_fused_vs_oracle(device, tau, Q):
    chs, leaves = _batch(Q, seed=40)
    plan = RaggedTreePlan(chs, [L for _, L in SIZES])
    eng = RaggedSankoffEngine(plan, Q, device)
    cost = int_cost(Q, seed=8)
    lv = torch.as_tensor(plan.pack_leaves(leaves), device=device)
    c = torch.as_tensor(cost, device=device)
    dts = np.linspace(0.5, 2.0, plan.B)
    ts, dp, ss, dc, mg, an = eng.fwd_bwd(lv, c, tau, torch.as_tensor(dts, dtype=torch.float32),
                                         site_score=True, marginals=True)
    refs = _ref(chs, leaves, cost, tau, dts)
    np.testing.assert_allclose(ts.cpu().numpy(), [r["tree_score"] for r in refs], rtol=1e-5)
    ref_dc = sum(r["d_cost"] for r in refs)
    assert_grad_close(dc.cpu().numpy(), ref_dc, rtol=1e-5)
    dpn = dp.cpu().numpy()
    for b, r in enumerate(refs):  # per-entry DP bar (tests/_cases.py assert_dp_close)
        assert_bound_close(plan.tree_rows(dpn, b).transpose(0, 2, 1), r["dp"],
                           1e-5 * r["dp_mag"] + 1e-30, what=f"dp[{b}]")
    # fused == separate launches, bitwise
    ts2, dp2, _ = eng.forward(lv, c, tau)
    dc2, mg2, _ = eng.backward(lv, c, tau, dp2, torch.as_tensor(dts, dtype=torch.float32),
                               marginals=True)
    assert torch.equal(ts, ts2) and torch.equal(dp, dp2) and torch.equal(dc, dc2)
    assert torch.equal(mg, mg2)


@pytest.mark.parametrize("Q", [4, 20, 61, 100])
def test_ragged_backtrack_matches_reference(device, Q):
    chs, leaves = _batch(Q, seed=60)
    plan = RaggedTreePlan(chs, [L for _, L in SIZES])
    eng = RaggedSankoffEngine(plan, Q, device)
    cost = int_cost(Q, seed=9)
    lv = torch.as_tensor(plan.pack_leaves(leaves), device=device)
    c = torch.as_tensor(cost, device=device)
    _, dp, _ = eng.forward(lv, c, 0.0)
    an = eng.backtrack(c, dp).cpu().numpy()
    for b, (ch, leaf) in enumerate(zip(chs, leaves)):
        adj = adjacency_from_children(ch[None])[0]
        n_all = ch.shape[0]
        nl = (n_all + 1) // 2
        recon, _, total = run_sankoff_ref(adj, cost, leaf.astype(np.float32), n_all, Q, nl,
                                          return_path=True)
        np.testing.assert_array_equal(plan.tree_rows(an, b), recon[nl:].astype(np.int8))


def test_from_padded_strips_trex_padding(device):
    """A trex-style padded batch (pad_adjacency to MAX_NODES = 63,
    pad_sequence to the N bucket, create_*_mask) gives the unpadded per-tree
    Sankoff totals."""
    Q, MAX, NB = 4, 63, 128
    trees = [(4, 30), (16, 100), (32, 128), (8, 7)]
    B = len(trees)
    A = np.zeros((B, MAX, MAX), np.float32)
    nm = np.zeros((B, MAX), bool)
    S = np.zeros((B, 32, NB), np.float32)
    sm = np.zeros((B, NB), bool)
    rng = np.random.default_rng(3)
    for b, (nl, L) in enumerate(trees):
        n_all = 2 * nl - 1
        A[b, :n_all, :n_all] = create_balanced_binary_tree(nl)
        nm[b, :n_all] = True
        S[b, :nl, :L] = rng.integers(0, Q, size=(nl, L))
        sm[b, :L] = True
    plan, packed, shapes = from_padded(A, nm, S, sm, Q)
    eng = RaggedSankoffEngine(plan, Q, device)
    cost = (np.ones((Q, Q)) - np.eye(Q)).astype(np.float32)
    ts, _, _ = eng.forward(torch.as_tensor(packed, device=device),
                           torch.as_tensor(cost, device=device), 0.0)
    for b, (nl, L) in enumerate(trees):
        n_all = 2 * nl - 1
        _, _, total = run_sankoff_ref(A[b, :n_all, :n_all], cost, S[b, :nl, :L], n_all, Q, nl)
        assert ts[b].item() == np.float32(total)
    assert shapes == [(2 * nl - 1, L) for nl, L in trees]


def test_ragged_rejects_q_above_128(device):
    chs, _ = _batch(4, seed=1)
    plan = RaggedTreePlan(chs, [L for _, L in SIZES])
    RaggedSankoffEngine(plan, 128, device)
    with pytest.raises(NotImplementedError):
        RaggedSankoffEngine(plan, 129, device)
