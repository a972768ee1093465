"""GPU parity of the large-alphabet kernel (64 < Q <= 128, sankoff_bigq.hip)
vs the CPU oracle.

trex sizes its tables from n_states with no cap (src/trex/sankoff.py:151-152);
the engine serves Q up to 128 (int8 leaf codes and ancestral states) and
refuses larger alphabets with TREX_E_UNSUPPORTED; run_sankoff then takes the
raw-table kernels (trex_run_dp, trex_backtrack_generic, trex_dp_root_total),
checked here bit-exact at Q = 129 and 257.  Bars as everywhere: hard
DP table / totals / reconstruction bit-exact, hard gradient rtol 1e-6,
softmin score and dC rtol 1e-5 elementwise, marginals by the per-entry
fp32-D conditioning bound (tests/_cases.py).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (assert_dp_close, assert_grad_close, assert_marginals_close, hamming,
                    int_cost, random_leaves, random_topologies)
from oracle.sankoff_ref import run_sankoff_ref
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, TrexError, run_sankoff
from trex_amd.topology import adjacency_from_children

pytestmark = pytest.mark.gpu


def _dev(x, device, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


def _sm(t):
    return t.cpu().numpy().transpose(0, 1, 3, 2)


@pytest.mark.parametrize("Q", [65, 100, 128])
@pytest.mark.parametrize("L", [1, 37, 300])
def test_run_sankoff_bitexact_bigq(device, Q, L):
    ch = random_topologies(1, 12, seed=300 + L + Q)[0]
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(L * 5 + Q)
    seqs = rng.integers(0, Q, size=(12, L)).astype(np.float32)
    cost = int_cost(Q, seed=Q + L)
    recon, dp, total = run_sankoff(adj, cost, seqs, 23, Q, 12, return_path=True, device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 23, Q, 12, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


@pytest.mark.parametrize("Q,ties", [(128, True), (77, False)])
def test_batched_hard_fwd_grad_bigq(device, Q, ties):
    B, n, L = 3, 10, 70
    ch = random_topologies(B, n, seed=Q)
    leaves = random_leaves(B, n, L, Q, seed=Q + 1, missing=0.05)
    cost = hamming(Q) if ties else int_cost(Q, seed=2)
    dts_np = np.arange(1, B + 1) / B
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0, d_tree_score=dts_np)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, 0.0, dp=True, site_score=True)
    np.testing.assert_array_equal(_sm(f.dp), ref["dp"].astype(np.float32))
    np.testing.assert_array_equal(f.site_score.cpu().numpy(), ref["site_score"].astype(np.float32))
    np.testing.assert_array_equal(f.tree_score.cpu().numpy(), ref["tree_score"].astype(np.float32))
    dts = torch.as_tensor(dts_np, dtype=torch.float32, device=device)
    dc, mg, an = eng.backward(lv, c, 0.0, f.dp, dts, marginals=True, anc_states=True)
    np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(_sm(mg), ref["marginals"], rtol=1e-6, atol=1e-7)
    # ancestral states = first index of the (device's own) marginals' max
    np.testing.assert_array_equal(an.cpu().numpy(), _sm(mg).argmax(axis=2))
    # trex-exact reconstruction (hard forward + backtrack) per tree, on leaves
    # without missing states (trex wraps negative float states, the engine's
    # int8 codes treat them as missing: test_leaf_state_semantics)
    full = random_leaves(B, n, L, Q, seed=Q + 2)
    lf = _dev(full, device)
    anc = eng.backtrack(c, eng.forward(lf, c, 0.0).dp).cpu().numpy()
    adj = adjacency_from_children(ch)
    for b in range(B):
        r = run_sankoff_ref(adj[b], cost, full[b].astype(np.float32), 2 * n - 1, Q, n,
                            return_path=True)
        np.testing.assert_array_equal(anc[b].astype(np.float32), r[0][n:])


@pytest.mark.parametrize("tau", [1.0, 0.2])
@pytest.mark.parametrize("Q", [65, 128])
def test_softmin_fwd_grad_bigq_vs_fp64(device, tau, Q):
    B, n, L = 2, 12, 90
    ch = random_topologies(B, n, seed=n + Q)
    leaves = random_leaves(B, n, L, Q, seed=L + Q)
    cost = int_cost(Q, seed=5)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, tau, dp=True, site_score=True)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=1e-5)
    np.testing.assert_allclose(f.site_score.cpu().numpy(), ref["site_score"], rtol=1e-5)
    assert_dp_close(_sm(f.dp), ref, 1e-5)
    dc, mg, _ = eng.backward(lv, c, tau, f.dp, marginals=True)
    rel = assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=1e-5)
    assert rel <= 1e-5
    assert_marginals_close(_sm(mg), ref["marginals"], ch, ref["dp"], tau)


def test_fused_equals_separate_bigq(device):
    B, n, L, Q = 2, 9, 40, 96
    ch = random_topologies(B, n, seed=7)
    leaves = random_leaves(B, n, L, Q, seed=8, missing=0.02)
    cost = int_cost(Q, seed=9)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    dts = torch.linspace(0.5, 2.0, B, device=device)
    f, dc, mg, an = eng.fwd_bwd(lv, c, 0.5, dts, site_score=True, marginals=True, anc_states=True)
    f2 = eng.forward(lv, c, 0.5, site_score=True)
    dc2, mg2, an2 = eng.backward(lv, c, 0.5, f2.dp, dts, marginals=True, anc_states=True)
    assert torch.equal(f.dp, f2.dp) and torch.equal(f.tree_score, f2.tree_score)
    assert torch.equal(dc, dc2) and torch.equal(mg, mg2) and torch.equal(an, an2)


def test_alphabet_above_128_is_refused(device):
    ch = random_topologies(1, 4, seed=0)
    with pytest.raises(TrexError, match="Q=129"):
        eng = SankoffEngine(TreePlan(ch), 10, 129, device)
        lv = torch.zeros((1, 4, 10), dtype=torch.int8, device=device)
        eng.forward(lv, torch.ones((129, 129), device=device), 0.0)


@pytest.mark.parametrize("Q,L,n", [(129, 40, 12), (257, 9, 7)])
def test_run_sankoff_past_the_engine_alphabet(device, Q, L, n):
    """n_states > 128: run_sankoff on the raw-table kernels, bit-exact vs the
    oracle (dp, reconstruction, total; sankoff.py:114-188), incl. a wrapped
    negative and an out-of-range leaf state (the reference's dropped
    scatter) and an odd n_leaves that disagrees with (n_all + 1) // 2."""
    ch = random_topologies(1, n, seed=Q + L)[0]
    adj = adjacency_from_children(ch)[0]
    n_all = 2 * n - 1
    rng = np.random.default_rng(Q * 3 + L)
    seqs = rng.integers(0, Q, size=(n, L)).astype(np.float32)
    seqs[0, 0] = -1.0  # wraps to Q - 1
    seqs[1, 1] = Q + 3.0  # dropped: all-1e5 leaf row
    cost = int_cost(Q, seed=Q)
    for n_leaves in (n, n - 1):
        recon, dp, total = run_sankoff(adj, cost, seqs, n_all, Q, n_leaves, return_path=True,
                                       device=device)
        r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, n_all, Q, n_leaves,
                                                 return_path=True)
        np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
        np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
        assert float(total) == float(r_total)

