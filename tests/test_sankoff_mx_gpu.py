"""The matrix-core kernel (trex_amd/csrc/sankoff_mx.hip, TREX_MX=1, opt-in
while it is slower than the state-parallel kernel on C3) vs the fp64 oracle
and vs the state-parallel kernel: factored softmin, 4 < Q <= 20.

Bars as tests/test_sankoff_wide_gpu.py: scores rtol 1e-5, every dC entry
rtol 1e-5 (tests/_cases.assert_grad_close), DP table and marginals at the
fp32 rules; fused == separate launches bit for bit; the hard path (tau = 0)
and the per-row stabilised softmin never reach it (its device-side mode
check hands them to the state-parallel kernels)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (assert_grad_close, cond_rtol, hamming, int_cost, random_leaves,
                    random_topologies, weird_children)
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def mx_on(monkeypatch):
    monkeypatch.setenv("TREX_MX", "1")


def _sm(t):
    return t.permute(0, 1, 3, 2).cpu().numpy()


@pytest.mark.parametrize("n,L,Q,tau,missing", [(16, 300, 20, 0.5, 0.0), (16, 300, 20, 1.0, 0.05),
                                               (12, 257, 7, 0.3, 0.0), (12, 100, 13, 1.0, 0.0),
                                               (24, 333, 18, 0.5, 0.02), (8, 16, 5, 0.7, 0.0)])
def test_mx_softmin_vs_fp64(device, n, L, Q, tau, missing):
    B = 2
    ch = random_topologies(B, n, seed=n + Q)
    leaves = random_leaves(B, n, L, Q, seed=L + Q, missing=missing)
    cost = int_cost(Q, seed=Q, hi=3)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv = torch.as_tensor(leaves, device=device)
    c = torch.as_tensor(cost, device=device)
    f, dc, mg, an = eng.fwd_bwd(lv, c, tau, site_score=True, marginals=True, anc_states=True)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=1e-5)
    rt = cond_rtol(ref["dp"], tau) if missing else 1e-5
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=rt)
    np.testing.assert_allclose(_sm(f.dp), ref["dp"], rtol=1e-5, atol=1e-5 * np.abs(ref["dp"]).max())
    mtol = max(2e-5, 8 * 1.2e-7 * np.abs(ref["dp"]).max() / tau)
    np.testing.assert_allclose(_sm(mg), ref["marginals"], atol=mtol)
    m = ref["marginals"]
    top2 = np.sort(m, axis=2)[:, :, -2:, :]
    clear = (top2[:, :, 1] - top2[:, :, 0]) > 4 * mtol
    np.testing.assert_array_equal(an.cpu().numpy()[clear], m.argmax(axis=2)[clear])
    # fused == separate launches, bit for bit
    f2 = eng.forward(lv, c, tau, site_score=True)
    d2, m2, a2 = eng.backward(lv, c, tau, f2.dp, marginals=True, anc_states=True)
    assert torch.equal(f2.dp, f.dp) and torch.equal(f2.tree_score, f.tree_score)
    assert torch.equal(d2, dc) and torch.equal(m2, mg) and torch.equal(a2, an)


@pytest.mark.parametrize("case", ["fwdref", "dag"])
def test_mx_reference_quirks(device, case):
    """-1 fills / forward references (the all-1e5 row) and shared children
    (the staged program runs DAG trees serially on one wave)."""
    Q, L, tau = 9, 200, 0.5
    ch = weird_children(case)[None]
    leaves = random_leaves(1, 8, L, Q, seed=3)
    cost = int_cost(Q, seed=4)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    f, dc, _, _ = eng.fwd_bwd(torch.as_tensor(leaves, device=device),
                              torch.as_tensor(cost, device=device), tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=1e-5)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=cond_rtol(ref["dp"], tau))


def test_mx_hands_other_modes_to_the_state_parallel_kernel(device):
    """tau = 0 and range(C) / tau > 40 are not its modes: results equal the
    TREX_MX=0 run bit for bit (the device flag makes the state-parallel
    launch behind it do the work)."""
    B, n, L, Q = 2, 16, 200, 20
    ch = random_topologies(B, n, seed=1)
    leaves = random_leaves(B, n, L, Q, seed=2)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv = torch.as_tensor(leaves, device=device)
    for cost, tau in ((int_cost(Q, seed=3, lo=1, hi=9), 0.05), (hamming(Q), 0.5)):
        c = torch.as_tensor(cost, device=device)
        import os

        outs = []
        for mx in ("1", "0"):
            os.environ["TREX_MX"] = mx
            f, dc, _, _ = eng.fwd_bwd(lv, c, tau)
            outs.append((f.tree_score.clone(), dc.clone(), f.dp.clone()))
        if tau == 0.05:  # per-row stabilised mode: identical
            assert all(torch.equal(x, y) for x, y in zip(outs[0], outs[1]))
        else:  # factored mode: the matrix-core kernel ran, same results to fp32
            np.testing.assert_allclose(outs[0][0].cpu().numpy(), outs[1][0].cpu().numpy(),
                                       rtol=1e-6)
