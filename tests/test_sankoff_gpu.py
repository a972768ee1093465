"""GPU parity: libtrexhip.so (HIP, gfx950) vs the CPU oracle.

Bars (DESIGN.md "Parity"):
  * hard (tau = 0) DP table, totals, reconstruction, ancestral states:
    bit-exact (integer costs; fp32 values are exact integers);
  * hard gradient (tie-averaged subgradient): rtol 1e-6 vs fp64 oracle;
  * softmin score / gradient: rtol 1e-5 elementwise vs fp64 oracle
    (north_star: "grads within 1e-5 for the softmin relaxation");
  * softmin marginals: elementwise relative, max(1e-5, 8 eps path_dmax /
    tau) per entry -- fp32 D's conditioning along the entry's root path
    (tests/_cases.py marginal_rtol; 1e-5 wherever that is below it).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (assert_dp_close, assert_grad_close, assert_marginals_close,
                    balanced_children, clear_argmax_mask, cond_rtol, hamming, int_cost, random_leaves,
                    random_topologies, simulate_leaves, weird_children)
from oracle.sankoff_ref import normalize_leaves, run_sankoff_ref
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, run_sankoff, sankoff_value_and_grad
from trex_amd.topology import adjacency_from_children

pytestmark = pytest.mark.gpu

SOFT_RTOL = 1e-5


@pytest.fixture(autouse=True, params=["lane-per-site", "state-parallel", "staged"])
def q4_kernel(request, monkeypatch):
    """Every Q <= 4 case runs once on each of the three live kernels the
    policy (sankoff.hip wide_small_q / use_staged) chooses between: the
    lane-per-site kernel (the C4 headline path), the state-parallel kernel
    (4 lanes per site, one DPP quad, G = 4; Q = 2 / 3 pad the quad) and the
    staged kernel (the state-parallel item as a workgroup of waves over the
    tree's levels, sankoff_staged.hip).  The policy itself runs in
    tests/test_configs_full_gpu.py and tests/test_rundp_gpu.py."""
    if request.param == "lane-per-site":
        monkeypatch.setenv("TREX_WIDE_SMALLQ", "0")
    else:
        monkeypatch.setenv("TREX_WIDE_SMALLQ", "1")
        monkeypatch.setenv("TREX_STAGED", "1" if request.param == "staged" else "0")
    return request.param


def _engine(children, L, Q, device):
    return SankoffEngine(TreePlan(children), L, Q, device)


def _rows(eng, t):
    """engine table -> the oracle's (B, n_int, Q, L) layout (numpy)."""
    return eng.state_rows(t).cpu().numpy()


def _dev(x, device, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


# ---------------------------------------------------------------------------
# reference fixtures + hand-derived known answers
# ---------------------------------------------------------------------------
def test_run_sankoff_reference_fixture_kat(device):
    """tests/test_sankoff.py:39-72 fixture; values hand-derived."""
    adj = np.zeros((5, 5), dtype=np.int32)
    adj[0, 3] = adj[1, 3] = adj[2, 4] = adj[3, 4] = 1
    cost = np.ones((2, 2)) - np.eye(2)
    seqs = np.array([[0, 1], [1, 0], [0, 0], [0, 0], [0, 0]], dtype=np.float32)
    recon, dp, total = run_sankoff(adj, cost, seqs[:3], 5, 2, 3, return_path=True,
                                   device=device)
    assert tuple(recon.shape) == (5, 2) and tuple(dp.shape) == (2, 5, 2)
    assert float(total) == 2.0
    np.testing.assert_array_equal(dp.cpu().numpy(), np.array(
        [[[0, 1e5], [1e5, 0], [0, 1e5], [1, 1], [1, 2]],
         [[1e5, 0], [0, 1e5], [0, 1e5], [1, 1], [1, 2]]], dtype=np.float32))
    np.testing.assert_array_equal(recon.cpu().numpy(),
                                  np.array([[0, 1], [1, 0], [0, 0], [0, 0], [0, 0]], np.float32))
    assert torch.all(recon[:3] == torch.as_tensor(seqs[:3], device=device))


def test_convergence_setup_invariant(device):
    """tests/test_convergence.py:42-73: Sankoff total == compute_cost(onehot(recon))."""
    seqs, adj = simulate_leaves(4, 20, 4, 3, seed=42)
    cost = hamming(4)
    recon, dp, total = run_sankoff(adj, cost, seqs[:4], 7, 4, 4, return_path=True,
                                   device=device)
    r = recon.cpu().numpy().astype(np.int64)
    parent = adj.argmax(axis=1)
    direct = cost[r[parent], r][:-1].sum()
    assert abs(float(total) - direct) < 1e-3
    ref = run_sankoff_ref(adj, cost, seqs[:4], 7, 4, 4, return_path=True)
    np.testing.assert_array_equal(recon.cpu().numpy(), ref[0])
    np.testing.assert_array_equal(dp.cpu().numpy(), ref[1])
    assert float(total) == float(ref[2])


# ---------------------------------------------------------------------------
# run_sankoff == trex restatement, bit for bit
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("L", [1, 3, 64, 130, 1000, 4096])
@pytest.mark.parametrize("Q", [2, 3, 4])
def test_run_sankoff_bitexact_random_trees(device, L, Q):
    """The backtrack runs on the split-lane kernel (4 lanes per site); its
    one-lane-per-site twin is forced in tests/test_sankoff_wide_gpu.py."""
    ch = random_topologies(1, 16, seed=100 + L + Q)[0]
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(L * 7 + Q)
    seqs = rng.integers(0, Q, size=(16, L)).astype(np.float32)
    cost = int_cost(Q, seed=Q + L)
    recon, dp, total = run_sankoff(adj, cost, seqs, 31, Q, 16, return_path=True, device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 31, Q, 16, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


@pytest.mark.parametrize("case", ["fwdref", "dag"])
def test_run_sankoff_reference_quirks(device, case):
    """-1 fills, forward references (1e5 rows), shared children, orphans."""
    ch = weird_children(case)
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(5)
    seqs = rng.integers(0, 4, size=(8, 257)).astype(np.float32)
    cost = int_cost(4, seed=9)
    recon, dp, total = run_sankoff(adj, cost, seqs, 15, 4, 8, return_path=True, device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 15, 4, 8, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


def test_cycle_topology_refuses_backtrack(device):
    ch = weird_children("cycle")
    adj = adjacency_from_children(ch)[0]
    seqs = np.zeros((8, 16), dtype=np.float32)
    cost = hamming(4)
    _, dp, total = run_sankoff(adj, cost, seqs, 15, 4, 8, return_path=False, device=device)
    r = run_sankoff_ref(adj, cost, seqs, 15, 4, 8, return_path=False)
    np.testing.assert_array_equal(dp.cpu().numpy(), r[1])
    from trex_amd import TrexError

    with pytest.raises(TrexError):
        run_sankoff(adj, cost, seqs, 15, 4, 8, return_path=True, device=device)


def test_leaf_state_semantics(device):
    """Negative states wrap once; out-of-range states leave an all-1e5 row;
    fractional states truncate (sankoff.py:49-52)."""
    adj = adjacency_from_children(balanced_children(4))[0]
    seqs = np.array([[0, -1, 7, 2.9, -5, 3],
                     [1, 1, 1, -4, 0, 0],
                     [2, 3, -2, 0.5, 1, 4],
                     [3, 0, 1, 1, 2, -0.5]], dtype=np.float32)
    cost = int_cost(4, seed=1)
    recon, dp, total = run_sankoff(adj, cost, seqs, 7, 4, 4, return_path=True, device=device)
    r = run_sankoff_ref(adj, cost, seqs, 7, 4, 4, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r[1])
    np.testing.assert_array_equal(recon.cpu().numpy(), r[0])
    assert float(total) == float(r[2])


# ---------------------------------------------------------------------------
# batched engine: hard forward / gradient / ancestral states
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("L,Q,n", [(1, 4, 8), (300, 4, 16), (1024, 4, 32), (777, 3, 12),
                                   (2048, 2, 20)])
def test_batched_hard_fwd_grad(device, L, Q, n):
    B = 6
    ch = random_topologies(B, n, seed=L + n)
    leaves = random_leaves(B, n, L, Q, seed=L, missing=0.05)
    cost = int_cost(Q, seed=L + 1)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0, d_tree_score=np.arange(1, B + 1) / B)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, 0.0, dp=True, site_score=True)
    np.testing.assert_array_equal(_rows(eng, f.dp), ref["dp"].astype(np.float32))
    np.testing.assert_array_equal(f.site_score.cpu().numpy(),
                                  ref["site_score"].astype(np.float32))
    np.testing.assert_array_equal(f.tree_score.cpu().numpy(), ref["tree_score"].astype(np.float32))
    dts = torch.arange(1, B + 1, dtype=torch.float32, device=device) / B
    dc, mg, _ = eng.backward(lv, c, 0.0, f.dp, dts, marginals=True)
    np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(_rows(eng, mg), ref["marginals"], rtol=1e-6, atol=1e-7)


def test_batched_backtrack_matches_reference(device):
    B, n, L, Q = 5, 24, 515, 4
    ch = random_topologies(B, n, seed=3)
    leaves = random_leaves(B, n, L, Q, seed=4)
    cost = int_cost(Q, seed=5)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, 0.0)
    anc = eng.backtrack(c, f.dp).cpu().numpy()
    adj = adjacency_from_children(ch)
    for b in range(B):
        r = run_sankoff_ref(adj[b], cost, leaves[b].astype(np.float32), 2 * n - 1, Q, n,
                            return_path=True)
        np.testing.assert_array_equal(anc[b].astype(np.float32), r[0][n:])


# ---------------------------------------------------------------------------
# softmin relaxation
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("tau", [1.0, 0.5, 0.1, 0.02])
@pytest.mark.parametrize("L,n", [(100, 8), (1000, 64), (501, 32)])
def test_softmin_fwd_grad_vs_fp64(device, tau, L, n):
    B, Q = 3, 4
    ch = random_topologies(B, n, seed=n + 11)
    leaves = random_leaves(B, n, L, Q, seed=L + 3)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, tau, dp=True, site_score=True)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    np.testing.assert_allclose(f.site_score.cpu().numpy(), ref["site_score"], rtol=SOFT_RTOL,
                               atol=1e-5)
    assert_dp_close(_rows(eng, f.dp), ref, SOFT_RTOL)
    dc, mg, anc = eng.backward(lv, c, tau, f.dp, marginals=True, anc_states=True)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    # per-site marginals are products of softmax weights of D / tau along the
    # root path: elementwise relative, bounded by fp32 D's conditioning
    m = ref["marginals"]
    _, rt = assert_marginals_close(_rows(eng, mg), m, ch, ref["dp"], tau)
    # soft ancestral states = argmax marginals wherever the top two differ
    clear = clear_argmax_mask(m, rt)
    np.testing.assert_array_equal(anc.cpu().numpy()[clear], m.argmax(axis=2)[clear])


def test_softmin_missing_leaves_fp32_offset(device):
    """A leaf whose state is out of range keeps trex's all-1e5 row
    (sankoff.py:49-52,152).  Under the softmin every ancestor's D then carries
    a ~1e5 offset, where fp32's ulp is 0.0078, so cotangents that depend on
    differences of such D values are only good to ~ulp(1e5)/tau relative --
    the same loss the reference's own fp32 arithmetic has.  Scores keep 1e-5."""
    B, n, L, Q, tau = 3, 8, 100, 4, 1.0
    ch = random_topologies(B, n, seed=19)
    leaves = random_leaves(B, n, L, Q, seed=103, missing=0.02)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    dc, _, _ = eng.backward(lv, c, tau, f.dp)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=cond_rtol(ref["dp"], tau))


def test_softmin_direct_path_large_cost_over_tau(device):
    """max(C)-min(C) > 40 tau switches the kernel to the per-row stabilised
    softmin; both paths must meet the same tolerance."""
    B, n, L, Q = 2, 16, 300, 4
    ch = random_topologies(B, n, seed=1)
    leaves = random_leaves(B, n, L, Q, seed=2)
    cost = int_cost(Q, seed=3, lo=1, hi=9)
    tau = 0.05
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    dc, _, _ = eng.backward(lv, c, tau, f.dp)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)


def test_softmin_hard_root_flag(device):
    B, n, L, Q = 2, 8, 200, 4
    ch = random_topologies(B, n, seed=8)
    leaves = random_leaves(B, n, L, Q, seed=9)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.3, hard_root=True)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, 0.3, hard_root=True)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    dc, _, _ = eng.backward(lv, c, 0.3, f.dp, hard_root=True)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)


def test_value_and_grad_api_tau0_matches_tie_averaged(device):
    seqs, adj = simulate_leaves(16, 500, 4, 5, seed=1)
    cost = hamming(4)
    total, dc = sankoff_value_and_grad(adj, cost, seqs[:16], 31, 4, 16, device=device)
    from trex_amd.topology import children_from_adjacency

    ch = children_from_adjacency(adj)
    ref = batched_fwd_bwd_ref(ch, normalize_leaves(seqs[None, :16], 4), cost, 0.0)
    assert float(total) == ref["tree_score"][0]
    np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6)


# ---------------------------------------------------------------------------
# size-independent properties at benchmark scale
# ---------------------------------------------------------------------------
def test_c4_scale_properties(device):
    """C4 shape (32 taxa x 5000 sites x 4 states, tau=0.5) on 64 trees:
    determinism, spot checks of sampled trees vs oracle, dC linearity in
    d_tree_score."""
    B, n, L, Q, tau = 64, 32, 5000, 4, 0.5
    ch = random_topologies(B, n, seed=4)
    leaves = random_leaves(B, n, L, Q, seed=5)
    cost = hamming(Q)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f1 = eng.forward(lv, c, tau)
    d1, _, _ = eng.backward(lv, c, tau, f1.dp)
    f2 = eng.forward(lv, c, tau)
    d2, _, _ = eng.backward(lv, c, tau, f2.dp)
    assert torch.equal(f1.tree_score, f2.tree_score) and torch.equal(d1, d2)
    assert torch.equal(f1.dp, f2.dp)
    # the benchmark's fused kernel at this scale == the separate launches
    f3, d3f, _, _ = eng.fwd_bwd(lv, c, tau)
    assert torch.equal(f3.dp, f1.dp) and torch.equal(f3.tree_score, f1.tree_score)
    assert torch.equal(d3f, d1)
    sample = [0, 17, 63]
    ref = batched_fwd_bwd_ref(ch[sample], leaves[sample], cost, tau)
    np.testing.assert_allclose(f1.tree_score.cpu().numpy()[sample], ref["tree_score"],
                               rtol=SOFT_RTOL)
    assert_dp_close(_rows(eng, f1.dp)[sample], ref, SOFT_RTOL)
    dts = torch.zeros(B, device=device)
    dts[sample] = 1.0
    ds, _, _ = eng.backward(lv, c, tau, f1.dp, dts)
    assert_grad_close(ds.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    d3, _, _ = eng.backward(lv, c, tau, f1.dp, torch.full((B,), 3.0, device=device))
    np.testing.assert_allclose(d3.cpu().numpy(), 3.0 * d1.cpu().numpy(), rtol=1e-6)


@pytest.mark.parametrize("tau", [0.0, 0.5, 0.05])
@pytest.mark.parametrize("B,L", [(7, 999), (16, 2000)])
def test_fused_fwd_bwd_equals_separate_launches(device, tau, B, L):
    """trex_sankoff_fwd_bwd == trex_sankoff_fwd + trex_sankoff_bwd, bit for bit
    (same per-wave arithmetic, same fixed-order reductions).  7 x 999 sites
    is 112 work items (<= one wave per CU: the LDS-resident fused kernel);
    16 x 2000 is 512 items (the re-reading fused kernel of the benchmark)."""
    n, Q = 24, 4
    ch = random_topologies(B, n, seed=21)
    leaves = random_leaves(B, n, L, Q, seed=22, missing=0.01)
    cost = int_cost(Q, seed=23, hi=9 if tau == 0.05 else 4)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    dts = torch.linspace(0.5, 2.0, B, device=device)
    f, dc, mg, an = eng.fwd_bwd(lv, c, tau, dts, site_score=True, marginals=True,
                                anc_states=True)
    f2 = eng.forward(lv, c, tau, site_score=True)
    dc2, mg2, an2 = eng.backward(lv, c, tau, f2.dp, dts, marginals=True, anc_states=True)
    assert torch.equal(f.dp, f2.dp)
    assert torch.equal(f.tree_score, f2.tree_score)
    assert torch.equal(f.site_score, f2.site_score)
    assert torch.equal(dc, dc2) and torch.equal(mg, mg2) and torch.equal(an, an2)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau, d_tree_score=dts.cpu().numpy())
    if tau == 0.0:
        np.testing.assert_array_equal(f.tree_score.cpu().numpy(),
                                      ref["tree_score"].astype(np.float32))
        np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6)
    else:
        np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)


def _pectinate(B, nl):
    """caterpillar trees: node nl + i joins leaf i + 1 to node nl + i - 1
    (node nl the cherry (0, 1))."""
    ch = -np.ones((B, 2 * nl - 1, 2), dtype=np.int32)
    ch[:, nl] = (0, 1)
    for i in range(1, nl - 1):
        ch[:, nl + i] = (i + 1, nl + i - 1)
    return ch


@pytest.mark.parametrize("tau", [0.0, 0.5])
@pytest.mark.parametrize("topo", ["random", "balanced", "pectinate"])
def test_deferral_levels_agree(device, monkeypatch, tau, topo):
    """Deferred cherry edges (plan.cpp, TREX_DEFER = 0 none / default on):
    the adjoint rebuilds a deferred cherry's D exactly as the forward built
    it, so the DP table, scores, marginals and ancestral states are bitwise
    the undeferred run's; only the dC accumulation order moves (same value
    within rounding; hard costs also vs fp64 -- with missing leaves the soft
    dC carries the f32 1e5-sentinel rounding the other tests bound, the same
    either way).  16 trees x 2 000 sites: the re-reading fused kernel of the
    benchmark; caterpillar trees have one cherry each."""
    B, L, Q = 16, 2000, 4
    if topo == "random":
        ch = random_topologies(B, 32, seed=41)
    elif topo == "balanced":
        ch = balanced_children(32, B=B)
    else:
        ch = _pectinate(B, 32)
    leaves = random_leaves(B, 32, L, Q, seed=42, missing=0.02)
    cost = int_cost(Q, seed=43, hi=4)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    dts = torch.linspace(0.5, 2.0, B, device=device)
    runs = []
    for level in ("0", "1"):
        monkeypatch.setenv("TREX_DEFER", level)
        eng = _engine(ch, L, Q, device)
        runs.append(eng.fwd_bwd(lv, c, tau, dts, site_score=True, marginals=True,
                                anc_states=True))
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau, d_tree_score=dts.cpu().numpy()) if tau == 0.0 else None
    f0, dc0, mg0, an0 = runs[0]
    for f, dc, mg, an in runs[1:]:
        assert torch.equal(f.dp, f0.dp)
        assert torch.equal(f.tree_score, f0.tree_score)
        assert torch.equal(f.site_score, f0.site_score)
        assert torch.equal(mg, mg0) and torch.equal(an, an0)
        np.testing.assert_allclose(dc.cpu().numpy(), dc0.cpu().numpy(), rtol=1e-5, atol=1e-3)
        if tau == 0.0:
            np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6)


def test_repeated_launches_reset_reduction_counters(device):
    """The in-kernel reductions leave their arrival counters at zero, so
    back-to-back launches (and hipGraph replays) keep producing the same sums."""
    B, n, L, Q = 33, 16, 300, 4
    ch = random_topologies(B, n, seed=31)
    leaves = random_leaves(B, n, L, Q, seed=32)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(hamming(Q), device, torch.float32)
    f0, d0, _, _ = eng.fwd_bwd(lv, c, 0.5)
    t0, dd0 = f0.tree_score.clone(), d0.clone()
    g = torch.cuda.CUDAGraph()
    out = {"dp": f0.dp, "tree_score": f0.tree_score, "d_cost": d0}
    with torch.cuda.graph(g):
        eng.fwd_bwd(lv, c, 0.5, out=out)
    for _ in range(5):
        out["tree_score"].zero_()
        out["d_cost"].zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out["tree_score"], t0) and torch.equal(out["d_cost"], dd0)


# ---------------------------------------------------------------------------
# BASELINE.json configs as parity cases
# ---------------------------------------------------------------------------
def test_config_c1_balanced_8x100x4_hard_forward(device):
    """C1 (BASELINE configs[0]): balanced 8-leaf tree numbered as
    src/trex/evals/benchmark.py:781-791 (parents [8,8,9,9,...,14,14]),
    C = 1 - I, leaves uniform in [0,4) from numpy PCG64(seed=0), integer-cost
    forward + trex backtrack: bit-exact vs the restatement."""
    from trex_amd.topology import create_balanced_binary_tree

    adj = create_balanced_binary_tree(8)
    assert list(adj[:14].argmax(1)) == [8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14]
    seqs = np.random.Generator(np.random.PCG64(0)).integers(0, 4, size=(8, 100)).astype(np.float32)
    cost = hamming(4)
    recon, dp, total = run_sankoff(adj, cost, seqs, 15, 4, 8, return_path=True, device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 15, 4, 8, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


@pytest.mark.parametrize("tau", [1.0, 0.1])
@pytest.mark.parametrize("sim", [True, False])
def test_config_c2_full_size_softmin_fwd_grad(device, tau, sim):
    """C2 (BASELINE configs[1]) at full size: balanced 64-taxa tree x 10 000
    sites x 4 states, C = 1 - I, leaves simulated along the tree (restated
    ground_truth.mutate, 5 mutations per edge, seed 1) or iid uniform (seed 2);
    score and d score / d C vs the fp64 oracle at rtol 1e-5."""
    from trex_amd.topology import children_from_adjacency, create_balanced_binary_tree

    nl, L, Q = 64, 10000, 4
    if sim:
        seqs, adj = simulate_leaves(nl, L, Q, 5, seed=1)
        leaves = seqs[None, :nl].astype(np.int8)
    else:
        adj = create_balanced_binary_tree(nl)
        leaves = random_leaves(1, nl, L, Q, seed=2)
    ch = children_from_adjacency(adj)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    fwd, dc, _, _ = eng.fwd_bwd(_dev(leaves, device), _dev(cost, device, torch.float32), tau)
    np.testing.assert_allclose(fwd.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    assert_dp_close(_rows(eng, fwd.dp), ref, SOFT_RTOL)
