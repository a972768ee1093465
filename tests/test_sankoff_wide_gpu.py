"""GPU parity of the Q > 4 (lane-per-state) Sankoff kernels vs the CPU oracle.

Same bars as tests/test_sankoff_gpu.py: hard DP table / totals / ancestral
states bit-exact, hard gradient rtol 1e-6, softmin score / gradient rtol 1e-5
elementwise vs the fp64 oracle, marginals elementwise at max(1e-5, 8 eps
path_dmax / tau) per entry (fp32 D's conditioning, tests/_cases.py).  Q > 4 tables are site-major
([B][n_int][L][Q], trex_hip.h), so oracle tables are transposed to compare.
Q = 20 is the protein alphabet of BASELINE config C3; 5, 13, 21 and 32
exercise the padded-state groups (G = 8, 16, 32); 61 and 64 are codon
alphabets (G = 64, one site per wave; trex sizes everything from n_states
with no cap, sankoff.py:151-152).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (assert_dp_close, assert_grad_close, assert_marginals_close, balanced_children,
                    clear_argmax_mask, cond_rtol, hamming, int_cost, random_leaves,
                    random_topologies)
from oracle.sankoff_ref import run_sankoff_ref
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, run_sankoff
from trex_amd.topology import adjacency_from_children

pytestmark = pytest.mark.gpu

SOFT_RTOL = 1e-5


@pytest.fixture(autouse=True, params=["wave", "staged"])
def wide_kernel(request, monkeypatch):
    """Every case runs on the one-wave-per-item kernel (sankoff_wide.hip)
    and on the staged workgroup kernel (sankoff_staged.hip)."""
    monkeypatch.setenv("TREX_STAGED", "1" if request.param == "staged" else "0")
    return request.param


def _engine(children, L, Q, device):
    return SankoffEngine(TreePlan(children), L, Q, device)


def _dev(x, device, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


def _sm(t):
    """engine site-major table (B, n_int, L, Q) -> oracle layout (B, n_int, Q, L)."""
    return t.cpu().numpy().transpose(0, 1, 3, 2)


def test_site_major_layout_flag(device):
    eng = _engine(random_topologies(1, 4, seed=0), 10, 20, device)
    assert eng.site_major and eng.dp_shape == (1, 3, 10, 20)
    eng4 = _engine(random_topologies(1, 4, seed=0), 10, 4, device)
    assert eng4.site_major and eng4.dp_shape == (1, 3, 10, 4)  # every Q since v4


@pytest.mark.parametrize("Q", [5, 20, 21, 61, 64])
@pytest.mark.parametrize("L", [1, 7, 130, 1000])
def test_run_sankoff_bitexact_wide(device, Q, L):
    ch = random_topologies(1, 16, seed=200 + L + Q)[0]
    adj = adjacency_from_children(ch)[0]
    rng = np.random.default_rng(L * 3 + Q)
    seqs = rng.integers(0, Q, size=(16, L)).astype(np.float32)
    cost = int_cost(Q, seed=Q + L)
    recon, dp, total = run_sankoff(adj, cost, seqs, 31, Q, 16, return_path=True, device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, seqs, 31, Q, 16, return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


@pytest.mark.parametrize("L,Q,n", [(1, 20, 8), (300, 20, 16), (1000, 20, 64), (777, 5, 12),
                                   (513, 13, 20), (200, 32, 10), (64, 21, 9), (300, 61, 12),
                                   (65, 64, 9)])
def test_batched_hard_fwd_grad_wide(device, L, Q, n):
    B = 4
    ch = random_topologies(B, n, seed=L + n + Q)
    leaves = random_leaves(B, n, L, Q, seed=L + Q, missing=0.05)
    cost = int_cost(Q, seed=L + 1)
    dts_np = np.arange(1, B + 1) / B
    ref = batched_fwd_bwd_ref(ch, leaves, cost, 0.0, d_tree_score=dts_np)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, 0.0, dp=True, site_score=True)
    np.testing.assert_array_equal(_sm(f.dp), ref["dp"].astype(np.float32))
    np.testing.assert_array_equal(f.site_score.cpu().numpy(),
                                  ref["site_score"].astype(np.float32))
    np.testing.assert_array_equal(f.tree_score.cpu().numpy(), ref["tree_score"].astype(np.float32))
    dts = torch.as_tensor(dts_np, dtype=torch.float32, device=device)
    dc, mg, _ = eng.backward(lv, c, 0.0, f.dp, dts, marginals=True)
    np.testing.assert_allclose(dc.cpu().numpy(), ref["d_cost"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(_sm(mg), ref["marginals"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("bt", ["split", "0"])
@pytest.mark.parametrize("Q,ties", [(20, False), (20, True), (7, False), (5, True), (32, True),
                                    (61, False)])
def test_backtrack_wide_matches_reference(device, Q, ties, bt, monkeypatch):
    """trex-exact states on both live backtrack kernels: 8 lanes per site
    (Q <= 32, the policy) and one lane per site (codons, ragged, forced here
    by TREX_BT4=0); Hamming costs (ties: the first-index argmin rule across
    the lanes' state ranges)."""
    if bt == "0":
        monkeypatch.setenv("TREX_BT4", "0")
    else:
        monkeypatch.delenv("TREX_BT4", raising=False)
    B, n, L = 3, 24, 515
    ch = random_topologies(B, n, seed=3 + Q)
    leaves = random_leaves(B, n, L, Q, seed=4 + Q)
    cost = hamming(Q) if ties else int_cost(Q, seed=5)
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


@pytest.mark.parametrize("tau", [1.0, 0.5, 0.1])
@pytest.mark.parametrize("L,n,Q", [(100, 8, 20), (1000, 64, 20), (301, 16, 6), (257, 12, 32),
                                   (129, 10, 61)])
def test_softmin_fwd_grad_wide_vs_fp64(device, tau, L, n, Q):
    B = 2
    ch = random_topologies(B, n, seed=n + 13)
    leaves = random_leaves(B, n, L, Q, seed=L + 5)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f = eng.forward(lv, c, tau, dp=True, site_score=True)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    np.testing.assert_allclose(f.site_score.cpu().numpy(), ref["site_score"], rtol=SOFT_RTOL,
                               atol=1e-5)
    assert_dp_close(_sm(f.dp), ref, SOFT_RTOL)
    dc, mg, anc = eng.backward(lv, c, tau, f.dp, marginals=True, anc_states=True)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    m = ref["marginals"]
    _, rt = assert_marginals_close(_sm(mg), m, ch, ref["dp"], tau)
    clear = clear_argmax_mask(m, rt)
    np.testing.assert_array_equal(anc.cpu().numpy()[clear], m.argmax(axis=2)[clear])


def test_softmin_wide_direct_path_and_hard_root(device):
    """range(C) > 40 tau selects the per-row stabilised softmin; hard_root
    scores the root with a hard min."""
    B, n, L, Q = 2, 16, 200, 20
    ch = random_topologies(B, n, seed=1)
    leaves = random_leaves(B, n, L, Q, seed=2)
    cost = int_cost(Q, seed=3, lo=1, hi=9)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    for tau, hard_root in ((0.05, False), (0.3, True)):
        ref = batched_fwd_bwd_ref(ch, leaves, cost, tau, hard_root=hard_root)
        f = eng.forward(lv, c, tau, hard_root=hard_root)
        np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"],
                                   rtol=SOFT_RTOL)
        dc, _, _ = eng.backward(lv, c, tau, f.dp, hard_root=hard_root)
        # tau = 0.05 with costs up to 9: tiny weights (e^-40) carry the fp32
        # D conditioning |D| / tau (measured 4.6e-5 on 20 of 400 entries)
        assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=cond_rtol(ref["dp"], tau))


def test_softmin_wide_missing_leaves(device):
    B, n, L, Q, tau = 2, 8, 100, 20, 1.0
    ch = random_topologies(B, n, seed=19)
    leaves = random_leaves(B, n, L, Q, seed=103, missing=0.03)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    f = eng.forward(_dev(leaves, device), _dev(cost, device, torch.float32), tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    dc, _, _ = eng.backward(_dev(leaves, device), _dev(cost, device, torch.float32), tau, f.dp)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=cond_rtol(ref["dp"], tau))


@pytest.mark.parametrize("site", ["1", "0"])
@pytest.mark.parametrize("tau", [1000.0, 200.0])
def test_softmin_missing_leaves_adjoint_high_tau(device, tau, site, monkeypatch):
    """Leaves with a missing state send trex's all-1e5 row's message
    (sankoff.py:49-52,152), which depends on C through log sum_j K_ij; its
    adjoint adds g_i K_ij / sum_j K_ij to dC at every such site.  At large
    tau the fp32 1e5 offset conditions dC only to 2 eps 1e5 / tau (1.2e-5 at
    tau = 1000), so the missing-leaf term (a few % of dC here) is checked
    sharply -- on the lane-per-site kernel (TREX_SITE=1, ADVICE r03: it used
    to drop the term) and on the state-parallel kernel."""
    monkeypatch.setenv("TREX_SITE", site)
    B, n, L, Q = 2, 12, 300, 20
    ch = random_topologies(B, n, seed=29)
    leaves = random_leaves(B, n, L, Q, seed=31, missing=0.05)
    cost = int_cost(Q, seed=3)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = _engine(ch, L, Q, device)
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    f, dc, _, _ = eng.fwd_bwd(lv, c, tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=2 * cond_rtol(ref["dp"], tau))


@pytest.mark.parametrize("tau", [0.0, 0.5])
def test_fused_equals_separate_wide(device, tau):
    B, n, L, Q = 3, 20, 999, 20
    ch = random_topologies(B, n, seed=21)
    leaves = random_leaves(B, n, L, Q, seed=22, missing=0.01)
    cost = int_cost(Q, seed=23)
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


def test_c3_scale_properties(device):
    """C3 at its stated size: 64 taxa x 10 000 sites x 20 states, softmin
    (tau 0.5) + ancestral reconstruction.  Score, dC, DP table, marginals and
    soft ancestral states vs the fp64 oracle; determinism; tau = 0 DP table,
    total and trex ancestral states bit-exact vs the reference restatement."""
    n, L, Q, tau = 64, 10000, 20, 0.5
    ch = random_topologies(1, n, seed=31)
    leaves = random_leaves(1, n, L, Q, seed=32)
    cost = int_cost(Q, seed=3)
    eng = _engine(ch, L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f, dc, mg, an = eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True)
    f2, dc2, mg2, an2 = eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True)
    assert torch.equal(f.tree_score, f2.tree_score) and torch.equal(dc, dc2)
    assert torch.equal(mg, mg2) and torch.equal(an, an2)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    np.testing.assert_allclose(f.tree_score.cpu().numpy(), ref["tree_score"], rtol=SOFT_RTOL)
    assert_grad_close(dc.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    # full-size DP table, per entry at 1e-5 of its terms' magnitudes (D sums
    # messages of either sign: tests/_cases.py assert_dp_close), marginals and
    # soft ancestral states (the elementwise marginal rule of
    # tests/test_sankoff_gpu.py: fp32 D's conditioning along the root path)
    assert_dp_close(_sm(f.dp), ref, SOFT_RTOL)
    m = ref["marginals"]
    _, rt = assert_marginals_close(_sm(mg), m, ch, ref["dp"], tau)
    clear = clear_argmax_mask(m, rt)
    np.testing.assert_array_equal(an.cpu().numpy()[clear], m.argmax(axis=2)[clear])
    del ref, m, rt, clear
    # hard path + trex backtrack at full size: DP table, total, states exact
    h = eng.forward(lv, c, 0.0)
    anc = eng.backtrack(c, h.dp).cpu().numpy()[0]
    adj = adjacency_from_children(ch)[0]
    r = run_sankoff_ref(adj, cost, leaves[0].astype(np.float32), 2 * n - 1, Q, n,
                        return_path=True)
    assert float(h.tree_score[0]) == float(r[2])
    np.testing.assert_array_equal(h.dp.cpu().numpy()[0], r[1][:, n:, :].transpose(1, 0, 2))
    np.testing.assert_array_equal(anc.astype(np.float32), r[0][n:])


@pytest.mark.parametrize("tau", [0.5, 0.02])  # 0.02: range / tau > 40, the gate refuses
def test_site_gate_repeat_calls_no_sync(device, tau, wide_kernel):
    """Every call runs the lane-per-site gate (v8's TREX_FLAG_SITE_REUSE is
    gone): repeated eager calls on one engine equal a fresh engine's bit for
    bit, including after the cost is changed in place, and none of them
    synchronises with the host (torch's sync debug mode raises on any)."""
    B, n, L, Q = 2, 16, 700, 20
    ch = random_topologies(B, n, seed=31)
    lv = _dev(random_leaves(B, n, L, Q, seed=32, missing=0.01), device)
    c = _dev(int_cost(Q, seed=33), device, torch.float32)
    eng = _engine(ch, L, Q, device)

    def fresh(cost):
        f, dc, mg, _ = _engine(ch, L, Q, device).fwd_bwd(lv, cost.clone(), tau, marginals=True)
        return f.tree_score, dc, mg

    ref = fresh(c)
    outs = {"dp": torch.empty(eng.dp_shape, device=device),
            "marginals": torch.empty(eng.dp_shape, device=device),
            "tree_score": torch.empty(B, device=device),
            "d_cost": torch.empty(Q, Q, device=device)}
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for _ in range(10):
            eng.fwd_bwd(lv, c, tau, marginals=True, out=outs)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    assert torch.equal(outs["tree_score"], ref[0]) and torch.equal(outs["d_cost"], ref[1])
    assert torch.equal(outs["marginals"], ref[2])
    c.mul_(2.0)
    ref2 = fresh(c)
    for i in range(3):
        f, dc, mg, _ = eng.fwd_bwd(lv, c, tau, marginals=True)
        assert torch.equal(f.tree_score, ref2[0]) and torch.equal(dc, ref2[1]), i
        assert torch.equal(mg, ref2[2]), i


@pytest.mark.parametrize("topo", ["balanced", "random"])
@pytest.mark.parametrize("knob,Q", [("TREX_SITE_CHERRY", 20), ("TREX_SITE_SROW", 20),
                                    ("TREX_SITE_SROW", 13)])
def test_site_kernel_shortcuts_are_bitwise_neutral(device, monkeypatch, topo, knob, Q):
    """The lane-per-site kernel's two shortcuts are bitwise what they
    replace: the cherry tables (wide_dev.h site_pair_tables: a height-1 row's
    forward message and softmin row sums by its children's code pair, built
    by the gate) == the per-lane mat-vecs (TREX_SITE_CHERRY=0, the Q = 20
    build without tables), and the fused kernel's kept s rows (the forward's
    K u of each computed child, re-read by the adjoint) == the adjoint's own
    mat-vec (TREX_SITE_SROW=0): DP table, scores, dC, marginals and soft
    ancestral states, fused and separate launches, with missing leaf states
    (code Q: the all-1e5 row's message) and cherries both under height-2
    rows and directly under task rows (random topologies)."""
    B, n, L, tau = 2, 64, 777, 0.5
    ch = (balanced_children(n, B) if topo == "balanced" else random_topologies(B, n, seed=71))
    leaves = random_leaves(B, n, L, Q, seed=72, missing=0.03)
    cost = int_cost(Q, seed=73)
    lv, c = _dev(leaves, device), _dev(cost, device, torch.float32)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv(knob, flag)
        eng = _engine(ch, L, Q, device)
        f, dc, mg, an = eng.fwd_bwd(lv, c, tau, site_score=True, marginals=True,
                                    anc_states=True)
        f2 = eng.forward(lv, c, tau)
        dc2, _, _ = eng.backward(lv, c, tau, f2.dp)
        torch.cuda.synchronize()
        runs.append((f.dp.clone(), f.tree_score.clone(), f.site_score.clone(), dc.clone(),
                     mg.clone(), an.clone(), f2.dp.clone(), dc2.clone()))
    for a, b, what in zip(runs[0], runs[1], ("dp", "tree", "site", "dC", "marg", "anc", "dp2",
                                             "dC2")):
        assert torch.equal(a, b), what
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    assert_grad_close(runs[0][3].cpu().numpy(), ref["d_cost"], rtol=cond_rtol(ref["dp"], tau))
    assert_dp_close(_sm(runs[0][0]), ref, SOFT_RTOL)


def test_site_kernel_smaller_workspace_recomputes_s_rows_bitwise(device):
    """the fused lane-per-site call's kept s rows are optional --
    a workspace of trex_workspace_bytes - B n_int L Q 4 bytes is accepted
    (the adjoint recomputes s, bitwise the same: the TREX_SITE_SROW=0 path)
    and one byte less is refused (include/trex_hip.h)."""
    from trex_amd._lib import TrexError

    B, n, L, Q, tau = 2, 64, 777, 20, 0.5
    ch = random_topologies(B, n, seed=81)
    leaves = random_leaves(B, n, L, Q, seed=82, missing=0.03)
    lv = _dev(leaves, device)
    c = _dev(int_cost(Q, seed=83), device, torch.float32)
    eng = _engine(ch, L, Q, device)
    f, dc, mg, _ = eng.fwd_bwd(lv, c, tau, marginals=True)
    ref = (f.dp.clone(), f.tree_score.clone(), dc.clone(), mg.clone())
    n_int = n - 1  # n taxa: 2n - 1 nodes, n - 1 internal rows
    small = eng.workspace.numel() - B * n_int * L * Q * 4
    full = eng.workspace
    try:
        eng.workspace = full[:small]
        f2, dc2, mg2, _ = eng.fwd_bwd(lv, c, tau, marginals=True)
        torch.cuda.synchronize()
        assert torch.equal(f2.dp, ref[0]) and torch.equal(f2.tree_score, ref[1])
        assert torch.equal(dc2, ref[2]) and torch.equal(mg2, ref[3])
        eng.workspace = full[:small - 1]
        with pytest.raises(TrexError):
            eng.fwd_bwd(lv, c, tau)
    finally:
        eng.workspace = full
