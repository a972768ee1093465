"""BASELINE.json configs at their stated sizes on one MI355X, vs the oracle.

SURVEY.md §8(d) defines the five configs; the bench times C2, C3, C4 (shard
and full batch) and C5 at these sizes, so each is checked here at the same
size (VERDICT r01 "What's weak" 1):

* C2  one balanced 64-taxa tree x 10 000 sites x 4 states: the tau = 0 DP
      table, per-site scores, total and trex reconstruction bit-exact vs the
      fp32 restatement of run_sankoff (sankoff.py:114-188), on every Q <= 4
      kernel (lane-per-site, state-parallel G = 4, library policy);
* C4  128-tree shard and the full 1024-tree batch (32 taxa x 5 000 x 4,
      tau = 0.5): every tree score and, elementwise, every entry of the
      batch dC vs the OpenMP C restatement in fp64 (pinned to the numpy
      oracle by tests/test_cpu_port_cpu.py) at rtol 1e-5, sampled trees vs
      the fp64 oracle at rtol 1e-5, hard path (tau = 0) tree scores
      bit-exact;
* C5  256 taxa (511 nodes) x 50 000 sites x 4 states, three
      TreeOptimizer steps for both GEMM precisions (f16x3 split products and
      f32 MFMA), each vs the fp64 oracle at the GPU's parameters before the
      step: loss, Gram, dA, d loss / dS at rtol 1e-5, d tree_params at its
      fp32 conditioning bound, the Adam updates of both parameter tensors
      (see test_c5_full_size_steps_vs_fp64 for why per step).
      This is the only proof the x3 GEMMs hold at K = L*Q = 200 000.

C3 at full size is in tests/test_sankoff_wide_gpu.py (test_c3_scale_properties).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import (EPS_VJP, assert_bound_close, assert_dp_close, assert_grad_close, hamming,
                    random_leaves, softmax_vjp_bound, tree_param_select,
                    random_topologies, simulate_leaves, surrogate_grad_bounds)
from oracle import cpu_port
from oracle import tree_ref as T
from oracle.sankoff_ref import run_sankoff_ref
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, run_sankoff

pytestmark = pytest.mark.gpu

SOFT_RTOL = 1e-5


def _dev(x, device, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(device).contiguous()


@pytest.mark.parametrize("kernel", ["0", "1", "staged", "auto"])
def test_c2_full_size_hard_dp_table_bitexact(device, kernel, monkeypatch):
    """C2 at full size, tau = 0: trex's (L, n_all, Q) DP table, the total and
    the reconstruction equal the fp32 restatement bit for bit.  kernel "0" =
    lane-per-site, "1" = state-parallel (G = 4, DPP quads), "staged" = the
    state-parallel items as workgroups over the tree's levels, "auto" =
    policy."""
    if kernel == "auto":
        monkeypatch.delenv("TREX_WIDE_SMALLQ", raising=False)
        monkeypatch.delenv("TREX_STAGED", raising=False)
    else:
        monkeypatch.setenv("TREX_WIDE_SMALLQ", "1" if kernel == "staged" else kernel)
        monkeypatch.setenv("TREX_STAGED", "1" if kernel == "staged" else "0")
    nl, L, Q = 64, 10000, 4
    seqs, adj = simulate_leaves(nl, L, Q, 5, seed=1)
    cost = hamming(Q)
    leaf = seqs[:nl].astype(np.float32)
    recon, dp, total = run_sankoff(adj, cost, leaf, 2 * nl - 1, Q, nl, return_path=True,
                                   device=device)
    r_recon, r_dp, r_total = run_sankoff_ref(adj, cost, leaf, 2 * nl - 1, Q, nl,
                                             return_path=True)
    np.testing.assert_array_equal(dp.cpu().numpy(), r_dp)
    np.testing.assert_array_equal(recon.cpu().numpy(), r_recon)
    assert float(total) == float(r_total)


def _c4_case(B):
    n, L, Q = 32, 5000, 4
    ch = random_topologies(B, n, seed=4)
    leaves = random_leaves(B, n, L, Q, seed=5)
    return ch, leaves, hamming(Q), L, Q


@pytest.mark.parametrize("B", [128, 1024])
def test_c4_full_batch_vs_cpu_port(device, B):
    """C4: the bench's 128-tree shard and the whole 1024-tree batch on one
    GPU (2.5 GB DP table), fused fwd + adjoint as timed.  Every tree score
    and every entry of the summed dC vs the OpenMP C restatement in fp64
    (oracle/cpu_port.c, precision "f64") at rtol 1e-5; three sampled trees' score and dC vs the
    fp64 oracle; tau = 0 tree scores bit-exact (integer totals < 2^24)."""
    tau = 0.5
    ch, leaves, cost, L, Q = _c4_case(B)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    lv = _dev(leaves, device)
    c = _dev(cost, device, torch.float32)
    f, dc, _, _ = eng.fwd_bwd(lv, c, tau)
    ts = f.tree_score.cpu().numpy()
    dcn = dc.cpu().numpy()
    p_ts, p_dc, _ = cpu_port.fwd_bwd(ch, leaves, cost, tau, precision="f64")
    np.testing.assert_allclose(ts, p_ts, rtol=SOFT_RTOL)
    assert_grad_close(dcn, p_dc, rtol=SOFT_RTOL)
    sample = [0, B // 2 + 1, B - 1]
    ref = batched_fwd_bwd_ref(ch[sample], leaves[sample], cost, tau)
    np.testing.assert_allclose(ts[sample], ref["tree_score"], rtol=SOFT_RTOL)
    # the sampled trees' DP tables (what the fused kernel writes), per entry
    assert_dp_close(f.dp[sample].transpose(2, 3).cpu().numpy(), ref, SOFT_RTOL)
    dts = torch.zeros(B, device=device)
    dts[sample] = 1.0
    ds, _, _ = eng.backward(lv, c, tau, f.dp, dts)
    assert_grad_close(ds.cpu().numpy(), ref["d_cost"], rtol=SOFT_RTOL)
    # hard path over the whole batch: integer scores, exact
    h = eng.forward(lv, c, 0.0)
    h_ts, _, _ = cpu_port.fwd_bwd(ch, leaves, cost, 0.0, want_grad=False)
    np.testing.assert_array_equal(h.tree_score.cpu().numpy(), h_ts.astype(np.float32))


# ---------------------------------------------------------------------------
# C5: the full optimisation step at its stated size
# ---------------------------------------------------------------------------
def _c5_case():
    from trex_amd.datagen import generate_groundtruth

    nl, L, Q = 256, 50000, 4
    n = 2 * nl - 1
    seqs = generate_groundtruth(nl, Q, 5, L, seed=6).all_sequences.astype(np.int64)
    S = np.zeros((n, L, Q), np.float32)
    S[:nl] = np.eye(Q, dtype=np.float32)[seqs[:nl]]
    rng = np.random.default_rng(7)
    params = {"tree_params": rng.normal(size=(n - 1, nl - 1)).astype(np.float32),
              "ancestors": rng.normal(size=(nl - 1, L, Q)).astype(np.float32)}
    noise = rng.gumbel(size=(n - 1, nl - 1)).astype(np.float32)
    return S, params, noise


def _adam_tol(g, b, m0, v0, k, lr, b1=0.9, b2=0.999, eps=1e-8):
    """Bound on |u(g') - u(g)| over |g' - g| <= b for one optax Adam update u
    (scale_by_adam, bias-corrected, eps_root 0) from the same state (m0, v0):

      |du/dg| <= lr [(1-b1)/(c1 (sqrt(v^) + eps)) + |m^| sqrt((1-b2)/c2) / (sqrt(v^) + eps)^2]

    (using (1-b2)|g| / (c2 sqrt(v^)) <= sqrt((1-b2)/c2)), with |m^| maximised
    and sqrt(v^) minimised over the interval; capped by 2 lr R_k, where
    R_k = (1-b1)/c1 sqrt(c2/(1-b2)) sqrt(sum_i<k (b1^2/b2)^i) bounds |m^ / sqrt(v^)|
    (Cauchy-Schwarz; R_1 = 1, R_3 ~ 1.004)."""
    c1, c2 = 1.0 - b1 ** k, 1.0 - b2 ** k
    ag = np.abs(g)
    mh = (b1 * np.abs(m0) + (1 - b1) * (ag + b)) / c1
    s = np.sqrt((b2 * v0 + (1 - b2) * np.maximum(ag - b, 0.0) ** 2) / c2)
    D = (1 - b1) / (c1 * (s + eps)) + mh * np.sqrt((1 - b2) / c2) / (s + eps) ** 2
    R = (1 - b1) / c1 * np.sqrt(c2 / (1 - b2)) * np.sqrt(sum((b1 * b1 / b2) ** i
                                                            for i in range(k)))
    return lr * np.minimum(b * D, 2 * R), 2 * lr * R


def _adam64(p, g, m0, v0, k, lr, b1=0.9, b2=0.999, eps=1e-8):
    m = b1 * m0 + (1 - b1) * g
    v = b2 * v0 + (1 - b2) * g * g
    return p - lr * (m / (1 - b1 ** k)) / (np.sqrt(v / (1 - b2 ** k)) + eps)


def _f64(t):
    return t.cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("gemm", ["x3", "f32"])
def test_c5_full_size_steps_vs_fp64(device, gemm):
    """Three TreeOptimizer steps at C5 size (511 nodes x 50 000 sites x 4,
    the bench's step), each checked against the fp64 oracle evaluated at the
    GPU's own parameters before that step (tree.py:299-342 + optax adam):

    * loss at rtol 1e-5; the Gram elementwise at rtol 1e-5 (sums of
      non-negative terms); dA and d loss / dS (ancestor rows) elementwise at
      1e-5 times the sum of each entry's terms' magnitudes
      (tests/_cases.py surrogate_grad_bounds);
    * d tree_params at its fp32 conditioning bound (written out below);
    * tree_params after the step == the fp64 Adam update of the GPU's own
      (exactly read back) gradient from the GPU's Adam state, to fp32 rounding;
    * ancestor logits after the fused update_seq-VJP + Adam kernel == the fp64
      Adam update of the fp64 gradient, within the propagation of the asserted
      d loss / dS bound through update_seq's VJP and one Adam update
      (_adam_tol); at most 1 % of entries may sit at the sign-flip cap.

    A per-step check, not a comparison of two 3-step trajectories: Adam's
    first update is lr * sign(g), so a gradient entry within its fp32 error
    of 0 moves its parameter by +-lr either way, and two trajectories then
    legitimately differ by O(lr) in those entries (seen at this size: a few
    dozen of 130 050 tree_params).  This is the only proof the x3 GEMMs hold
    at K = L*Q = 200 000."""
    from trex_amd import tree as G

    S, params, noise = _c5_case()
    n, L, Q = S.shape
    nl = (n + 1) // 2
    lr = 0.01
    opt = G.TreeOptimizer(_dev(S, device), {k: _dev(v, device) for k, v in params.items()},
                          lr=lr, gemm=gemm)
    assert opt.gemm == gemm
    nz = _dev(noise, device)
    temps = [2.0, 1.9996, 1.9992]
    losses = []
    ratios = {k: [] for k in ("dA", "dS", "d tree_params", "ancestors", "ancestors at cap")}
    for k in range(3):
        T_k = temps[k]
        nxt = temps[k + 1] if k + 1 < len(temps) else T_k
        p64 = {kk: _f64(v) for kk, v in opt.params.items()}
        mu0 = {kk: _f64(v) for kk, v in opt.opt.mu.items()}
        nu0 = {kk: _f64(v) for kk, v in opt.opt.nu.items()}
        loss = float(opt.step(T_k, nz, next_temperature=nxt))
        torch.cuda.synchronize()
        losses.append(loss)
        # fp64 oracle at the GPU's parameters before this step
        S64 = T.update_seq(p64["ancestors"], S, T_k)
        A64 = T.update_tree(p64["tree_params"], noise, 1.0)
        val, dS64, dA64 = T.compute_surrogate_cost_grads(S64, A64)
        dA64 = dA64 + T_k * T.enforce_graph_constraints_grad(A64, 10.0)
        rloss = val + T_k * T.enforce_graph_constraints(A64, 10.0)
        np.testing.assert_allclose(loss, rloss, rtol=SOFT_RTOL)
        F = S64.reshape(n, -1)
        assert_grad_close(opt.G.cpu().numpy(), F @ F.T, rtol=SOFT_RTOL, what="G")
        del F
        cg = T_k * T.enforce_graph_constraints_grad(A64, 10.0)
        bS, bA = surrogate_grad_bounds(S64, A64, SOFT_RTOL, constraint_grad=cg)
        ratios["dA"].append(assert_bound_close(opt.dA.cpu().numpy(), dA64, bA, what="dA"))
        ratios["dS"].append(assert_bound_close(opt.dS[nl:].cpu().numpy(), dS64[nl:], bS[nl:],
                                               what="dS"))
        # d tree_params = A (dA - sum_k A dA) per row (update_tree's softmax
        # VJP, tree.py:50-107), per entry: the dA bound just asserted carried
        # through that VJP, plus the VJP's own fp32 rounding at the exact
        # cotangent's magnitude (tests/_cases.py loss_grad_bounds)
        g_th = _f64(opt.grads["tree_params"])
        ref_th = T.update_tree_vjp(p64["tree_params"], noise, 1.0, None, A64, dA64)
        dz = (softmax_vjp_bound(A64, bA, axis=1)
              + EPS_VJP * softmax_vjp_bound(A64, np.abs(dA64), axis=1))
        ratios["d tree_params"].append(assert_bound_close(
            g_th, ref_th, tree_param_select(dz, ref_th.shape[1]), what="d tree_params"))
        del bA, dz
        # tree_params: fp64 Adam of the GPU's own gradient, to fp32 rounding
        new_th = _f64(opt.params["tree_params"])
        want = _adam64(p64["tree_params"], g_th, mu0["tree_params"], nu0["tree_params"],
                       k + 1, lr)
        slack = 4.8e-7 * np.abs(want) + 1e-5 * lr
        assert np.all(np.abs(new_th - want) <= slack), np.abs(new_th - want).max()
        # ancestors: fused VJP + Adam vs fp64.  The gradient's bound per entry
        # is the asserted dS bound through update_seq's softmax VJP plus the
        # VJP's own rounding (loss_grad_bounds), then _adam_tol carries it
        # through one Adam update from the GPU's own state
        anc = p64["ancestors"]
        S_anc = S64[nl:]
        g_anc = T.update_seq_vjp(anc, T_k, S_anc, dS64[nl:])
        b = T_k * (softmax_vjp_bound(S_anc, bS[nl:])
                   + EPS_VJP * softmax_vjp_bound(S_anc, np.abs(dS64[nl:])))
        del S64, dS64, bS
        tol, cap = _adam_tol(g_anc, b, mu0["ancestors"], nu0["ancestors"], k + 1, lr)
        want = _adam64(anc, g_anc, mu0["ancestors"], nu0["ancestors"], k + 1, lr)
        new_anc = _f64(opt.params["ancestors"])
        # + the update's own fp32 rounding (a few ulps of the parameter and of
        # the lr-sized step)
        ratios["ancestors"].append(assert_bound_close(
            new_anc, want, tol + 4.8e-7 * np.abs(want) + 4.8e-7 * lr * 2, what="ancestors"))
        # entries whose gradient bound straddles 0 may move by the sign-flip
        # cap (Adam's first steps are ~lr sign(g)); that is a property of the
        # data, measured here, and the check is only meaningful if it is rare
        at_cap = float(np.mean(tol >= cap))
        ratios["ancestors at cap"].append(at_cap)
        assert at_cap < 1e-3, at_cap  # measured 5e-5 (step 1) at this size
        del anc, S_anc, g_anc, b, tol, want, new_anc
    print(f"C5 {gemm}: max err / bound per step", {k: [f"{x:.3g}" for x in v]
                                                   for k, v in ratios.items()})
    assert losses[0] > losses[1] > losses[2]
