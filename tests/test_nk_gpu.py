"""GPU parity of the NK landscape-aware path (trex_nk_*) vs the fp64 oracle
(oracle/nk_ref.py; reference src/trex/evals/benchmark.py:235-306, 586-663).

Tolerances: logits are fp32 sums of Q^k products of probabilities and table
entries, accumulated in a fixed order: rtol 1e-5; one-hot parents reproduce
the table entries exactly.  Loss: rtol 1e-5.  Gradients: per entry, 1e-5 of
the magnitudes of the entry's terms carried through the chain
(tests/_cases.py landscape_grad_bound).  The optimisation loop is checked
step by step against the oracle at the GPU's own parameters.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import assert_bound_close, landscape_grad_bound
from oracle import nk_ref as nk
from trex_amd import nk as NK

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _n(x):
    return x.detach().cpu().numpy().astype(np.float64)


def _case(n_leaves, L, Q, k, seed, mask=False, root_self=False):
    rng = np.random.default_rng(seed)
    n_all = 2 * n_leaves - 1
    inter, F = nk.random_landscape(L, k, Q, seed=seed + 1)
    leaves = rng.integers(0, Q, size=(n_leaves, L))
    A = np.zeros((n_all, n_all), np.float32)
    par = n_leaves + np.arange(n_all - 1) // 2
    A[np.arange(n_all - 1), par] = 1.0
    if root_self:
        A[-1, -1] = 1.0  # trex's update_tree convention (tree.py:104)
    anc = rng.normal(size=(n_all - n_leaves, L, Q)).astype(np.float32)
    m = (rng.random(L) > 0.25) if mask else None
    S0 = np.zeros((n_all, L, Q), np.float32)
    S0[np.arange(n_leaves)[:, None], np.arange(L)[None, :], leaves] = 1.0
    return dict(S0=S0, A=A, inter=inter, F=F, anc=anc, mask=m, n_leaves=n_leaves,
                leaves=leaves, n_all=n_all)


@pytest.mark.parametrize("Q,k,P,L", [(4, 2, 7, 33), (4, 4, 70, 20), (20, 2, 5, 9), (2, 6, 3, 40),
                                     (20, 1, 65, 12), (3, 3, 1, 1), (2, 10, 63, 15)])
def test_parental_logits_vs_oracle(device, Q, k, P, L):
    rng = np.random.default_rng(Q * 100 + k)
    inter, F = nk.random_landscape(L, k, Q, seed=k)
    seqs = rng.dirichlet(np.ones(Q), size=(P, L)).astype(np.float32)
    land = NK.NKLandscape(inter, F, Q, device)
    out = _n(NK.compute_parental_logits(torch.as_tensor(seqs, device=device), land, k))
    ref = nk.compute_parental_logits(seqs.astype(np.float64), inter, F.astype(np.float64), k)
    np.testing.assert_allclose(out, ref, rtol=RTOL, atol=1e-6)


def test_parental_logits_one_hot_exact(device):
    Q, k, L, P = 4, 3, 17, 9
    rng = np.random.default_rng(0)
    inter, F = nk.random_landscape(L, k, Q, seed=2)
    seqs = np.eye(Q, dtype=np.float32)[rng.integers(0, Q, size=(P, L))]
    land = NK.NKLandscape(inter, F, Q, device)
    out = NK.compute_parental_logits(torch.as_tensor(seqs, device=device), land, k)
    ref = nk.compute_parental_logits(seqs.astype(np.float64), inter, F.astype(np.float64), k)
    np.testing.assert_array_equal(out.cpu().numpy(), ref.astype(np.float32))


def test_parental_logits_k0_and_padded(device):
    L, Q = 10, 4
    F0 = np.random.default_rng(1).uniform(size=(L, Q)).astype(np.float32)
    seqs = np.random.default_rng(2).dirichlet(np.ones(Q), size=(3, L)).astype(np.float32)
    land0 = NK.NKLandscape(np.zeros((L, 0), np.int32), F0, Q, device)
    out = NK.compute_parental_logits(torch.as_tensor(seqs, device=device), land0, 0)
    np.testing.assert_array_equal(out.cpu().numpy(), np.broadcast_to(F0, (3, L, Q)))
    # padded landscape (padding.py:144-216): k_eff = padded k, as the reference
    inter, F = nk.random_landscape(L, 2, Q, seed=4)
    ip, Fp = nk.pad_landscape(inter, F, 3, Q)
    landp = NK.NKLandscape(ip, Fp, Q, device)
    out = _n(NK.compute_parental_logits(torch.as_tensor(seqs, device=device), landp, 2))
    ref = nk.compute_parental_logits(seqs.astype(np.float64), ip, Fp.astype(np.float64), 2)
    np.testing.assert_allclose(out, ref, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("n_leaves,L,Q,k,mask,root_self",
                         [(4, 12, 4, 2, False, False), (8, 30, 4, 3, True, False),
                          (16, 20, 20, 1, True, True), (5, 7, 3, 2, False, True),
                          (32, 15, 2, 10, False, False)])  # benchmark.py:981-985 eval shape
def test_landscape_loss_and_grad_vs_oracle(device, n_leaves, L, Q, k, mask, root_self):
    c = _case(n_leaves, L, Q, k, seed=L + Q, mask=mask, root_self=root_self)
    land = NK.NKLandscape(c["inter"], c["F"], Q, device)
    lam, T = 0.8, 1.0
    fn = NK.LandscapeAwareLoss(c["A"], n_leaves, land, lam, k, temperature=T,
                               seq_mask=c["mask"])
    loss, g = fn.value_and_grad(torch.as_tensor(c["anc"], device=device),
                                torch.as_tensor(c["S0"], device=device))
    args = (c["anc"].astype(np.float64), c["S0"].astype(np.float64), n_leaves, c["inter"],
            c["F"].astype(np.float64), c["A"], lam, k, T, c["mask"])
    rl, rg = nk.landscape_loss_grad(*args)
    np.testing.assert_allclose(float(loss[0]), rl, rtol=RTOL)
    assert_bound_close(_n(g), rg, landscape_grad_bound(*args, rtol=RTOL), what="d ancestors")
    # functional form == class
    lf = NK.landscape_aware_loss(torch.as_tensor(c["anc"], device=device),
                                 torch.as_tensor(c["S0"], device=device), n_leaves, land, c["A"],
                                 c["n_all"], lam, k, T, c["mask"])
    assert float(lf) == float(loss[0])


def test_landscape_loss_real_k0_is_surrogate(device):
    c = _case(4, 9, 4, 2, seed=3)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    fn = NK.LandscapeAwareLoss(c["A"], 4, land, 0.5, 0)
    loss, g = fn.value_and_grad(torch.as_tensor(c["anc"], device=device),
                                torch.as_tensor(c["S0"], device=device))
    args = (c["anc"].astype(np.float64), c["S0"].astype(np.float64), 4, c["inter"], c["F"],
            c["A"], 0.5, 0)
    rl, rg = nk.landscape_loss_grad(*args)
    np.testing.assert_allclose(float(loss[0]), rl, rtol=RTOL)
    assert_bound_close(_n(g), rg, landscape_grad_bound(*args, rtol=RTOL), what="d ancestors")


def test_landscape_loss_deterministic(device):
    c = _case(16, 64, 4, 3, seed=11, mask=True)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    fn = NK.LandscapeAwareLoss(c["A"], 16, land, 1.0, 3, seq_mask=c["mask"])
    a = torch.as_tensor(c["anc"], device=device)
    s = torch.as_tensor(c["S0"], device=device)
    l1, g1 = fn.value_and_grad(a, s)
    l1, g1 = l1.clone(), g1.clone()
    l2, g2 = fn.value_and_grad(a, s)
    assert torch.equal(l1, l2) and torch.equal(g1, g2)


def test_landscape_loss_follows_masked_sequence_updates(device):
    """The loss caches its copy of masked_sequences between calls: writing
    into the same tensor, or passing another one, must reach the result
    (the cache keys on the tensor object and torch's version counter)."""
    c = _case(8, 20, 4, 2, seed=5)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    fn = NK.LandscapeAwareLoss(c["A"], 8, land, 0.7, 2)
    a = torch.as_tensor(c["anc"], device=device)
    s = torch.as_tensor(c["S0"], device=device)
    alt = c["S0"].copy()
    alt[:8] = np.roll(alt[:8], 1, axis=-1)  # every leaf's state changed
    l0 = float(fn.value_and_grad(a, s)[0][0])
    s.copy_(torch.as_tensor(alt, device=device))  # in-place write
    l1 = float(fn.value_and_grad(a, s)[0][0])
    l2 = float(fn.value_and_grad(a, torch.as_tensor(c["S0"], device=device))[0][0])
    r0 = nk.landscape_loss_grad(c["anc"].astype(np.float64), c["S0"].astype(np.float64), 8,
                                c["inter"], c["F"].astype(np.float64), c["A"], 0.7, 2)[0]
    r1 = nk.landscape_loss_grad(c["anc"].astype(np.float64), alt.astype(np.float64), 8,
                                c["inter"], c["F"].astype(np.float64), c["A"], 0.7, 2)[0]
    np.testing.assert_allclose([l0, l1, l2], [r0, r1, r0], rtol=RTOL)
    assert abs(r1 - r0) > 1e-3 * abs(r0)


def test_run_landscape_aware_adam_matches_oracle_loop(device):
    """The reference driver (run_trex_landscape_aware_configurable) == the
    same loop stepped here (LandscapeAwareLoss + Adam), bitwise; and each
    step of that loop vs the fp64 oracle at the GPU's own parameters before
    the step: loss at rtol 1e-5, the gradient per entry
    (landscape_grad_bound), the updated parameters == the fp64 optax Adam
    update of the GPU's own gradient from the GPU's moments, to fp32
    rounding.  A per-step check, not two 5-step trajectories: Adam's first
    update is lr * sign(g), so two runs legitimately drift apart by O(lr)
    wherever a gradient sits within its fp32 error of 0.  Then the argmax
    reconstruction of the final parameters."""
    from trex_amd.tree import Adam

    c = _case(4, 10, 4, 2, seed=21)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    steps, lr = 5, 0.05
    out, losses = NK.run_trex_landscape_aware_configurable(
        c["leaves"], c["n_all"], 4, 4, land, 0.6, c["A"], c["anc"], real_k=2,
        learning_rate=lr, n_iterations=steps, return_losses=True)
    fn = NK.LandscapeAwareLoss(c["A"], 4, land, 0.6, 2)
    params = {"ancestors": torch.as_tensor(c["anc"], device=device).clone()}
    opt = Adam(params, lr)
    S0 = torch.as_tensor(c["S0"], device=device)
    F64 = c["F"].astype(np.float64)
    mine = []
    for step in range(1, steps + 1):
        p64 = _n(params["ancestors"])
        mu0, nu0 = _n(opt.mu["ancestors"]), _n(opt.nu["ancestors"])
        loss, g = fn.value_and_grad(params["ancestors"], S0)
        mine.append(float(loss[0]))
        g64 = _n(g)
        args = (p64, c["S0"].astype(np.float64), 4, c["inter"], F64, c["A"], 0.6, 2)
        rl, rg = nk.landscape_loss_grad(*args)
        np.testing.assert_allclose(mine[-1], rl, rtol=RTOL)
        assert_bound_close(g64, rg, landscape_grad_bound(*args, rtol=RTOL), what=f"grad {step}")
        opt.step(params, {"ancestors": g})
        b1, b2, eps = 0.9, 0.999, 1e-8
        mu = (1 - b1) * g64 + b1 * mu0
        nu = (1 - b2) * g64 ** 2 + b2 * nu0
        want = p64 - lr * (mu / (1 - b1 ** step)) / (np.sqrt(nu / (1 - b2 ** step)) + eps)
        got = _n(params["ancestors"])
        assert np.all(np.abs(got - want) <= 4.8e-7 * np.abs(want) + 1e-5 * lr), step
    torch.cuda.synchronize()
    assert mine == [float(x) for x in _n(losses)]
    assert torch.equal(out.cpu(), params["ancestors"].argmax(-1).cpu().to(out.dtype))


def test_nk_adam_step_graph_replay_is_bitwise_eager(device):
    """The reference's eval shape (32 leaves, 15 sites, Q = 2, K = 10;
    benchmark.py:981-985): one landscape-aware loss + grad + Adam step
    captured in a hipGraph (the Adam count lives on the device,
    trex_step_advance) and replayed 6 times == 6 eager steps, bitwise; and the
    device-count Adam == the host-count trex_adam_step, bitwise."""
    from trex_amd._lib import check, lib, ptr, stream_handle
    from trex_amd.tree import Adam

    c = _case(32, 15, 2, 10, seed=5)
    land = NK.NKLandscape(c["inter"], c["F"], 2, device)
    S0 = torch.as_tensor(c["S0"], device=device)
    runs = []
    for mode in ("eager", "graph", "host"):
        fn = NK.LandscapeAwareLoss(c["A"], c["n_leaves"], land, 3.0, 10)
        params = {"ancestors": torch.as_tensor(c["anc"], device=device).clone()}
        opt = Adam(params, 1e-3)
        g = torch.empty_like(params["ancestors"])
        mu, nu = torch.zeros_like(g), torch.zeros_like(g)

        def step(k):
            fn.value_and_grad(params["ancestors"], S0, out=g)
            if mode == "host":  # the pre-v7 host-count update
                check(lib().trex_adam_step(ptr(params["ancestors"]), ptr(g), ptr(mu), ptr(nu),
                                           g.numel(), k, 1e-3, 0.9, 0.999, 1e-8, None, 0, 0.0,
                                           stream_handle(device)))
            else:
                opt.step(params, {"ancestors": g})

        if mode == "graph":
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                step(0)
            for _ in range(6):
                graph.replay()
        else:
            for k in range(1, 7):
                step(k)
        torch.cuda.synchronize()
        runs.append((float(fn.loss[0]), params["ancestors"].clone()))
    assert runs[1][0] == runs[0][0] and torch.equal(runs[1][1], runs[0][1])
    assert runs[2][0] == runs[0][0] and torch.equal(runs[2][1], runs[0][1])


@pytest.mark.parametrize("capture", [False, True])
def test_nk_fused_adam_is_bitwise_the_unfused_loop(device, capture):
    """LandscapeAwareAdam (update_seq VJP + Adam + next update_seq in one
    pass, trex_adam_seq_update_step_dev) == value_and_grad + Adam.step,
    bitwise, over 6 steps at the eval shape -- eager and as hipGraph replays
    of one captured step."""
    from trex_amd.tree import Adam

    c = _case(32, 15, 2, 10, seed=7)
    land = NK.NKLandscape(c["inter"], c["F"], 2, device)
    S0 = torch.as_tensor(c["S0"], device=device)
    fn = NK.LandscapeAwareLoss(c["A"], c["n_leaves"], land, 3.0, 10)
    params = {"ancestors": torch.as_tensor(c["anc"], device=device).clone()}
    opt = Adam(params, 1e-3)
    ref_losses = []
    for _ in range(6):
        loss, g = fn.value_and_grad(params["ancestors"], S0)
        ref_losses.append(float(loss[0]))
        opt.step(params, {"ancestors": g})
    fn2 = NK.LandscapeAwareLoss(c["A"], c["n_leaves"], land, 3.0, 10)
    fused = NK.LandscapeAwareAdam(fn2, c["anc"], S0, 1e-3)
    losses = []
    if capture:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fused.step()
        for _ in range(6):
            graph.replay()
            losses.append(float(fn2.loss[0]))
    else:
        for _ in range(6):
            losses.append(float(fused.step()[0]))
    assert losses == ref_losses
    assert torch.equal(fused.ancestors, params["ancestors"])
    assert torch.equal(fused.mu, opt.mu["ancestors"]) and torch.equal(fused.nu, opt.nu["ancestors"])


@pytest.mark.parametrize("Q,k", [(4, 1), (4, 2), (4, 3), (4, 4), (2, 3), (2, 6)])
def test_register_kernels_bitwise_the_rolled_kernels(device, monkeypatch, Q, k):
    """The register kernels (Q, k compile-time, csrc/nk.hip nk_logits_reg_kernel
    / nk_logits_bwd_reg_kernel; the DNA shape's path) == the rolled
    wave-per-64-parents kernels (TREX_NK_REG=0) bit for bit: logits, and the
    loss + gradient through the reverse sweep.  127 parents (a partial last
    lane group) x 2 100 sites keeps the rolled kernels at one wave per
    (parent group, site), the arithmetic order the register kernels follow."""
    c = _case(128, 2100, Q, k, seed=Q * 10 + k, mask=True)
    land = NK.NKLandscape(c["inter"], c["F"], Q, device)
    a = torch.as_tensor(c["anc"], device=device)
    s = torch.as_tensor(c["S0"], device=device)
    par = torch.as_tensor(c["S0"][:127] + 0.1, device=device)
    par = par / par.sum(-1, keepdim=True)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TREX_NK_REG", flag)
        lg = NK.compute_parental_logits(par, land, k).clone()
        fn = NK.LandscapeAwareLoss(c["A"], 128, land, 0.7, k, seq_mask=c["mask"])
        loss, g = fn.value_and_grad(a, s)
        torch.cuda.synchronize()
        runs.append((lg, loss.clone(), g.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    assert torch.equal(runs[0][1], runs[1][1]) and torch.equal(runs[0][2], runs[1][2])
    ref = nk.compute_parental_logits(_n(par)[:, :64], c["inter"][:64] % 64,
                                     c["F"][:64].astype(np.float64), k)
    got = _n(NK.compute_parental_logits(par[:, :64].contiguous(),
                                        NK.NKLandscape(c["inter"][:64] % 64, c["F"][:64], Q,
                                                       device), k))
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=1e-6)


@pytest.mark.parametrize("k,mask,L", [(1, False, 300), (2, True, 300), (4, True, 300),
                                      (4, True, 3000)])
def test_q4_vector_kernels_bitwise_the_generic_kernels(device, monkeypatch, k, mask, L):
    """Q = 4's float4 cross-entropy / combine kernels (csrc/nk.hip nk_ce4_kernel;
    nk_combine4_lds_kernel when a parent's G block fits the LDS, L = 300,
    else nk_combine4_kernel, L = 3000 at k = 4) == the generic per-state
    kernels (TREX_NK_V4=0) bit for bit: loss and d ancestors, with and
    without the site mask."""
    c = _case(64, L, 4, k, seed=40 + k, mask=mask)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    a = torch.as_tensor(c["anc"], device=device)
    s = torch.as_tensor(c["S0"], device=device)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TREX_NK_V4", flag)
        fn = NK.LandscapeAwareLoss(c["A"], 64, land, 0.7, k, seq_mask=c["mask"] if mask else None)
        loss, g = fn.value_and_grad(a, s)
        torch.cuda.synchronize()
        runs.append((loss.clone(), g.clone()))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])


@pytest.mark.parametrize("mode", ["split_x3", "split_f32", "whole"])
def test_landscape_loss_surrogate_paths_vs_oracle(device, monkeypatch, mode):
    """The NK loss's surrogate as the C5 step runs it (leaf x leaf Gram block
    cached, d surrogate / dS for the ancestor rows only; f16x3 split GEMMs
    when K % 16 == 0, f32 with TREX_NK_X3=0) and trex_tree_surrogate's
    all-rows path (TREX_NK_SPLIT=0), each vs the fp64 oracle at a DNA-like
    shape: loss at rtol 1e-5, d ancestors per entry (landscape_grad_bound)."""
    monkeypatch.setenv("TREX_NK_SPLIT", "0" if mode == "whole" else "1")
    monkeypatch.setenv("TREX_NK_X3", "0" if mode == "split_f32" else "1")
    c = _case(128, 200, 4, 4, seed=17, mask=True)
    land = NK.NKLandscape(c["inter"], c["F"], 4, device)
    fn = NK.LandscapeAwareLoss(c["A"], 128, land, 0.9, 4, seq_mask=c["mask"])
    assert fn.split == (mode != "whole") and (mode == "whole" or fn.x3 == (mode == "split_x3"))
    s = torch.as_tensor(c["S0"], device=device)
    for step in range(2):  # the second call reuses the cached leaf x leaf block
        anc = c["anc"] * (1.0 + 0.1 * step)
        loss, g = fn.value_and_grad(torch.as_tensor(anc, device=device), s)
        args = (anc.astype(np.float64), c["S0"].astype(np.float64), 128, c["inter"],
                c["F"].astype(np.float64), c["A"], 0.9, 4, 1.0, c["mask"])
        rl, rg = nk.landscape_loss_grad(*args)
        np.testing.assert_allclose(float(loss[0]), rl, rtol=RTOL)
        assert_bound_close(_n(g), rg, landscape_grad_bound(*args, rtol=RTOL),
                           what=f"{mode} step {step}")
