"""Evaluation drivers (src/trex/evals/benchmark.py:41-200, 459-540) on device
vs the fp64 oracle loop: create_optimizer's four optimisers after
clip_by_global_norm(1.0), fixed tree, ancestors only.

Checked step by step at the GPU's own parameters before each step: loss at
rtol 1e-5, the gradient per entry (1e-5 of its terms' magnitudes through
update_seq's softmax VJP: tests/_cases.py), and the parameters after the
step == the fp64 optax update (oracle/tree_ref.py optax_update) of the GPU's
own gradient from the GPU's optimiser state, to fp32 rounding -- not two
6-step trajectories, which legitimately drift apart where a gradient entry
sits within its fp32 error of 0 (Adam's first step is lr * sign(g)).  The
optax boundary itself is "parity unpinned": no reference test checks
optimiser arithmetic."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import assert_bound_close, softmax_vjp_bound, surrogate_grad_bounds
from oracle import tree_ref as T
from trex_amd import evals as E
from trex_amd.topology import create_balanced_binary_tree

pytestmark = pytest.mark.gpu


def _case(nl, L, Q, seed):
    rng = np.random.default_rng(seed)
    n = 2 * nl - 1
    leaves = rng.integers(0, Q, size=(nl, L))
    S0 = np.zeros((n, L, Q), np.float32)
    S0[np.arange(nl)[:, None], np.arange(L)[None, :], leaves] = 1.0
    anc = rng.normal(size=(nl - 1, L, Q)).astype(np.float32)
    return leaves, S0, anc, create_balanced_binary_tree(nl)


@pytest.mark.parametrize("name", ["adam", "adamw", "sgd", "rmsprop"])
@pytest.mark.parametrize("L", [13, 64])  # K = 52 (f32 GEMMs) / 256 (f16x3 split GEMMs)
def test_ancestor_optimizer_matches_oracle_loop(device, name, L):
    nl, Q, lr = 8, 4, 0.05
    leaves, S0, anc, A = _case(nl, L, Q, seed=L)
    opt = E.AncestorOptimizer(S0, nl, A, anc, name, lr, device=device)

    def f64(t):
        return t.detach().cpu().numpy().astype(np.float64)

    for step in range(1, 7):
        p = f64(opt.params["ancestors"])
        st = {"count": opt.opt.count, "s1": {"ancestors": f64(opt.opt.s1["ancestors"])},
              "s2": {"ancestors": f64(opt.opt.s2["ancestors"])}}
        loss = float(opt.step())
        torch.cuda.synchronize()
        g = f64(opt.grads["ancestors"])
        rl, rg = T.fixed_tree_loss_grad(p, S0, nl, A)
        np.testing.assert_allclose(loss, rl, rtol=1e-5)
        # gradient bound: dS's terms at 1e-5 through the softmax VJP
        S = np.array(S0, dtype=np.float64)
        P = np.exp(p - p.max(-1, keepdims=True))
        P /= P.sum(-1, keepdims=True)
        S[nl:] = P
        bS, _ = surrogate_grad_bounds(S, A, 1e-5)
        assert_bound_close(g, rg, softmax_vjp_bound(P, bS[nl:]), what=f"grad step {step}")
        # the optimiser: fp64 optax of the GPU's own gradient and state
        upd, _ = T.optax_update(name, {"ancestors": g}, st, {"ancestors": p}, lr, clip_norm=1.0)
        want = p + upd["ancestors"]
        got = f64(opt.params["ancestors"])
        slack = 4.8e-7 * np.abs(want) + 1e-5 * lr
        err = np.abs(got - want)
        assert np.all(err <= slack), (step, float((err - slack).max()))


def test_optimizer_without_clipping_and_unknown_name(device):
    params = {"x": torch.ones(10, device=device)}
    opt = E.create_optimizer("sgd", 0.1, params, use_gradient_clipping=False)
    g = {"x": torch.full((10,), 5.0, device=device)}
    opt.step(params, g)
    opt.step(params, g)
    # trace t1 = 5, t2 = 5 + 0.9 * 5; p = 1 - 0.1 (5 + 9.5)
    np.testing.assert_allclose(params["x"].cpu().numpy(), 1 - 0.1 * 14.5, rtol=1e-6)
    with pytest.raises(ValueError):
        E.create_optimizer("lion", 0.1, params)


def test_run_trex_optimization_batched_returns_argmax(device):
    nl, L, Q = 4, 16, 4
    leaves, S0, anc, A = _case(nl, L, Q, seed=3)
    out, losses = E.run_trex_optimization_configurable(leaves, 2 * nl - 1, nl, Q, A, anc,
                                                       n_iterations=30, return_losses=True,
                                                       learning_rate=0.05, device=device)
    assert out.shape == (nl - 1, L) and losses.shape == (30,)
    lo = losses.cpu().numpy()
    assert lo[-1] < lo[0]  # the surrogate decreases under Adam
    out2 = E.run_trex_optimization_batched(leaves, 2 * nl - 1, nl, Q, A, anc, n_iterations=3,
                                           device=device)
    assert out2.shape == (nl - 1, L)
