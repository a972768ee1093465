"""trex's evaluation-side optimisation drivers on MI355X.

Mirrors maraxen/trex ``src/trex/evals/benchmark.py``:
* ``create_optimizer`` (:41-72): optax adam / adamw / sgd(momentum 0.9) /
  rmsprop, chained after ``clip_by_global_norm(1.0)`` by default -- one
  ``trex_optax_step`` launch per parameter tensor, clipping from a device
  squared-norm reduction (no host sync);
* ``run_trex_optimization_configurable`` (:75-200) and
  ``run_trex_optimization_batched`` (:459-540): a fixed tree, the stacked
  ancestor logits optimised on the surrogate cost (or ``compute_soft_cost``
  with C = I, which is the same quadratic form, tree.py:212-266), the whole
  loop body on device (update_seq -> Gram -> combine -> ancestor-rows dS ->
  update_seq VJP -> optimiser), the leaf x leaf Gram computed once.

As elsewhere in ``trex_amd``, the JAX PRNG draw of the initial logits
(:127, ``jax.random.normal``) is an explicit input (``init_ancestors``).
"""

from __future__ import annotations

import numpy as np

from ._lib import check, lib, ptr, stream_handle

_KINDS = {"adam": 0, "adamw": 1, "sgd": 2, "rmsprop": 3}


def _torch():
    import torch

    return torch


class Optimizer:
    """``create_optimizer(name, lr)`` on device (optax 0.2.6 defaults)."""

    def __init__(self, name: str, learning_rate: float, params: dict, *,
                 use_gradient_clipping: bool = True):
        torch = _torch()
        if name not in _KINDS:
            raise ValueError(f"Unknown optimizer: {name}. Choose from {list(_KINDS)}")
        self.name, self.kind, self.lr = name, _KINDS[name], float(learning_rate)
        self.clip = 1.0 if use_gradient_clipping else None
        # (b1, b2, eps, weight_decay): sgd uses b1 as the momentum, rmsprop b2 as the decay
        self.b1, self.b2, self.eps, self.wd = {
            "adam": (0.9, 0.999, 1e-8, 0.0), "adamw": (0.9, 0.999, 1e-8, 0.01),
            "sgd": (0.9, 0.0, 0.0, 0.0), "rmsprop": (0.0, 0.9, 1e-8, 0.0)}[name]
        self.s1 = {k: torch.zeros_like(v) for k, v in params.items()}
        self.s2 = {k: torch.zeros_like(v) for k, v in params.items()}
        self.count = 0
        dev = next(iter(params.values())).device
        self.parts = torch.zeros(512 * max(1, len(params)), dtype=torch.float64, device=dev)
        # device step count + bias corrections (graph-capturable steps)
        from .tree import step_state

        self.state = step_state(dev)

    def step(self, params: dict, grads: dict):
        self.count += 1
        st = stream_handle(next(iter(params.values())).device)
        check(lib().trex_step_advance(ptr(self.state), self.b1, self.b2, None, 0, st))
        keys = sorted(params)
        nparts = 0
        if self.clip is not None:
            for i, k in enumerate(keys):
                check(lib().trex_sq_norm_parts(ptr(grads[k]), grads[k].numel(),
                                               ptr(self.parts[512 * i:]), 512, st))
            nparts = 512 * len(keys)
        for k in keys:
            check(lib().trex_optax_step_dev(
                self.kind, ptr(params[k]), ptr(grads[k]), ptr(self.s1[k]), ptr(self.s2[k]),
                params[k].numel(), ptr(self.state), self.lr, self.b1, self.b2, self.eps, self.wd,
                ptr(self.parts) if nparts else None, nparts, float(self.clip or 0.0), st))


def create_optimizer(name: str, learning_rate: float, params: dict, *,
                     use_gradient_clipping: bool = True) -> Optimizer:
    return Optimizer(name, learning_rate, params, use_gradient_clipping=use_gradient_clipping)


class AncestorOptimizer:
    """The loop body of run_trex_optimization_configurable on device: fixed
    adjacency, ancestors only, T = 1 (benchmark.py:151-200)."""

    def __init__(self, masked_sequences, n_leaves: int, adj_matrix, init_ancestors,
                 optimizer_name: str = "adam", learning_rate: float = 1e-3, *,
                 use_gradient_clipping: bool = True, device=None):
        torch = _torch()
        dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.S = torch.as_tensor(masked_sequences).to(device=dev, dtype=torch.float32).clone()
        self.N, self.L, self.Q = self.S.shape
        self.K = self.L * self.Q
        self.n_leaf = int(n_leaves)
        self.n_anc = self.N - self.n_leaf
        self.A = torch.as_tensor(np.asarray(adj_matrix, dtype=np.float32)).to(dev).contiguous()
        if tuple(self.A.shape) != (self.N, self.N):
            raise ValueError("adj_matrix must be (n_all, n_all)")
        self.params = {"ancestors": torch.as_tensor(init_ancestors).to(
            device=dev, dtype=torch.float32).clone().contiguous()}
        if tuple(self.params["ancestors"].shape) != (self.n_anc, self.L, self.Q):
            raise ValueError(f"init_ancestors must be {(self.n_anc, self.L, self.Q)}")
        self.grads = {"ancestors": torch.zeros_like(self.params["ancestors"])}
        self.opt = create_optimizer(optimizer_name, learning_rate, self.params,
                                    use_gradient_clipping=use_gradient_clipping)
        f32 = dict(dtype=torch.float32, device=dev)
        self.G = torch.empty((self.N, self.N), **f32)
        self.M = torch.empty((self.N, self.N), **f32)
        self.dA = torch.empty((self.N, self.N), **f32)
        self.dS = torch.empty((self.n_anc, self.L, self.Q), **f32)
        self.loss = torch.zeros((1,), **f32)
        self.ws = torch.empty(int(lib().trex_tree_workspace_bytes(self.N, self.K)),
                              dtype=torch.uint8, device=dev)
        # f16x3 split GEMMs when the shapes allow (|S| <= 1; M has softmax-free
        # rows here, so its bound is the adjacency's row + column sums)
        self.x3 = self.K % 16 == 0
        A_host = np.asarray(adj_matrix, dtype=np.float64)
        self.m_bound = float(np.abs(A_host).sum(0).max() + np.abs(A_host).sum(1).max()
                             + 2.0 * np.abs(A_host).max()) + 1.0
        st = stream_handle(dev)
        # the leaf x leaf block of G is data: computed once, skipped per step
        check(lib().trex_tree_gram(ptr(self.S), self.N, self.K, ptr(self.G), ptr(self.ws),
                                   self.ws.numel(), st))

    def step(self):
        """One optimisation step; returns the (device) loss before the update."""
        L_ = lib()
        st = stream_handle(self.S.device)
        N, K = self.N, self.K
        anc = self.params["ancestors"]
        check(L_.trex_tree_update_seq(ptr(anc), self.n_anc, self.L, self.Q, 1.0,
                                      ptr(self.S[self.n_leaf:]), st))
        if self.x3:
            check(L_.trex_tree_gram_skip_x3(ptr(self.S), N, K, self.n_leaf, 1.0, ptr(self.G),
                                            ptr(self.ws), self.ws.numel(), st))
        else:
            check(L_.trex_tree_gram_skip(ptr(self.S), N, K, self.n_leaf, ptr(self.G),
                                         ptr(self.ws), self.ws.numel(), st))
        check(L_.trex_tree_surrogate_combine(ptr(self.A), ptr(self.G), N, ptr(self.loss),
                                             ptr(self.dA), ptr(self.M), ptr(self.ws), st))
        if self.x3:
            check(L_.trex_tree_mf_rows_x3(ptr(self.M), ptr(self.S), N, K, self.n_leaf,
                                          self.n_anc, self.m_bound, 1.0, ptr(self.dS), st))
        else:
            check(L_.trex_tree_mf_rows(ptr(self.M), ptr(self.S), N, K, self.n_leaf, self.n_anc,
                                       ptr(self.dS), st))
        check(L_.trex_tree_update_seq_bwd(ptr(self.S[self.n_leaf:]), ptr(self.dS), self.n_anc,
                                          self.L, self.Q, 1.0, ptr(self.grads["ancestors"]), st))
        self.opt.step(self.params, self.grads)
        return self.loss


def _masked_sequences(leaf_sequences, n_all, n_states):
    leaves = np.asarray(leaf_sequences).astype(np.int64)
    n_leaves, L = leaves.shape
    S = np.zeros((n_all, L, n_states), np.float32)
    S[np.arange(n_leaves)[:, None], np.arange(L)[None, :], leaves] = 1.0
    return S


def run_trex_optimization_configurable(leaf_sequences, n_all: int, n_leaves: int,
                                       n_states: int, adj_matrix, init_ancestors,
                                       use_soft_cost: bool = False, optimizer_name: str = "adam",
                                       learning_rate: float = 1e-3, n_iterations: int = 10000,
                                       return_losses: bool = False, device=None):
    """benchmark.py:75-200.  ``use_soft_cost`` selects compute_soft_cost with
    C = I, the same quadratic form as the surrogate (tree.py:212-266), so both
    run the surrogate kernels.  Returns argmax ancestors (n_anc, L)
    [, per-step losses (n_iterations,)]."""
    torch = _torch()
    del use_soft_cost
    opt = AncestorOptimizer(_masked_sequences(leaf_sequences, n_all, n_states), n_leaves,
                            adj_matrix, init_ancestors, optimizer_name, learning_rate,
                            device=device)
    losses = torch.empty((n_iterations,), dtype=torch.float32, device=opt.S.device) \
        if return_losses else None
    for it in range(n_iterations):
        loss = opt.step()
        if losses is not None:
            losses[it:it + 1].copy_(loss)
    out = torch.argmax(opt.params["ancestors"], dim=-1)
    return (out, losses) if return_losses else out


def run_trex_optimization_batched(leaf_sequences, n_all: int, n_leaves: int, n_states: int,
                                  adj_matrix, init_ancestors, use_soft_cost: bool = False,
                                  n_iterations: int = 10000, device=None):
    """benchmark.py:459-540: adam(1e-3) after clip_by_global_norm(1.0)."""
    return run_trex_optimization_configurable(leaf_sequences, n_all, n_leaves, n_states,
                                              adj_matrix, init_ancestors, use_soft_cost, "adam",
                                              1e-3, n_iterations, device=device)
