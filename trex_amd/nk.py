"""trex's NK landscape-aware objective on MI355X.

Mirrors maraxen/trex ``src/trex/evals/benchmark.py``:
* ``compute_parental_logits`` (:586-663) -- expected site fitness per state
  under the parent's soft sequence (``trex_nk_parental_logits``);
* ``_update_seq_stacked`` (:210-232) and
  ``_compute_loss_landscape_aware_stacked`` (:235-306) -- surrogate cost +
  lambda * masked cross-entropy of every node against its parent's logits,
  as ``landscape_aware_loss`` / ``LandscapeAwareLoss.value_and_grad``;
* ``run_trex_landscape_aware_configurable`` (:326-460) with
  ``optimizer_name="adam"`` -- ``run_trex_landscape_aware_configurable``.

Interface changes, as in ``trex_amd.tree``: the reference's JAX PRNG draws
(initial ancestor logits ``jax.random.normal``, :391) are explicit inputs
(``init_ancestors``); the landscape is a pair of arrays (interactions
``(L, k)`` int, fitness tables ``(L, Q**(k+1))``), as
``create_nk_model_landscape`` returns them (nk_model.py:31-43).  All
arithmetic runs in libtrexhip.so; the parent map (argmax of the adjacency
rows, :286) and the inverse-interaction lists are built once on the host.
"""

from __future__ import annotations

import os

import numpy as np

from ._lib import check, lib, ptr, stream_handle


def _torch():
    import torch

    return torch


def _f32(x, device):
    torch = _torch()
    return torch.as_tensor(x).to(device=device, dtype=torch.float32).contiguous()


def _i32(x, device):
    torch = _torch()
    return torch.as_tensor(np.ascontiguousarray(np.asarray(x, dtype=np.int32))).to(device)


def _host(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


class NKLandscape:
    """Device copy of an NK landscape (interactions int32 (L, k), fitness
    fp32 (L, Q**(k+1)))."""

    def __init__(self, interactions, fitness_tables, n_states: int, device=None):
        torch = _torch()
        device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        inter = _host(interactions).astype(np.int32)
        if inter.ndim != 2:
            raise ValueError("interactions must be (L, k)")
        self.L, self.k = inter.shape
        self.Q = int(n_states)
        F = _host(fitness_tables).astype(np.float32)
        if F.shape != (self.L, self.Q ** (self.k + 1)):
            raise ValueError(f"fitness_tables must be (L, Q**(k+1)) = "
                             f"{(self.L, self.Q ** (self.k + 1))}, got {F.shape}")
        self.interactions_host = inter
        self.device = device
        self.interactions = _i32(inter, device)
        self.fitness = _f32(F, device)

    @classmethod
    def from_dict(cls, landscape: dict, device=None):
        """The reference's landscape PyTree (nk_model.py:38-43)."""
        return cls(landscape["interactions"], landscape["fitness_tables"],
                   int(landscape["n_states"]), device)


def compute_parental_logits(parent_sequences, landscape: NKLandscape, real_k: int,
                            batch_size: int = 64):
    """(n_parents, L, Q) logits (benchmark.py:586-663).  ``batch_size`` is the
    reference's safe_map chunking and has no effect here."""
    torch = _torch()
    del batch_size
    P = _f32(parent_sequences, landscape.device)
    n_p, L, Q = P.shape
    if L != landscape.L or Q != landscape.Q:
        raise ValueError("parent_sequences must be (n_parents, L, Q) of the landscape")
    rows = torch.arange(n_p, dtype=torch.int32, device=P.device)
    out = torch.empty((n_p, L, Q), dtype=torch.float32, device=P.device)
    k = 0 if real_k == 0 else landscape.k
    if real_k == 0 and landscape.fitness.shape[1] != Q:
        raise ValueError("real_k == 0 needs (L, Q) fitness tables (benchmark.py:616-620)")
    check(lib().trex_nk_parental_logits(ptr(P), ptr(rows), n_p, L, Q,
                                        ptr(landscape.interactions), k, ptr(landscape.fitness),
                                        ptr(out), stream_handle(P.device)))
    return out


class LandscapeAwareLoss:
    """Device-resident ``_compute_loss_landscape_aware_stacked`` and its
    gradient w.r.t. the stacked ancestor logits (benchmark.py:235-306).

    The adjacency, landscape, lambda and mask are fixed per instance (the
    reference's jit statics / closure, :404-418); buffers are allocated once.
    """

    def __init__(self, adj_matrix, n_leaves: int, landscape: NKLandscape, lambda_val: float,
                 real_k: int, *, temperature: float = 1.0, seq_mask=None):
        torch = _torch()
        dev = landscape.device
        A = _host(adj_matrix).astype(np.float64)
        self.N = A.shape[0]
        self.n_leaves = int(n_leaves)
        self.landscape = landscape
        self.lam = float(lambda_val)
        self.real_k = int(real_k)
        self.T = float(temperature)
        self.L, self.Q = landscape.L, landscape.Q
        self.A = _f32(A, dev)
        self.fitness_on = self.lam > 0.0 and self.real_k > 0
        if seq_mask is None:
            self.mask = None
            self.n_valid = float(self.L)
        else:
            m = _host(seq_mask).astype(np.float32)
            self.mask = _f32(m, dev)
            self.n_valid = float(m.sum())
        parent = np.argmax(A, axis=1).astype(np.int32)  # first index of the max (:286)
        L_ = lib()
        k = landscape.k
        nints = int(L_.trex_nk_plan_ints(self.N, self.L, k))
        plan = np.zeros(nints, np.int32)
        info = np.zeros(2, np.int32)
        check(L_.trex_nk_plan_build(ptr(parent), self.N, ptr(landscape.interactions_host),
                                    self.L, k, ptr(plan), ptr(info)))
        self.parent = parent
        self.n_parents, self.n_nonroot = int(info[0]), int(info[1])
        self.plan = torch.as_tensor(plan).to(dev)
        f32 = dict(dtype=torch.float32, device=dev)
        self.S = torch.empty((self.N, self.L, self.Q), **f32)
        self._s_src, self._s_ver = None, None
        self.dS = torch.empty_like(self.S)
        self.dS_sur = torch.empty_like(self.S)
        self.loss = torch.zeros((1,), **f32)
        self.sur = torch.zeros((1,), **f32)
        self.dA = torch.empty((self.N, self.N), **f32)
        K = self.L * self.Q
        self.tree_ws = torch.empty(int(L_.trex_tree_workspace_bytes(self.N, K)),
                                   dtype=torch.uint8, device=dev)
        nb = int(L_.trex_nk_workspace_bytes(self.N, self.L, self.Q, k, self.n_parents))
        self.nk_ws = torch.empty(max(nb, 256), dtype=torch.uint8, device=dev)
        # the surrogate as the C5 step runs it (TreeOptimizer): the leaf x leaf
        # block of the Gram is data (computed when the leaves change, skipped
        # per call), and d surrogate / dS only for the ancestor rows (the
        # leaf rows of dS are never used: leaves are fixed data) -- f16x3
        # split-product MFMA GEMMs when K % 16 == 0 (|S| <= 1, |M| <= m_bound:
        # their contract), f32 MFMA otherwise.  Small problems keep
        # trex_tree_surrogate's one-launch kernel (N <= 64, N K <= 4096).
        self.split = not (self.N <= 64 and self.N * K <= 4096) and \
            os.environ.get("TREX_NK_SPLIT", "1") != "0"
        if self.split:
            self.x3 = K % 16 == 0 and os.environ.get("TREX_NK_X3", "1") != "0"
            # the x3 GEMMs' contract is |S| <= 1: the ancestor rows are
            # softmaxes, the leaf rows are the caller's masked_sequences and
            # are checked whenever they change (_set_leaves)
            self.x3_allowed = self.x3
            self.G = torch.empty((self.N, self.N), **f32)
            self.M = torch.empty((self.N, self.N), **f32)
            self.m_bound = float(np.abs(A).sum(0).max() + np.abs(A).sum(1).max()
                                 + 2.0 * np.abs(A).max()) + 1.0
            self.dS_sur[: self.n_leaves].zero_()  # never written: the leaf rows' dS is unused

    def value_and_grad(self, ancestors, masked_sequences, *, want_grad: bool = True, out=None,
                       refresh: bool = False):
        """(loss (1,) device tensor, d loss / d ancestors (n_anc, L, Q)).
        ``out``: a preallocated (n_anc, L, Q) gradient buffer (no allocation:
        the call launches only kernels and is hipGraph-capturable).
        ``masked_sequences`` is copied only when it is another tensor than
        last call's or torch's version counter moved; a write through a raw
        pointer (a trex_* kernel, DLPack) is invisible to that counter, so
        pass ``refresh=True`` after one."""
        torch = _torch()
        L_ = lib()
        dev = self.S.device
        st = stream_handle(dev)
        anc = _f32(ancestors, dev)
        n_anc = self.N - self.n_leaves
        if tuple(anc.shape) != (n_anc, self.L, self.Q):
            raise ValueError(f"ancestors must be {(n_anc, self.L, self.Q)}")
        self._set_leaves(masked_sequences, refresh)
        check(L_.trex_tree_update_seq(ptr(anc), n_anc, self.L, self.Q, self.T,
                                      ptr(self.S[self.n_leaves:]), st))
        dS = self._loss_and_dS(want_grad)
        if not want_grad:
            return self.loss, None
        d_anc = torch.empty_like(anc) if out is None else out
        check(L_.trex_tree_update_seq_bwd(ptr(self.S[self.n_leaves:]), ptr(dS[self.n_leaves:]),
                                          n_anc, self.L, self.Q, self.T, ptr(d_anc), st))
        return self.loss, d_anc

    def _set_leaves(self, masked_sequences, refresh=False):
        # S = masked_sequences with the ancestor rows rewritten: the copy is
        # needed only when the caller passes another tensor or wrote into
        # this one (torch's version counter); the cached reference keeps the
        # tensor alive, so its storage cannot be reused under the cache
        ms = _f32(masked_sequences, self.S.device)
        ver = getattr(ms, "_version", None)
        if refresh or ms is not self._s_src or ver is None or ver != self._s_ver:
            self.S.copy_(ms)
            self._s_src, self._s_ver = ms, ver
            if self.split and self.x3_allowed:
                # one-hot / softmax leaves (|S| <= 1) keep the f16x3 GEMMs;
                # anything larger would overflow their f16 pieces, so those
                # leaves (and leaves copied while a hipGraph is being
                # captured, where the check cannot sync) take the f32 GEMMs
                torch = _torch()
                if torch.cuda.is_current_stream_capturing():
                    self.x3 = False
                else:
                    self.x3 = bool(self.S[: self.n_leaves].abs().max().item() <= 1.0)
            if self.split:  # the leaf x leaf Gram block of these leaves
                check(lib().trex_tree_gram(ptr(self.S), self.N, self.L * self.Q, ptr(self.G),
                                           ptr(self.tree_ws), self.tree_ws.numel(),
                                           stream_handle(self.S.device)))

    def _loss_and_dS(self, want_grad: bool):
        """Loss and d loss / d S (all rows) of the current S."""
        L_ = lib()
        st = stream_handle(self.S.device)
        K = self.L * self.Q
        N, nl = self.N, self.n_leaves
        if self.split:
            ws, wsb = ptr(self.tree_ws), self.tree_ws.numel()
            if self.x3:
                check(L_.trex_tree_gram_skip_x3(ptr(self.S), N, K, nl, 1.0, ptr(self.G), ws, wsb,
                                                st))
            else:
                check(L_.trex_tree_gram_skip(ptr(self.S), N, K, nl, ptr(self.G), ws, wsb, st))
            check(L_.trex_tree_surrogate_combine(ptr(self.A), ptr(self.G), N, ptr(self.sur),
                                                 ptr(self.dA), ptr(self.M), ws, st))
            if want_grad:
                dS = ptr(self.dS_sur[nl:])
                if self.x3:
                    check(L_.trex_tree_mf_rows_x3(ptr(self.M), ptr(self.S), N, K, nl, N - nl,
                                                  self.m_bound, 1.0, dS, st))
                else:
                    check(L_.trex_tree_mf_rows(ptr(self.M), ptr(self.S), N, K, nl, N - nl, dS,
                                               st))
        else:
            check(L_.trex_tree_surrogate(ptr(self.S), ptr(self.A), N, K, ptr(self.sur),
                                         ptr(self.dS_sur) if want_grad else None,
                                         ptr(self.dA) if want_grad else None, None,
                                         ptr(self.tree_ws), self.tree_ws.numel(), st))
        if self.fitness_on:
            check(L_.trex_nk_landscape_loss(
                ptr(self.plan), self.n_parents, ptr(self.S), self.N, self.L, self.Q,
                ptr(self.landscape.interactions), self.landscape.k, ptr(self.landscape.fitness),
                ptr(self.mask), self.n_valid, self.lam, self.n_nonroot, ptr(self.sur),
                ptr(self.dS_sur) if want_grad else None, ptr(self.loss),
                ptr(self.dS) if want_grad else None, ptr(self.nk_ws), self.nk_ws.numel(), st))
            return self.dS
        self.loss.copy_(self.sur)
        return self.dS_sur


class LandscapeAwareAdam:
    """optax.adam on the ancestor logits of a LandscapeAwareLoss, one fused
    step: the loss and dS of the current S, then the update_seq VJP, the Adam
    update and the next step's update_seq in one pass over the logits
    (trex_adam_seq_update_step_dev) -- bitwise the loop
    ``loss, g = fn.value_and_grad(anc, S0); Adam.step(...)`` of
    run_trex_landscape_aware_configurable (benchmark.py:326-460), two
    launches fewer per step.  The step count lives on the device, so a
    captured step replays (``step()`` launches only kernels)."""

    def __init__(self, fn: LandscapeAwareLoss, ancestors, masked_sequences, lr: float = 1e-3,
                 b1: float = 0.9, b2: float = 0.999, eps: float = 1e-8):
        torch = _torch()
        from .tree import step_state

        self.fn = fn
        dev = fn.S.device
        self.ancestors = _f32(ancestors, dev).clone()
        n_anc = fn.N - fn.n_leaves
        if tuple(self.ancestors.shape) != (n_anc, fn.L, fn.Q):
            raise ValueError(f"ancestors must be {(n_anc, fn.L, fn.Q)}")
        self.lr, self.b1, self.b2, self.eps = float(lr), float(b1), float(b2), float(eps)
        self.mu = torch.zeros_like(self.ancestors)
        self.nu = torch.zeros_like(self.ancestors)
        self.count = 0
        # device step record: count / bias corrections advance per step, the
        # update_seq temperature (fixed for this loss) in T and T_next
        self.state = step_state(dev)
        tbits = int(np.array([fn.T], dtype=np.float32).view(np.int32)[0])
        self.state[3] = tbits
        self.state[4] = tbits
        fn._set_leaves(masked_sequences)
        check(lib().trex_tree_update_seq(ptr(self.ancestors), n_anc, fn.L, fn.Q, fn.T,
                                         ptr(fn.S[fn.n_leaves:]), stream_handle(dev)))

    def step(self):
        """One step; returns the (device) loss before the update."""
        fn = self.fn
        L_ = lib()
        st = stream_handle(fn.S.device)
        dS = fn._loss_and_dS(True)
        self.count += 1
        check(L_.trex_step_advance(ptr(self.state), self.b1, self.b2, None, 0, st))
        check(L_.trex_adam_seq_update_step_dev(ptr(dS[fn.n_leaves:]), fn.N - fn.n_leaves, fn.L,
                                               fn.Q, ptr(self.state), ptr(self.ancestors),
                                               ptr(self.mu), ptr(self.nu), self.lr, self.b1,
                                               self.b2, self.eps, ptr(fn.S[fn.n_leaves:]), st))
        return fn.loss


def landscape_aware_loss(ancestors, masked_sequences, n_leaves: int, landscape: NKLandscape,
                         adj_matrix, n_all: int, lambda_val: float, real_k: int,
                         temperature: float = 1.0, seq_mask=None, batch_size: int = 64):
    """Functional ``_compute_loss_landscape_aware_stacked`` (benchmark.py:235-306)."""
    del batch_size
    if _host(adj_matrix).shape[0] != n_all:
        raise ValueError("adj_matrix must be (n_all, n_all)")
    fn = LandscapeAwareLoss(adj_matrix, n_leaves, landscape, lambda_val, real_k,
                            temperature=temperature, seq_mask=seq_mask)
    loss, _ = fn.value_and_grad(ancestors, masked_sequences, want_grad=False)
    return loss[0]


def masked_sequences_from_leaves(leaf_sequences, n_all: int, n_states: int, device=None):
    """one_hot(leaves) stacked over zero ancestor rows (benchmark.py:398-408)."""
    torch = _torch()
    leaves = torch.as_tensor(_host(leaf_sequences).astype(np.int64))
    n_leaves, L = leaves.shape
    S = torch.zeros((n_all, L, n_states), dtype=torch.float32)
    S[:n_leaves].scatter_(2, leaves[..., None], 1.0)
    return S.to(device) if device is not None else S


def run_trex_landscape_aware_configurable(leaf_sequences, n_all: int, n_leaves: int,
                                          n_states: int, landscape: NKLandscape,
                                          lambda_val: float, adj_matrix, init_ancestors,
                                          real_k: int = 0, learning_rate: float = 1e-3,
                                          n_iterations: int = 10000, return_losses: bool = False,
                                          seq_mask=None):
    """Adam on the stacked ancestor logits (benchmark.py:326-460,
    optimizer_name="adam"); ``init_ancestors`` replaces the JAX normal draw
    (:391).  Returns argmax ancestors (n_anc, L) [, per-step losses]."""
    torch = _torch()
    dev = landscape.device
    S0 = masked_sequences_from_leaves(leaf_sequences, n_all, n_states, dev)
    fn = LandscapeAwareLoss(adj_matrix, n_leaves, landscape, lambda_val, real_k,
                            seq_mask=seq_mask)
    opt = LandscapeAwareAdam(fn, init_ancestors, S0, learning_rate)
    losses = torch.empty((n_iterations,), dtype=torch.float32, device=dev) if return_losses \
        else None
    for it in range(n_iterations):
        loss = opt.step()
        if losses is not None:
            losses[it:it + 1].copy_(loss)
    out = torch.argmax(opt.ancestors, dim=-1)
    return (out, losses) if return_losses else out
