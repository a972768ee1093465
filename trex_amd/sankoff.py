"""trex's ``sankoff`` module on MI355X.

Mirrors maraxen/trex ``src/trex/sankoff.py``: ``run_sankoff`` (:114-188),
``run_dp`` (:24-94), ``vectorized_dp`` (:97) and ancestral reconstruction
(:166-185, 191-267), plus what trex's readme promises but its code lacks -- a
differentiable score: ``sankoff_value_and_grad`` returns d(total)/d(cost)
(the tie-averaged subgradient JAX would give for tau=0, the softmin adjoint
for tau>0; DESIGN.md "Softmin").

All arithmetic runs in libtrexhip.so (HIP, gfx950).  torch is used only for
device memory and streams.  There is no CPU fallback.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._lib import TREX_FLAG_HARD_ROOT, check, lib, ptr, stream_handle
from .topology import TreePlan

SENTINEL = 1e5  # src/trex/sankoff.py:152


def _torch():
    import torch

    return torch


def _default_device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("trex_amd needs a ROCm GPU (MI355X); no CPU fallback exists")
    return torch.device("cuda", torch.cuda.current_device())


def leaf_codes(sequences, n_states: int, device=None):
    """trex leaf states -> int8 codes on the device.

    ``seq.astype(int32)`` truncates toward zero, negative states wrap once,
    anything else out of range is a dropped scatter (all-1e5 row,
    sankoff.py:49-52); such leaves get code -1.
    """
    torch = _torch()
    device = device or _default_device()
    s = torch.as_tensor(sequences).to(device=device, dtype=torch.float64)
    s = torch.trunc(s)
    s = torch.where(s < 0, s + n_states, s)
    ok = (s >= 0) & (s < n_states)
    return torch.where(ok, s, torch.full_like(s, -1)).to(torch.int8).contiguous()


@dataclass
class ForwardResult:
    tree_score: "object"  # (B,) float32
    dp: "object"  # (B, n_int, L, Q) float32, site-major (trex's per-site rows)
    site_score: "object"  # (B, L) float32 or None


class SankoffEngine:
    """Batched Sankoff for a fixed (topology batch, L, Q): the hot path.

    leaves: int8 (B, n_leaves, L) codes on the device; cost: float32 (Q, Q).
    Everything is enqueued on torch's current stream; nothing synchronises.
    """

    def __init__(self, plan: TreePlan, n_sites: int, n_states: int, device=None):
        torch = _torch()
        self.plan = plan
        self.L = int(n_sites)
        self.Q = int(n_states)
        self.device = torch.device(device) if device is not None else _default_device()
        self.plan_dev = plan.device(self.device)
        nbytes = lib().trex_workspace_bytes(plan.B, self.L, plan.n_all, self.Q)
        if nbytes <= 0:
            raise ValueError("bad shape for workspace")
        self.workspace = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        # arrival counters of the in-kernel reductions start at zero
        check(lib().trex_workspace_init(ptr(self.workspace), nbytes, stream_handle(self.device)))

    # -- shapes ------------------------------------------------------------
    @property
    def site_major(self) -> bool:
        """DP / marginal tables are site-major (B, n_int, L, Q) for every Q
        (trex_dp_site_major, include/trex_hip.h)."""
        return bool(lib().trex_dp_site_major(self.Q))

    @property
    def dp_shape(self):
        if self.site_major:
            return (self.plan.B, self.plan.n_int, self.L, self.Q)
        return (self.plan.B, self.plan.n_int, self.Q, self.L)

    def state_rows(self, table):
        """(B, n_int, Q, L) view of a DP / marginal table (the oracle's
        node-state-site order)."""
        return table.transpose(2, 3) if self.site_major else table

    def _check_inputs(self, leaves, cost):
        torch = _torch()
        p = self.plan
        if leaves.dtype != torch.int8 or tuple(leaves.shape) != (p.B, p.n_leaves, self.L):
            raise ValueError(f"leaves must be int8 {(p.B, p.n_leaves, self.L)}, got "
                             f"{leaves.dtype} {tuple(leaves.shape)}")
        if cost.dtype != torch.float32 or tuple(cost.shape) != (self.Q, self.Q):
            raise ValueError(f"cost must be float32 ({self.Q}, {self.Q})")
        for t in (leaves, cost):
            if not t.is_contiguous() or t.device != self.device:
                raise ValueError("inputs must be contiguous tensors on the engine's device")

    # -- kernels -----------------------------------------------------------
    def forward(self, leaves, cost, tau: float = 0.0, *, dp=True, site_score=False,
                hard_root=False, out=None) -> ForwardResult:
        """Post-order DP (sankoff.py:24-97) + per-tree total (sankoff.py:187)."""
        torch = _torch()
        self._check_inputs(leaves, cost)
        p = self.plan
        o = out or {}
        if dp is True:
            dp_t = o.get("dp")
            if dp_t is None:
                dp_t = torch.empty(self.dp_shape, dtype=torch.float32, device=self.device)
        elif dp is not False and dp is not None:
            dp_t = dp
        else:
            raise ValueError("forward writes the DP table (trex returns it); pass dp=True")
        ss = None
        if site_score:
            ss = o.get("site_score")
            if ss is None:
                ss = torch.empty((p.B, self.L), dtype=torch.float32, device=self.device)
        ts = o.get("tree_score")
        if ts is None:
            ts = torch.empty((p.B,), dtype=torch.float32, device=self.device)
        flags = TREX_FLAG_HARD_ROOT if hard_root else 0
        check(lib().trex_sankoff_fwd(
            ptr(self.plan_dev), p.n_slots, ptr(leaves), ptr(cost), p.B, self.L, p.n_all,
            self.Q, float(tau), flags, ptr(dp_t), ptr(ss), ptr(ts), ptr(self.workspace),
            self.workspace.numel(), stream_handle(self.device)))
        return ForwardResult(ts, dp_t, ss)

    def backward(self, leaves, cost, tau: float, dp, d_tree_score=None, *, marginals=False,
                 anc_states=False, hard_root=False, out=None):
        """Adjoint sweep: (d_cost, marginals | None, anc_states | None)."""
        torch = _torch()
        self._check_inputs(leaves, cost)
        p = self.plan
        if dp is None or tuple(dp.shape) != self.dp_shape:
            raise ValueError("backward needs the forward's dp table")
        o = out or {}
        dc = o.get("d_cost")
        if dc is None:
            dc = torch.empty((self.Q, self.Q), dtype=torch.float32, device=self.device)
        mg = None
        if marginals:
            mg = o.get("marginals")
            if mg is None:
                mg = torch.empty(self.dp_shape, dtype=torch.float32, device=self.device)
        an = None
        if anc_states:
            an = torch.empty((p.B, p.n_int, self.L), dtype=torch.int8, device=self.device)
        if d_tree_score is not None:
            d_tree_score = torch.as_tensor(d_tree_score, dtype=torch.float32,
                                           device=self.device).contiguous()
            if d_tree_score.shape != (p.B,):
                raise ValueError("d_tree_score must be (B,)")
        flags = TREX_FLAG_HARD_ROOT if hard_root else 0
        check(lib().trex_sankoff_bwd(
            ptr(self.plan_dev), p.n_slots, ptr(leaves), ptr(cost), p.B, self.L, p.n_all,
            self.Q, float(tau), flags, ptr(dp), ptr(d_tree_score), ptr(dc), ptr(mg), ptr(an),
            ptr(self.workspace), self.workspace.numel(), stream_handle(self.device)))
        return dc, mg, an

    def fwd_bwd(self, leaves, cost, tau: float = 0.0, d_tree_score=None, *, site_score=False,
                marginals=False, anc_states=False, hard_root=False, out=None):
        """Fused forward + adjoint in one launch (trex_sankoff_fwd_bwd).

        Returns (ForwardResult, d_cost, marginals | None, anc_states | None).
        """
        torch = _torch()
        self._check_inputs(leaves, cost)
        p = self.plan
        o = out or {}

        def buf(key, shape, dtype, want=True):
            if not want:
                return None
            t = o.get(key)
            if t is None:
                t = torch.empty(shape, dtype=dtype, device=self.device)
            return t

        dp_t = buf("dp", self.dp_shape, torch.float32)
        ss = buf("site_score", (p.B, self.L), torch.float32, site_score)
        ts = buf("tree_score", (p.B,), torch.float32)
        dc = buf("d_cost", (self.Q, self.Q), torch.float32)
        mg = buf("marginals", self.dp_shape, torch.float32, marginals)
        an = buf("anc_states", (p.B, p.n_int, self.L), torch.int8, anc_states)
        if d_tree_score is not None:
            d_tree_score = torch.as_tensor(d_tree_score, dtype=torch.float32,
                                           device=self.device).contiguous()
            if d_tree_score.shape != (p.B,):
                raise ValueError("d_tree_score must be (B,)")
        flags = TREX_FLAG_HARD_ROOT if hard_root else 0
        check(lib().trex_sankoff_fwd_bwd(
            ptr(self.plan_dev), p.n_slots, ptr(leaves), ptr(cost), p.B, self.L, p.n_all,
            self.Q, float(tau), flags, ptr(dp_t), ptr(ss), ptr(ts), ptr(d_tree_score), ptr(dc),
            ptr(mg), ptr(an), ptr(self.workspace), self.workspace.numel(),
            stream_handle(self.device)))
        return ForwardResult(ts, dp_t, ss), dc, mg, an

    def backtrack(self, cost, dp):
        """trex-exact ancestral states (B, n_int, L) int8 (sankoff.py:166-185)."""
        torch = _torch()
        p = self.plan
        an = torch.empty((p.B, p.n_int, self.L), dtype=torch.int8, device=self.device)
        check(lib().trex_sankoff_backtrack(
            ptr(self.plan_dev), p.backtrack_ok, ptr(cost), ptr(dp), p.B, self.L, p.n_all,
            self.Q, ptr(an), stream_handle(self.device)))
        return an

    def value_and_grad(self, leaves, cost, tau: float = 0.0, d_tree_score=None,
                       hard_root=False):
        """(tree_score (B,), d_cost (Q, Q)) -- fused fwd + adjoint launch."""
        f, dc, _, _ = self.fwd_bwd(leaves, cost, tau, d_tree_score, hard_root=hard_root)
        return f.tree_score, dc

    def to_trex_layout(self, dp, leaves):
        """engine dp table -> trex VmappedDPTable per tree: (B, L, n_all, Q)."""
        torch = _torch()
        p = self.plan
        out = torch.empty((p.B, self.L, p.n_all, self.Q), dtype=torch.float32,
                          device=self.device)
        check(lib().trex_dp_to_trex_layout(ptr(dp), ptr(leaves), p.B, self.L, p.n_all, self.Q,
                                           ptr(out), stream_handle(self.device)))
        return out


# ---------------------------------------------------------------------------
# trex module API
# ---------------------------------------------------------------------------
_PLANS: dict = {}
_ENGINES: dict = {}


def _plan_for(adjacency) -> TreePlan:
    a = np.ascontiguousarray(np.asarray(adjacency, dtype=np.float32))
    key = (a.shape, a.tobytes())
    plan = _PLANS.get(key)
    if plan is None:
        if len(_PLANS) > 256:
            _PLANS.clear()
        plan = TreePlan.from_adjacency(a)
        _PLANS[key] = plan
    return plan


def _engine_for(plan: TreePlan, L: int, Q: int, device) -> SankoffEngine:
    key = (id(plan), L, Q, str(device))
    eng = _ENGINES.get(key)
    if eng is None:
        if len(_ENGINES) > 64:
            _ENGINES.clear()
        eng = SankoffEngine(plan, L, Q, device)
        _ENGINES[key] = eng
    return eng


def _to_host(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def _prepare(adjacency_matrix, cost_matrix, sequences, n_all, n_states, n_leaves, device):
    torch = _torch()
    adj = _to_host(adjacency_matrix)
    if adj.shape != (n_all, n_all):
        raise ValueError(f"adjacency_matrix must be ({n_all}, {n_all}), got {adj.shape}")
    if n_leaves != (n_all + 1) // 2:
        raise NotImplementedError(
            "trex's DP initialises (n_all+1)//2 leaf rows (sankoff.py:46); n_leaves must match")
    device = device or _default_device()
    seqs = torch.as_tensor(sequences)
    if seqs.ndim != 2 or seqs.shape[0] < n_leaves:
        raise ValueError(f"sequences must be (>= {n_leaves}, L), got {tuple(seqs.shape)}")
    cost = torch.as_tensor(cost_matrix).to(device=device, dtype=torch.float32).contiguous()
    if tuple(cost.shape) != (n_states, n_states):
        raise ValueError(f"cost_matrix must be ({n_states}, {n_states})")
    plan = _plan_for(adj)
    L = int(seqs.shape[1])
    eng = _engine_for(plan, L, n_states, device)
    codes = leaf_codes(seqs[:n_leaves], n_states, device)[None].contiguous()
    return plan, eng, codes, cost, seqs


def run_sankoff(adjacency_matrix, cost_matrix, sequences, n_all: int, n_states: int,
                n_leaves: int, *, return_path: bool = False, device=None):
    """Sankoff over one tree (sankoff.py:114-188).

    Returns (reconstructed (n_all, L) f32, dp (L, n_all, Q) f32, total f32[]) as
    device tensors with trex's layouts and values.
    """
    torch = _torch()
    plan, eng, codes, cost, seqs = _prepare(adjacency_matrix, cost_matrix, sequences, n_all,
                                            n_states, n_leaves, device)
    f = eng.forward(codes, cost, 0.0, dp=True)
    dp_trex = eng.to_trex_layout(f.dp, codes)[0]
    L = eng.L
    recon = torch.zeros((n_all, L), dtype=torch.float32, device=eng.device)
    recon[:n_leaves] = seqs[:n_leaves].to(device=eng.device, dtype=torch.float32)
    if return_path:
        anc = eng.backtrack(cost, f.dp)[0]
        recon[n_leaves:] = anc.to(torch.float32)
    return recon, dp_trex, f.tree_score[0]


def sankoff_value_and_grad(adjacency_matrix, cost_matrix, sequences, n_all: int,
                           n_states: int, n_leaves: int, *, tau: float = 0.0,
                           hard_root: bool = False, device=None):
    """(total, d total / d cost_matrix) for one tree.

    tau = 0: exactly ``jax.value_and_grad(lambda C: run_sankoff(adj, C, ...)[2])``
    semantics (hard min, tie-averaged subgradient).  tau > 0: softmin score
     and its exact gradient.
    """
    _, eng, codes, cost, _ = _prepare(adjacency_matrix, cost_matrix, sequences, n_all,
                                      n_states, n_leaves, device)
    ts, dc = eng.value_and_grad(codes, cost, tau, hard_root=hard_root)
    return ts[0], dc
