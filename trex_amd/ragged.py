"""Ragged tree batches: mixed tree sizes and site counts in one launch.

trex serves mixed sizes from one jit by padding: every tree to
``MAX_NODES`` nodes, every alignment to an N bucket, with node / site masks
(``src/trex/padding.py:25-27`` buckets, ``:77-297`` pad / mask helpers,
``masked_mean`` / ``masked_sum``).  The HIP kernels take runtime shapes, so
the build maps that onto a *ragged* batch instead: each tree keeps its own
size (n_all_b) and alignment length (L_b), the per-tree programs are
concatenated in one plan (``trex_ragged_plan_build``) and one launch walks
all (tree, 64-site tile) work items -- no padded nodes or sites are computed.

* ``RaggedTreePlan(children_list, L_list)`` -- host planner.
* ``RaggedSankoffEngine`` -- forward / adjoint / fused / trex backtrack over
  packed tensors (layouts in include/trex_hip.h, "Ragged batches").
* ``from_padded(...)`` -- trex's padded representation (adjacency padded by
  ``pad_adjacency``, sequences by ``pad_tree_sequences`` / ``pad_sequence``,
  ``create_node_mask`` / ``create_sequence_mask``) -> the ragged batch with
  the padding stripped, so results equal the unpadded per-tree Sankoff.
"""

from __future__ import annotations

import numpy as np

from ._lib import TREX_FLAG_HARD_ROOT, TREX_PLAN_HEADER_INTS, check, lib, ptr, stream_handle
from .topology import children_from_adjacency


def _torch():
    import torch

    return torch


class RaggedTreePlan:
    """Per-tree child lists of different sizes + per-tree site counts."""

    def __init__(self, children_list, L_list):
        chs = [np.ascontiguousarray(np.asarray(c, dtype=np.int32)) for c in children_list]
        if not chs:
            raise ValueError("empty batch")
        for c in chs:
            if c.ndim != 2 or c.shape[1] != 2:
                raise ValueError(f"each children array must be (n_all_b, 2), got {c.shape}")
        self.B = len(chs)
        self.n_all = np.array([c.shape[0] for c in chs], dtype=np.int32)
        self.L = np.broadcast_to(np.asarray(L_list, dtype=np.int32), (self.B,)).copy()
        self.n_leaves = (self.n_all + 1) // 2
        self.n_int = self.n_all - self.n_leaves
        L_ = lib()
        n = int(L_.trex_ragged_plan_ints(self.B, ptr(self.n_all), ptr(self.L)))
        if n <= 0:
            raise ValueError("bad ragged plan shape (n_all_b >= 3, L_b >= 1)")
        self.host = np.zeros(n, dtype=np.int32)
        info = np.zeros(8, dtype=np.int64)
        packed = np.concatenate(chs, axis=0)
        check(L_.trex_ragged_plan_build(ptr(packed), ptr(self.n_all), ptr(self.L), self.B,
                                        ptr(self.host), ptr(info)))
        self.n_slots, self.max_leaves, self.items = int(info[0]), int(info[1]), int(info[2])
        self.leaf_bytes, self.row_sites, self.sites = int(info[3]), int(info[4]), int(info[5])
        self.backtrack_ok = int(info[6])
        self.steps = int(self.n_int.sum())
        meta = self.host[TREX_PLAN_HEADER_INTS:TREX_PLAN_HEADER_INTS + 12 * self.B].reshape(
            self.B, 12)
        self.site_offsets = meta[:, 4].astype(np.int64)
        self.leaf_offsets = meta[:, 6].astype(np.int64) | (meta[:, 7].astype(np.int64) << 32)
        self.row_offsets = meta[:, 8].astype(np.int64) | (meta[:, 9].astype(np.int64) << 32)
        self._dev = {}

    @classmethod
    def from_adjacencies(cls, adjacencies, L_list) -> "RaggedTreePlan":
        return cls([children_from_adjacency(a)[0] for a in adjacencies], L_list)

    def device(self, device):
        import torch

        key = str(device)
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(self.host).to(device)
        return self._dev[key]

    # -- packing helpers (host) -------------------------------------------
    def pack_leaves(self, leaves_list) -> np.ndarray:
        """per-tree int8 codes (n_leaves_b, L_b) -> packed [sum n_leaves_b L_b]."""
        out = np.empty(self.leaf_bytes, dtype=np.int8)
        for b, lv in enumerate(leaves_list):
            lv = np.asarray(lv, dtype=np.int8)
            if lv.shape != (self.n_leaves[b], self.L[b]):
                raise ValueError(f"tree {b}: leaves must be {(self.n_leaves[b], self.L[b])}")
            o = self.leaf_offsets[b]
            out[o:o + lv.size] = lv.reshape(-1)
        return out

    def tree_rows(self, packed, b: int):
        """tree b's view of a packed dp / marginal ([rows][Q]) or anc tensor."""
        o = int(self.row_offsets[b])
        n = int(self.n_int[b]) * int(self.L[b])
        t = packed[o:o + n]
        return t.reshape((int(self.n_int[b]), int(self.L[b])) + tuple(packed.shape[1:]))

    def tree_sites(self, packed, b: int):
        o = int(self.site_offsets[b])
        return packed[o:o + int(self.L[b])]


class RaggedSankoffEngine:
    """Sankoff over a ragged batch on the device (Q <= 128: Q <= 4 lane per
    site, up to 64 states state-parallel (sankoff_wide.hip), 64 < Q <= 128 a
    workgroup per state vector (sankoff_bigq.hip)).

    leaves: packed int8 device tensor (RaggedTreePlan.pack_leaves); cost (Q, Q)
    float32.  Mirrors SankoffEngine's forward / backward / fwd_bwd /
    backtrack; dp and marginals are packed ([sum n_int_b L_b], Q).
    """

    def __init__(self, plan: RaggedTreePlan, n_states: int, device=None):
        torch = _torch()
        if n_states > 128:
            raise NotImplementedError("alphabets above 128 states are not supported "
                                      "(int8 leaf codes / ancestral states)")
        self.plan = plan
        self.Q = int(n_states)
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.plan_dev = plan.device(self.device)
        nb = int(lib().trex_ragged_workspace_bytes(plan.items, self.Q))
        self.workspace = torch.empty(nb, dtype=torch.uint8, device=self.device)

    @property
    def dp_shape(self):
        return (self.plan.row_sites, self.Q)

    def _check(self, leaves, cost):
        torch = _torch()
        if leaves.dtype != torch.int8 or leaves.numel() != self.plan.leaf_bytes:
            raise ValueError(f"leaves must be packed int8 of {self.plan.leaf_bytes} codes")
        if cost.dtype != torch.float32 or tuple(cost.shape) != (self.Q, self.Q):
            raise ValueError(f"cost must be float32 ({self.Q}, {self.Q})")
        for t in (leaves, cost):
            if not t.is_contiguous() or t.device != self.device:
                raise ValueError("inputs must be contiguous tensors on the engine's device")

    def _run(self, phase, leaves, cost, tau, dp, site_score, tree_score, dts, dc, mg, an,
             hard_root):
        p = self.plan
        flags = TREX_FLAG_HARD_ROOT if hard_root else 0
        check(lib().trex_sankoff_ragged(
            phase, ptr(self.plan_dev), p.B, p.n_slots, p.max_leaves, p.items, ptr(leaves),
            ptr(cost), self.Q, float(tau), flags, ptr(dp), ptr(site_score), ptr(tree_score),
            ptr(dts), ptr(dc), ptr(mg), ptr(an), ptr(self.workspace), self.workspace.numel(),
            stream_handle(self.device)))

    def _dts(self, d_tree_score):
        torch = _torch()
        if d_tree_score is None:
            return None
        t = torch.as_tensor(d_tree_score, dtype=torch.float32, device=self.device).contiguous()
        if t.shape != (self.plan.B,):
            raise ValueError("d_tree_score must be (B,)")
        return t

    def forward(self, leaves, cost, tau: float = 0.0, *, site_score=False, hard_root=False):
        """(tree_score (B,), dp packed, site_score packed | None)."""
        torch = _torch()
        self._check(leaves, cost)
        f32 = dict(dtype=torch.float32, device=self.device)
        dp = torch.empty(self.dp_shape, **f32)
        ts = torch.empty((self.plan.B,), **f32)
        ss = torch.empty((self.plan.sites,), **f32) if site_score else None
        self._run(1, leaves, cost, tau, dp, ss, ts, None, None, None, None, hard_root)
        return ts, dp, ss

    def backward(self, leaves, cost, tau, dp, d_tree_score=None, *, marginals=False,
                 anc_states=False, hard_root=False):
        """(d_cost, marginals packed | None, anc_states packed | None)."""
        torch = _torch()
        self._check(leaves, cost)
        if tuple(dp.shape) != self.dp_shape:
            raise ValueError("backward needs the forward's packed dp table")
        dc = torch.empty((self.Q, self.Q), dtype=torch.float32, device=self.device)
        mg = torch.empty(self.dp_shape, dtype=torch.float32, device=self.device) \
            if marginals else None
        an = torch.empty((self.plan.row_sites,), dtype=torch.int8, device=self.device) \
            if anc_states else None
        self._run(2, leaves, cost, tau, dp, None, None, self._dts(d_tree_score), dc, mg, an,
                  hard_root)
        return dc, mg, an

    def fwd_bwd(self, leaves, cost, tau: float = 0.0, d_tree_score=None, *, site_score=False,
                marginals=False, anc_states=False, hard_root=False):
        """Fused launch: (tree_score, dp, site_score | None, d_cost, marginals | None,
        anc_states | None)."""
        torch = _torch()
        self._check(leaves, cost)
        f32 = dict(dtype=torch.float32, device=self.device)
        dp = torch.empty(self.dp_shape, **f32)
        ts = torch.empty((self.plan.B,), **f32)
        ss = torch.empty((self.plan.sites,), **f32) if site_score else None
        dc = torch.empty((self.Q, self.Q), **f32)
        mg = torch.empty(self.dp_shape, **f32) if marginals else None
        an = torch.empty((self.plan.row_sites,), dtype=torch.int8, device=self.device) \
            if anc_states else None
        self._run(3, leaves, cost, tau, dp, ss, ts, self._dts(d_tree_score), dc, mg, an,
                  hard_root)
        return ts, dp, ss, dc, mg, an

    def value_and_grad(self, leaves, cost, tau: float = 0.0, d_tree_score=None,
                       hard_root=False):
        ts, _, _, dc, _, _ = self.fwd_bwd(leaves, cost, tau, d_tree_score, hard_root=hard_root)
        return ts, dc

    def backtrack(self, cost, dp):
        """trex-exact ancestral states, packed int8 [sum n_int_b L_b]."""
        torch = _torch()
        p = self.plan
        an = torch.empty((p.row_sites,), dtype=torch.int8, device=self.device)
        check(lib().trex_sankoff_ragged_backtrack(
            ptr(self.plan_dev), p.B, p.items, p.steps, p.backtrack_ok, ptr(cost), ptr(dp),
            self.Q, ptr(an), stream_handle(self.device)))
        return an


# ---------------------------------------------------------------------------
# trex's padded representation -> ragged batch
# ---------------------------------------------------------------------------
def _host(x):
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def from_padded(adjacency, node_mask, sequences, seq_mask, n_states: int):
    """Strip trex-style padding (padding.py) from a batch of trees.

    adjacency (B, MAX, MAX) padded by ``pad_adjacency`` (zeros past the real
    nodes); node_mask (B, MAX) from ``create_node_mask`` (a prefix of True);
    sequences (B, >= n_leaves, N_pad) leaf states padded by ``pad_sequence``;
    seq_mask (B, N_pad) from ``create_sequence_mask`` (a prefix of True).
    Returns (RaggedTreePlan, packed int8 leaf codes (host), per-tree
    (n_all_b, L_b)).  Leaf states follow run_sankoff's conversion
    (sankoff.py:49-52: truncate, wrap negatives once, out of range -> all-1e5).
    """
    A = _host(adjacency)
    nm = _host(node_mask).astype(bool)
    S = _host(sequences)
    sm = _host(seq_mask).astype(bool)
    if A.ndim != 3 or nm.shape != A.shape[:2] or S.ndim != 3 or sm.shape != (S.shape[0],
                                                                              S.shape[2]):
        raise ValueError("shapes: adjacency (B, M, M), node_mask (B, M), sequences (B, n, N), "
                         "seq_mask (B, N)")
    children, Ls, leaves, shapes = [], [], [], []
    for b in range(A.shape[0]):
        n_all = int(nm[b].sum())
        L = int(sm[b].sum())
        if not nm[b, :n_all].all() or not sm[b, :L].all():
            raise ValueError(f"tree {b}: masks must be a prefix of True (create_*_mask)")
        nl = (n_all + 1) // 2
        children.append(children_from_adjacency(A[b, :n_all, :n_all])[0])
        Ls.append(L)
        s = np.trunc(S[b, :nl, :L].astype(np.float64))
        s = np.where(np.isnan(s), 0.0, s)  # XLA's f32 -> s32 convert: NaN -> 0
        s = np.where(s < 0, s + n_states, s)
        leaves.append(np.where((s >= 0) & (s < n_states), s, -1).astype(np.int8))
        shapes.append((n_all, L))
    plan = RaggedTreePlan(children, Ls)
    return plan, plan.pack_leaves(leaves), shapes
