"""Tree topologies: trex adjacency conventions -> device plans.

Adjacency orientation follows trex: ``adj[i, j] == 1`` means node ``i`` is a
child of node ``j`` (src/trex/utils/types.py:30-35).  Leaves are
0..n_leaves-1, internal nodes n_leaves..n_all-1, the root is n_all-1.
"""

from __future__ import annotations

import numpy as np

from ._lib import TREX_PLAN_HEADER_INTS, check, lib


def children_from_adjacency(adj, *, drop_root_self_loop: bool = True) -> np.ndarray:
    """trex's child lists for every node.

    ``jnp.where(adj[:, node] == 1, size=2, fill_value=-1)[0]``
    (src/trex/sankoff.py:60) applied after run_sankoff zeroes ``adj[-1, -1]``
    (sankoff.py:141; ``drop_root_self_loop=False`` is run_dp called directly,
    which does not).  ``adj``: (n_all, n_all) or (B, n_all, n_all).
    Returns int32 (B, n_all, 2).
    """
    a = np.asarray(adj)
    if a.ndim == 2:
        a = a[None]
    if a.ndim != 3 or a.shape[1] != a.shape[2]:
        raise ValueError(f"adjacency must be (n_all, n_all) or (B, n_all, n_all), got {a.shape}")
    mask = a == 1
    if drop_root_self_loop:
        mask[:, -1, -1] = False
    B, n_all, _ = mask.shape
    # cumulative count down each column; first hit has count 1, second count 2
    cnt = np.cumsum(mask, axis=1)
    out = np.full((B, n_all, 2), -1, dtype=np.int32)
    for k in (1, 2):
        hit = mask & (cnt == k)
        has = hit.any(axis=1)  # (B, n_all)
        row = hit.argmax(axis=1)
        out[:, :, k - 1] = np.where(has, row, -1)
    return out


def create_balanced_binary_tree(n_leaves: int) -> np.ndarray:
    """Adjacency of trex's balanced tree (src/trex/evals/benchmark.py:781-791)."""
    n_anc = n_leaves - 1
    n_total = n_leaves + n_anc
    adj = np.zeros((n_total, n_total), dtype=np.float32)
    adj[np.arange(n_leaves), n_leaves + np.arange(n_leaves) // 2] = 1
    adj[n_leaves + np.arange(n_anc - 1), n_leaves + (np.arange(n_anc - 1) + n_leaves) // 2] = 1
    return adj


def random_topologies(B: int, n_leaves: int, seed: int) -> np.ndarray:
    """Random binary topologies as child lists (B, n_all, 2).

    Coalescent merge: two random active nodes join under new node n_leaves+k,
    so every child id is lower than its parent (trex's post-order numbering).
    """
    rng = np.random.default_rng(seed)
    n_all = 2 * n_leaves - 1
    out = np.full((B, n_all, 2), -1, dtype=np.int32)
    for b in range(B):
        active = list(range(n_leaves))
        for k in range(n_leaves - 1):
            i, j = rng.choice(len(active), size=2, replace=False)
            ci, cj = active[i], active[j]
            parent = n_leaves + k
            lo, hi = min(ci, cj), max(ci, cj)
            out[b, parent] = (lo, hi)  # jnp.where returns rows ascending
            active = [x for t, x in enumerate(active) if t not in (i, j)] + [parent]
    return out


def adjacency_from_children(children: np.ndarray) -> np.ndarray:
    """Inverse of children_from_adjacency for well-formed child lists."""
    ch = np.asarray(children)
    if ch.ndim == 2:
        ch = ch[None]
    B, n_all, _ = ch.shape
    adj = np.zeros((B, n_all, n_all), dtype=np.float32)
    for b in range(B):
        for node in range(n_all):
            for c in ch[b, node]:
                if c >= 0:
                    adj[b, c, node] = 1
    return adj


class TreePlan:
    """A batch of topologies compiled by the host planner (trex_plan_build)."""

    def __init__(self, children: np.ndarray):
        ch = np.ascontiguousarray(children, dtype=np.int32)
        if ch.ndim == 2:
            ch = ch[None]
        if ch.ndim != 3 or ch.shape[2] != 2:
            raise ValueError(f"children must be (B, n_all, 2), got {ch.shape}")
        self.B, self.n_all, _ = ch.shape
        self.n_leaves = (self.n_all + 1) // 2
        self.n_int = self.n_all - self.n_leaves
        L = lib()
        n = L.trex_plan_ints(self.B, self.n_all)
        if n <= 0:
            raise ValueError(f"bad plan shape B={self.B} n_all={self.n_all}")
        self.host = np.zeros(n, dtype=np.int32)
        info = np.zeros(4, dtype=np.int32)
        check(L.trex_plan_build(ch.ctypes.data, self.B, self.n_all, self.host.ctypes.data,
                                info.ctypes.data))
        self.children = ch
        # info[0]: stack depth | (lane-program slots + 1) << 16; the C calls
        # take the whole word
        self.slot_word = int(info[0])
        self.n_slots = self.slot_word & 0xFFFF
        self.lane_slots = ((self.slot_word >> 16) & 0xFF) - 1
        self.backtrack_ok = int(info[1])
        self.n_dag_nodes = int(info[2])
        self.n_unreached = int(info[3])
        self._dev = {}

    @classmethod
    def from_adjacency(cls, adj) -> "TreePlan":
        return cls(children_from_adjacency(adj))

    def device(self, device):
        """The plan as an int32 device tensor (cached per device)."""
        import torch

        key = str(device)
        if key not in self._dev:
            self._dev[key] = torch.from_numpy(self.host).to(device)
        return self._dev[key]

    @property
    def fwd_steps(self) -> np.ndarray:
        """(B, n_int, 4) encoded forward steps (see trex_common.h)."""
        o = TREX_PLAN_HEADER_INTS
        return self.host[o:o + self.B * self.n_int * 4].reshape(self.B, self.n_int, 4)
