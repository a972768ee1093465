"""Synthetic data generators of trex, restated on the host (numpy).

SURVEY.md §8(f) rank 3: the ground-truth and NK-model generators feed the
benchmarks; they are not on the hot path, and the survey's plan is that host
numpy suffices.  Restated processes (values differ: the reference draws with
JAX's threefry PRNG, which cannot run here; ``seed`` seeds numpy's PCG64):

* ``mutate``               src/trex/ground_truth.py:20-52
* ``generate_groundtruth`` src/trex/ground_truth.py:112-197
* ``create_nk_model_landscape`` src/trex/nk_model.py:17-43
* ``get_fitness``          src/trex/nk_model.py:46-110
* ``generate_tree_data``   src/trex/nk_model.py:116-278, including its index
  semantics: the root is the first node whose argmax parent is itself
  (``jnp.where(..., size=1)`` fills 0 when there is none), the reference's
  fixed-size BFS queue with 0-padded child lists and dropped out-of-range
  writes (``reference_sorted_nodes``), and unfilled BFS slots are -1, which
  index the LAST node (numpy/JAX negative-index wrap), as in the reference.

Outputs are numpy arrays in the reference's dtypes/shapes; move them to the
device with torch when a kernel needs them.
"""

from __future__ import annotations

from collections import namedtuple

import numpy as np

PhylogeneticTree = namedtuple("PhylogeneticTree",
                              ["masked_sequences", "all_sequences", "adjacency"])


def _rng(seed):
    return seed if isinstance(seed, np.random.Generator) else np.random.default_rng(seed)


def mutate(rng, sequence, n_states: int, n_mutations: int) -> np.ndarray:
    """Exactly ``n_mutations`` distinct sites get (x + U{1..Q-1}) mod Q
    (ground_truth.py:39-52).  int8."""
    rng = _rng(rng)
    seq = np.asarray(sequence)
    mask = np.zeros(seq.shape[0], dtype=bool)
    if n_mutations > 0:
        mask[rng.choice(seq.shape[0], size=n_mutations, replace=False)] = True
    offsets = rng.integers(1, n_states, size=seq.shape)
    return np.where(mask, (seq + offsets) % n_states, seq).astype(np.int8)


def generate_groundtruth(n_leaves: int, n_states: int, n_mutations: int, seq_length: int,
                         seed: int = 42) -> PhylogeneticTree:
    """Balanced tree from a zero root, children = mutate(parent) per split
    (ground_truth.py:112-197).  float32 outputs as the reference."""
    if not (n_leaves > 0 and (n_leaves & (n_leaves - 1)) == 0):
        raise ValueError("n_leaves must be a power of 2.")
    rng = _rng(seed)
    n_anc = n_leaves - 1
    n_all = n_leaves + n_anc
    seqs = np.zeros((n_all, seq_length), dtype=np.int8)
    for i in range(n_anc):  # parents from the root down (:165-178)
        parent = n_all - 1 - i
        p_i = parent - n_leaves
        seqs[2 * p_i] = mutate(rng, seqs[parent], n_states, n_mutations)
        seqs[2 * p_i + 1] = mutate(rng, seqs[parent], n_states, n_mutations)
    masked = np.zeros_like(seqs)
    masked[:n_leaves] = seqs[:n_leaves]
    adj = np.zeros((n_all, n_all), dtype=np.float32)
    i = np.arange(n_anc)
    adj[2 * i, n_leaves + i] = 1
    adj[2 * i + 1, n_leaves + i] = 1
    return PhylogeneticTree(masked.astype(np.float32), seqs.astype(np.float32), adj)


def create_nk_model_landscape(n: int, k: int, seed=0, n_states: int = 2) -> dict:
    """interactions U{0..n-1} (n, k), fitness tables U[0, 1) (n, q^(k+1))
    (nk_model.py:31-43)."""
    rng = _rng(seed)
    return {"interactions": rng.integers(0, n, size=(n, k)).astype(np.int32),
            "fitness_tables": rng.uniform(size=(n, n_states ** (k + 1))).astype(np.float32),
            "n_states": n_states, "k": k}


def get_fitness(sequence, landscape: dict, seq_mask=None) -> float:
    """Masked mean of f_i at index sum_j s_j q^j with s_0 the site's own
    state (nk_model.py:89-110; least-significant-first, unlike the parental
    logits' table reshape)."""
    seq = np.asarray(sequence).astype(np.int64).reshape(-1)
    inter = np.asarray(landscape["interactions"])
    q = int(landscape["n_states"])
    n = seq.shape[0]
    mask = np.ones(n, bool) if seq_mask is None else np.asarray(seq_mask, bool)
    idx = np.concatenate([np.arange(n)[:, None], inter], axis=1)
    powers = q ** np.arange(idx.shape[1])
    table_idx = (seq[idx] * powers).sum(1)
    vals = np.asarray(landscape["fitness_tables"])[np.arange(n), table_idx]
    return float((vals * mask).sum() / mask.sum())


def reference_sorted_nodes(adjacency):
    """generate_tree_data's traversal, restated with JAX's semantics
    (nk_model.py:154-192).  Returns (root, parent, sorted_nodes int64 (n,)).

    * parent = first argmax of each adjacency row (:154); root = the first
      node that is its own parent, 0 when none is (``jnp.where(size=1)``'s
      fill value, :155);
    * a fixed queue of n slots, -1 = empty (:184); each step pops slot 0 and
      rolls (:163-165), writes the popped node to
      ``sorted_nodes[sum(visited)]`` BEFORE marking it (:167-168) -- so a
      node popped twice overwrites the slot the next new node then takes,
      and a write at index n is dropped (JAX scatter out of bounds);
    * children = ``jnp.where(adj[:, node] == 1, size=n)`` padded with 0
      (:170), each enqueued at ``sum(queue != -1)`` if not yet visited
      (:172-181) -- the pads enqueue node 0 over and over while it is
      unvisited, and enqueues past the last slot are dropped, so some nodes
      may never be reached (their rows stay zero in the reference);
    * unfilled slots stay -1 (:186), which the evolve loop indexes as the
      last node (:199-262).
    """
    A = np.asarray(adjacency)
    n = A.shape[0]
    parent = np.argmax(A, axis=1).astype(np.int64)
    selfp = np.nonzero(parent == np.arange(n))[0]
    root = int(selfp[0]) if selfp.size else 0
    queue = np.full(n, -1, np.int64)
    queue[0] = root
    visited = np.zeros(n, bool)
    order = np.full(n, -1, np.int64)
    steps = 0
    while (queue != -1).any():
        cur = int(queue[0])
        queue[0] = -1
        queue = np.roll(queue, -1)
        k = int(visited.sum())
        if k < n:
            order[k] = cur
        visited[cur] = True
        kids = np.nonzero(A[:, cur] == 1)[0]
        kids = np.concatenate([kids, np.zeros(n - kids.size, np.int64)])
        for c in kids:
            if not visited[c]:
                pos = int((queue != -1).sum())
                if pos < n:
                    queue[pos] = c
        steps += 1
        if steps > n * n + n:  # every pop either visits a node or drains a duplicate
            raise RuntimeError("reference_sorted_nodes: BFS did not terminate")
    return root, parent, order


def generate_tree_data(landscape: dict, adjacency, root_sequence, mutation_rate: float, seed=0,
                       coupled_mutation_prob: float = 0.5, n_states: int = 20,
                       mutation_rate_noise_std: float = 0.0,
                       branch_length: int = 1) -> PhylogeneticTree:
    """NK-model sequence evolution along a tree with Metropolis acceptance
    (nk_model.py:116-278)."""
    rng = _rng(seed)
    A = np.asarray(adjacency)
    n = A.shape[0]
    root_seq = np.asarray(root_sequence).reshape(-1)
    L = root_seq.shape[0]
    if "n_states" in landscape:
        n_states = int(landscape["n_states"])
    root, parent, order = reference_sorted_nodes(A)
    seqs = np.zeros((n, L), dtype=np.int64)
    seqs[root] = root_seq
    inter = np.asarray(landscape["interactions"])
    for i in range(n):
        node = int(order[i])  # -1 wraps to the last node, as in the reference
        if node == root:  # -1 != root_node (:257): a -1 slot evolves row n-1 even if it is the root
            continue
        rate = min(mutation_rate * np.exp(rng.normal() * mutation_rate_noise_std), 1.0)
        seq = seqs[parent[node]].copy()
        for _ in range(branch_length):
            if rng.random() < coupled_mutation_prob:
                site = int(rng.integers(0, L))
                mask = np.zeros(L, bool)
                mask[np.concatenate([[site], inter[site]]).astype(np.int64)] = True
                proposal = np.where(mask, rng.integers(0, n_states, size=L), seq)
            else:
                mask = rng.random(L) < rate
                proposal = np.where(mask, rng.integers(0, n_states, size=L), seq)
            acc = np.exp(get_fitness(proposal, landscape) - get_fitness(seq, landscape))
            if rng.random() < min(1.0, acc):
                seq = proposal
        seqs[node] = seq
    return PhylogeneticTree(np.zeros((n, L), np.float32), seqs.astype(np.float32),
                            A.astype(np.float32))


# ---------------------------------------------------------------------------
# Device generators (libtrexhip.so, trex_amd/csrc/datagen.hip): the same
# ground-truth process run where the data are consumed, so C4/C5-size inputs
# never cross PCIe.  Random numbers come from a counter-based generator
# (splitmix64 of (seed, stream, counter)); oracle/datagen_ref.py computes them
# bit for bit on the CPU.


def generate_groundtruth_device(n_leaves: int, n_states: int, n_mutations: int, seq_length: int,
                                seed: int = 42, device="cuda"):
    """generate_groundtruth's process on the device: returns (all_sequences
    int8 (2 n_leaves - 1, seq_length) on `device`, adjacency float32 numpy),
    same numbering as the host version (leaves first, root last)."""
    import torch

    from ._lib import check, lib, ptr, stream_handle

    if not (n_leaves > 1 and (n_leaves & (n_leaves - 1)) == 0):
        raise ValueError("n_leaves must be a power of 2 (and > 1).")
    dev = torch.device(device)
    n_all = 2 * n_leaves - 1
    seqs = torch.empty((n_all, seq_length), dtype=torch.int8, device=dev)
    ws = torch.empty(int(lib().trex_datagen_workspace_bytes(n_leaves, n_mutations)),
                     dtype=torch.uint8, device=dev)
    check(lib().trex_datagen_groundtruth(seed & (2**64 - 1), n_leaves, seq_length, n_states,
                                         n_mutations, ptr(seqs), ptr(ws), ws.numel(),
                                         stream_handle(dev)))
    adj = np.zeros((n_all, n_all), dtype=np.float32)
    i = np.arange(n_leaves - 1)
    adj[2 * i, n_leaves + i] = 1
    adj[2 * i + 1, n_leaves + i] = 1
    return seqs, adj


def uniform_states_device(shape, n_states: int, seed: int = 0, device="cuda"):
    """iid uniform states in [0, n_states), int8 tensor of `shape` on `device`."""
    import torch

    from ._lib import check, lib, ptr, stream_handle

    out = torch.empty(shape, dtype=torch.int8, device=torch.device(device))
    if out.numel():
        check(lib().trex_datagen_uniform_states(seed & (2**64 - 1), out.numel(), n_states,
                                                ptr(out), stream_handle(out.device)))
    return out


def bfs_levels(adjacency):
    """generate_tree_data's evolve order (nk_model.py:194-269) as launch
    levels for the device.  Returns (root, parent, order, offsets):
    ``order`` is the reference's sorted_nodes (``reference_sorted_nodes``)
    with its -1 slots resolved as the reference indexes them (node n - 1,
    evolved from parent[n - 1] even when that is the root), slot 0 the root
    (never evolved); ``offsets`` cut the slots into levels a launch may run
    in parallel: consecutive slots none of which writes a row another slot
    of the level reads or writes.  Sequential slot order is the semantics;
    levels only batch slots whose order does not matter."""
    root, parent, sorted_nodes = reference_sorted_nodes(adjacency)
    n = parent.shape[0]
    order = np.where(sorted_nodes < 0, n - 1, sorted_nodes).astype(np.int32)
    offsets = [0, 1]
    written, read = set(), set()
    for slot in range(1, n):
        node, par = int(order[slot]), int(parent[order[slot]])
        if node in written or node in read or par in written:
            offsets.append(slot)
            written, read = set(), set()
        written.add(node)
        read.add(par)
    if offsets[-1] != n:
        offsets.append(n)
    return root, parent.astype(np.int32), order, np.asarray(offsets, np.int32)


def generate_tree_data_device(landscape: dict, adjacency, root_sequence, mutation_rate: float,
                              seed: int = 0, coupled_mutation_prob: float = 0.5,
                              n_states: int = 20, mutation_rate_noise_std: float = 0.0,
                              branch_length: int = 1, device="cuda"):
    """generate_tree_data's process on the device (trex_datagen_nk_tree):
    returns the (n_nodes, L) int8 sequences on ``device`` (every node in BFS
    order evolved from its parent; the root row is root_sequence)."""
    import torch

    from ._lib import check, lib, ptr, stream_handle

    if "n_states" in landscape:
        n_states = int(landscape["n_states"])
    dev = torch.device(device)
    root, parent, order, offsets = bfs_levels(adjacency)
    inter = np.asarray(landscape["interactions"], np.int32)
    fit = np.asarray(landscape["fitness_tables"], np.float32)
    L = int(np.asarray(root_sequence).reshape(-1).shape[0])
    K = int(inter.shape[1]) if inter.ndim == 2 else 0
    n = parent.shape[0]
    # the kernel indexes LDS and the fitness table with these: validate here
    # (the reference's jnp gathers would clamp; out-of-range input is a bug)
    rs_host = np.asarray(root_sequence).reshape(-1)
    if inter.size and (inter.shape[0] != L or inter.min() < 0 or inter.max() >= L):
        raise ValueError(f"interactions must be (L={L}, K) with entries in [0, {L})")
    if rs_host.size and (rs_host.min() < 0 or rs_host.max() >= n_states):
        raise ValueError(f"root_sequence states must lie in [0, {n_states})")
    if fit.shape != (L, n_states ** (K + 1)):
        raise ValueError(f"fitness_tables must be (L, Q^(K+1)) = ({L}, {n_states ** (K + 1)}), "
                         f"got {fit.shape}")
    seqs = torch.zeros((n, L), dtype=torch.int8, device=dev)
    seqs[root] = torch.as_tensor(np.asarray(root_sequence).reshape(-1).astype(np.int8), device=dev)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    inter_d, fit_d, par_d, ord_d = t(inter), t(fit), t(parent), t(order)
    check(lib().trex_datagen_nk_tree(seed & (2**64 - 1), n, L, n_states, K, ptr(inter_d),
                                     ptr(fit_d), ptr(par_d), ptr(ord_d), offsets.ctypes.data,
                                     len(offsets) - 1, float(mutation_rate),
                                     float(mutation_rate_noise_std), float(coupled_mutation_prob),
                                     int(branch_length), ptr(seqs), stream_handle(dev)))
    return seqs
