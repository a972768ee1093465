"""CPU restatement of the device data generators (trex_amd/csrc/datagen.hip).

TEST INFRASTRUCTURE ONLY (import rule: see oracle/sankoff_ref.py header).

trex's generate_groundtruth / mutate (src/trex/ground_truth.py:20-52,
112-197) draw with JAX's threefry PRNG, which cannot run here; the build
keeps the process and replaces the random numbers with a counter-based
generator r(seed, stream, counter) = mix(seed ^ mix(stream << 32 | counter))
(mix = splitmix64's finaliser).  This file computes the same numbers with
numpy uint64 arithmetic, so the device generator is checked bit for bit; the
reference's own invariants (exactly n_mutations changed sites per edge,
states in [0, Q), zero root) are checked on both.
"""

from __future__ import annotations

import math

import numpy as np

_U = np.uint64


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + _U(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _U(30))) * _U(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U(27))) * _U(0x94D049BB133111EB)
    return z ^ (z >> _U(31))


def draw(seed, stream, counter):
    counter = np.asarray(counter, dtype=np.uint64) & _U(0xFFFFFFFF)
    stream = np.asarray(stream, dtype=np.uint64)
    return mix64(_U(seed) ^ mix64((stream << _U(32)) | counter))


def choose_sites(seed, child, L, n_mut):
    """Floyd's sampling without replacement (datagen.hip choose_sites_kernel)."""
    s = []
    for j in range(L - n_mut, L):
        r = int(draw(seed, 2 * child + 1, j) % _U(j + 1))
        s.append(j if r in s else r)
    return s


def generate_groundtruth(seed, n_leaves, L, Q, n_mutations):
    """int8 [2 n_leaves - 1][L], root (last row) zero, parents from the root down."""
    nl = n_leaves
    n_all = 2 * nl - 1
    seqs = np.zeros((n_all, L), dtype=np.int64)
    sites = np.arange(L)
    for i in range(nl - 1):  # ground_truth.py:165-178
        parent = n_all - 1 - i
        for child in (2 * (parent - nl), 2 * (parent - nl) + 1):
            x = seqs[parent].copy()
            if n_mutations > 0:
                hit = np.array(choose_sites(seed, child, L, n_mutations))
                off = 1 + (draw(seed, 2 * child, sites[hit]) % _U(Q - 1)).astype(np.int64)
                x[hit] = (x[hit] + off) % Q
            seqs[child] = x
    return seqs.astype(np.int8)


def uniform_states(seed, n, Q, start=0):
    """elements [start, n) of the device's uniform_states output"""
    i = np.arange(start, n, dtype=np.uint64)
    return (draw(seed, (i >> _U(32)) + _U(1 << 32), i) % _U(Q)).astype(np.int8)


def gumbel_noise(seed, step, n):
    """trex_gumbel_noise (datagen.hip gumbel_kernel): Gumbel(0, 1) noise of
    device-loop step `step`, f32 [n]; u in (0, 1) from 53 bits + 1/2,
    -log(-log u) in double."""
    with np.errstate(over="ignore"):
        sk = mix64(_U(seed) ^ (_U(0x6A09E667F3BCC909) * _U(step + 1)))
    i = np.arange(n, dtype=np.uint64)
    r = draw(sk, _U(0x7FFF0000) + (i >> _U(32)), i)
    u = ((r >> _U(11)).astype(np.float64) + 0.5) * 2.0 ** -53
    return (-np.log(-np.log(u))).astype(np.float32)


def _unit53(r):
    return float(int(r) >> 11) * 2.0 ** -53


def _unit24(r):
    return np.float32(int(r) >> 40) * np.float32(2.0 ** -24)


def _fixed_fitness(seq, inter, fit, Q):
    L, K = inter.shape if inter.size else (seq.shape[0], 0)
    idx = seq.astype(np.int64).copy()
    pw = Q
    for j in range(K):
        idx += seq[inter[:, j]].astype(np.int64) * pw
        pw *= Q
    vals = fit[np.arange(seq.shape[0]), idx].astype(np.float64)
    return int((vals * 2.0 ** 40).astype(np.int64).sum())


def sorted_nodes_ref(adjacency):
    """The traversal of trex's generate_tree_data, step by step as the JAX
    program runs it (src/trex/nk_model.py:154-192).  Written independently of
    trex_amd.datagen.reference_sorted_nodes so the two check each other.

    Returns (root, parent, sorted_nodes) with the reference's -1 slots kept.
    JAX semantics restated: jnp.argmax takes the first maximum (:154);
    jnp.where(..., size=k) pads with 0 (:155, :170); ``x.at[i].set(v)`` with
    i outside [0, n) is dropped (:167, :176); lax.cond reads ``visited``
    as updated at :168.
    """
    A = np.asarray(adjacency)
    n = A.shape[0]
    parent = [int(np.argmax(A[r])) for r in range(n)]
    selfp = [i for i in range(n) if parent[i] == i]
    root = (selfp + [0])[0]
    queue = [root] + [-1] * (n - 1)
    visited = [False] * n
    sorted_nodes = [-1] * n
    guard = 0
    while any(q != -1 for q in queue):
        current = queue[0]
        queue = queue[1:] + [-1]                    # .at[0].set(-1) then roll(-1)
        slot = sum(visited)
        if slot < n:
            sorted_nodes[slot] = current
        visited[current] = True
        children = [i for i in range(n) if A[i, current] == 1]
        children += [0] * (n - len(children))      # size=n, fill 0
        for child in children:                     # fori_loop(0, n)
            if not visited[child]:
                pos = sum(q != -1 for q in queue)
                if pos < n:
                    queue[pos] = child
        guard += 1
        assert guard <= n * n + n, "BFS did not terminate"
    return root, np.asarray(parent, np.int64), np.asarray(sorted_nodes, np.int64)


def evolve_order_ref(adjacency):
    """(root, parent, order) with the -1 slots resolved the way the evolve
    loop indexes them (nk_model.py:199-262): ``sorted_nodes[i] = -1`` reads
    ``parent_indices[-1]`` and writes ``sequences.at[-1]`` -- row n - 1 --
    and ``-1 != root_node``, so the slot evolves even when n - 1 is the
    root."""
    root, parent, sn = sorted_nodes_ref(adjacency)
    n = len(parent)
    return root, parent, np.where(sn < 0, n - 1, sn)


def generate_tree_data(seed, interactions, fitness, parent, order, root_seq, Q, mutation_rate,
                       noise_std, coupled_prob, branch_length):
    """trex_datagen_nk_tree restated (the device's draws and fixed-point
    fitness): the nodes of ``order`` (``evolve_order_ref``: the
    reference's BFS sorted_nodes, root first, -1 slots resolved to the last
    node) evolve from their parents in slot order, slot s drawing from
    streams 4s .. 4s + 3 (nk_model.py:192-262); returns int8 (n_nodes, L)."""
    inter = np.asarray(interactions, np.int64)
    fit = np.asarray(fitness, np.float32)
    L = len(root_seq)
    K = inter.shape[1] if inter.ndim == 2 else 0
    inter = inter.reshape(L, K)
    n = len(parent)
    seqs = np.zeros((n, L), np.int64)
    root = int(order[0])
    seqs[root] = np.asarray(root_seq).reshape(-1)
    sites = np.arange(L, dtype=np.uint64)
    mr32, cp32 = np.float32(mutation_rate), np.float32(coupled_prob)
    for slot in range(1, len(order)):  # slot 0 is the root; streams per BFS slot
        node = int(order[slot])
        sb = 4 * slot
        cur = seqs[int(parent[node])].copy()
        rate = np.float32(min(mr32, np.float32(1.0)))
        if np.float32(noise_std) != 0:
            u1 = 1.0 - _unit53(draw(seed, sb, 0))
            u2 = _unit53(draw(seed, sb, 1))
            z = math.sqrt(-2.0 * math.log(u1)) * math.cos(6.283185307179586 * u2)
            rate = min(np.float32(float(mr32) * math.exp(z * float(np.float32(noise_std)))),
                       np.float32(1.0))
        fcur = _fixed_fitness(cur, inter, fit, Q)
        for b in range(branch_length):
            coupled = _unit24(draw(seed, sb + 1, 4 * b)) < cp32
            site0 = int(draw(seed, sb + 1, 4 * b + 1) % _U(L))
            if coupled:
                m = np.zeros(L, bool)
                m[site0] = True
                m[inter[site0]] = True
            else:
                r = draw(seed, sb + 3, _U(b * L) + sites)
                m = ((r >> _U(40)).astype(np.float32) * np.float32(2.0 ** -24)) < rate
            v = (draw(seed, sb + 2, _U(b * L) + sites) % _U(Q)).astype(np.int64)
            prop = np.where(m, v, cur)
            fprop = _fixed_fitness(prop, inter, fit, Q)
            delta = float(fprop - fcur) * 2.0 ** -40 / L
            if delta >= 0.0 or _unit53(draw(seed, sb + 1, 4 * b + 2)) < math.exp(delta):
                cur, fcur = prop, fprop
        seqs[node] = cur
    return seqs.astype(np.int8)
