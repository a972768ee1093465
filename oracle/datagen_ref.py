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
