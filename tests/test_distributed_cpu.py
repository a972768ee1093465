"""world_size-2 gloo test of the N>1 path (tree sharding + [dC, loss] all-reduce).

Runs on CPU: each rank evaluates its shard with the C restatement
(oracle/cpu_port.c, standing in for the GPU kernel that has no CPU build) and
the ranks reduce through trex_amd.distributed.GradReducer -- the same code
bench.py uses over RCCL.  The reduced gradient and loss must equal the
single-process values over the whole batch.
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from _cases import hamming, random_leaves, random_topologies
from trex_amd.distributed import GradReducer, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle.cpu_port import fwd_bwd

    B, n, L, Q, tau = 10, 12, 200, 4, 0.5
    ch = random_topologies(B, n, seed=1)
    leaves = random_leaves(B, n, L, Q, seed=2)
    lo, hi = shard_bounds(B, rank, world)
    ts, dc, _ = fwd_bwd(ch[lo:hi], leaves[lo:hi], hamming(Q), tau, threads=1)
    red = GradReducer(Q, "cpu")
    gdc, gloss = red(torch.from_numpy(dc.astype(np.float32)),
                     torch.from_numpy(ts.astype(np.float32)))
    out[rank] = (gdc.numpy().copy(), float(gloss))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover_exactly():
    for n in (0, 1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(300)
def test_gloo_world2_allreduce_matches_single_process():
    from oracle.cpu_port import fwd_bwd

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    B, n, L, Q, tau = 10, 12, 200, 4, 0.5
    ts, dc, _ = fwd_bwd(random_topologies(B, n, seed=1), random_leaves(B, n, L, Q, seed=2),
                        hamming(Q), tau, threads=1)
    for r in range(world):
        gdc, gloss = out[r]
        np.testing.assert_allclose(gdc, dc, rtol=1e-6)
        np.testing.assert_allclose(gloss, ts.sum(), rtol=1e-6)


def _c5_case():
    from oracle import tree_ref as T

    rng = np.random.default_rng(9)
    nl, L, Q = 8, 40, 4
    n = 2 * nl - 1
    S = np.zeros((n, L, Q))
    S[:nl] = np.eye(Q)[rng.integers(0, Q, size=(nl, L))]
    S[nl:] = T.update_seq(rng.normal(size=(nl - 1, L, Q)), S, 0.7)[nl:]
    A = T.update_tree(rng.normal(size=(n - 1, nl - 1)), rng.gumbel(size=(n - 1, nl - 1)))
    return S, A


def _c5_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trex_amd.distributed import GramReducer

    S, A = _c5_case()
    lo, hi = shard_bounds(S.shape[1], rank, world)
    F = S[:, lo:hi].reshape(S.shape[0], -1)
    G = torch.from_numpy(F @ F.T)  # this rank's sites only
    GramReducer()(G)
    G = G.numpy()
    # the combine every rank runs on the reduced Gram (tree.py:199-209)
    E = np.diag(G)
    val = (np.sum(A * E[:, None]) + np.sum(A * E[None, :]) - 2 * np.sum(A * G)) / 2
    dA = 0.5 * (E[:, None] + E[None, :]) - G
    M = np.diag(A.sum(1) + A.sum(0)) - (A + A.T)
    dS_local = (M @ F).reshape(S.shape[0], hi - lo, -1)
    out[rank] = (val, dA, dS_local, lo, hi)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_c5_site_sharding_matches_single_process():
    """TreeOptimizer(group=...)'s decomposition: per-rank site-block Grams,
    one all-reduce (GramReducer), replicated combine, local dS == the
    single-process surrogate value / dA / dS (oracle/tree_ref.py)."""
    from oracle import tree_ref as T

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_c5_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    S, A = _c5_case()
    val, dS, dA = T.compute_surrogate_cost_grads(S, A)
    for r in range(world):
        v, a, ds, lo, hi = out[r]
        np.testing.assert_allclose(v, val, rtol=1e-12)
        np.testing.assert_allclose(a, dA, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(ds, dS[:, lo:hi], rtol=1e-12, atol=1e-12)
