"""Multi-rank rehearsal on one MI355X: the real sharded code paths, two fresh
processes sharing cuda:0 over gloo (RCCL needs one GPU per rank; the driver's
8-GPU runs use it, this box has one GPU).

* C4 tree-batch sharding: each rank runs the HIP engine on its block of trees
  and the real trex_amd.distributed.GradReducer sums [dC, loss]; equals the
  single-process engine over the whole batch.
* C5 site sharding: the real TreeOptimizer(group=WORLD) -- per-rank Gram,
  GramReducer all-reduce, replicated tree update, local ancestor update --
  with and without clip_by_global_norm (the sharded clip sums the ancestors'
  squared-norm partials over the ranks), vs a single-process TreeOptimizer
  over all sites.
* The C ABI's own RCCL exchange (trex_allreduce_sum) on a one-rank
  communicator.

Workers are spawned (fresh interpreters; the parent process does not touch
the GPU before spawning).
"""

from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)


def _c4_worker(rank, world, port, out):
    dev = _init(rank, world, port)
    from _cases import hamming, random_leaves, random_topologies

    from trex_amd import SankoffEngine, TreePlan
    from trex_amd.distributed import GradReducer, shard_bounds

    B, n, L, Q, tau = 16, 24, 1500, 4, 0.5
    ch = random_topologies(B, n, seed=41)
    lv = torch.as_tensor(random_leaves(B, n, L, Q, seed=42), device=dev)
    c = torch.as_tensor(hamming(Q), device=dev)
    full = SankoffEngine(TreePlan(ch), L, Q, dev)
    ff, dc_full, _, _ = full.fwd_bwd(lv, c, tau)
    lo, hi = shard_bounds(B, rank, world)
    eng = SankoffEngine(TreePlan(ch[lo:hi]), L, Q, dev)
    f, dc, _, _ = eng.fwd_bwd(lv[lo:hi].contiguous(), c, tau)
    gdc, gloss = GradReducer(Q, dev)(dc, f.tree_score)
    torch.cuda.synchronize()
    out[rank] = (gdc.cpu().numpy().copy(), float(gloss), dc_full.cpu().numpy(),
                 float(ff.tree_score.sum()))
    dist.barrier()
    dist.destroy_process_group()


def test_c4_tree_sharding_world2_on_one_gpu():
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_c4_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        gdc, gloss, dc_full, loss_full = out[r]
        # the shards' fp64 partials are summed in a different association
        # than the single-process reduce: elementwise to fp32 rounding
        from _cases import assert_grad_close

        assert_grad_close(gdc, dc_full, rtol=1e-6)
        np.testing.assert_allclose(gloss, loss_full, rtol=1e-6)
    assert np.array_equal(out[0][0], out[1][0])


def _c5_case(nl=32, L=512, Q=4, seed=3):
    rng = np.random.default_rng(seed)
    n = 2 * nl - 1
    S = np.zeros((n, L, Q), np.float32)
    S[:nl] = np.eye(Q, dtype=np.float32)[rng.integers(0, Q, size=(nl, L))]
    params = {"tree_params": rng.normal(size=(n - 1, nl - 1)).astype(np.float32),
              "ancestors": rng.normal(size=(nl - 1, L, Q)).astype(np.float32)}
    noise = rng.gumbel(size=(n - 1, nl - 1)).astype(np.float32)
    return S, params, noise


def _c5_worker(rank, world, port, clip, L, nl, out):
    dev = _init(rank, world, port)
    from trex_amd.distributed import shard_bounds
    from trex_amd.tree import TreeOptimizer

    S, params, noise = _c5_case(nl=nl, L=L)
    L = S.shape[1]
    lo, hi = shard_bounds(L, rank, world)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)  # noqa: E731
    nz = t(noise)
    single = TreeOptimizer(t(S), {k: t(v) for k, v in params.items()}, lr=0.01, clip_norm=clip)
    shard = TreeOptimizer(t(S[:, lo:hi]), {"tree_params": t(params["tree_params"]),
                                           "ancestors": t(params["ancestors"][:, lo:hi])},
                          lr=0.01, clip_norm=clip, group=dist.group.WORLD)
    # the split-product GEMMs on every shard, ragged K included (no silent f32)
    assert single.gemm == "x3" and shard.gemm == "x3", (single.gemm, shard.gemm)
    temps = [2.0, 1.5, 1.2, 1.0]
    l1, l2 = [], []
    gerr = 0.0
    for i, T_ in enumerate(temps):
        nxt = temps[i + 1] if i + 1 < len(temps) else T_
        l1.append(float(single.step(T_, nz, next_temperature=nxt)))
        l2.append(float(shard.step(T_, nz, next_temperature=nxt)))
        if i == 0:
            # same parameters before the first step: the sharded Gram (cached
            # leaf x leaf block, reduced ancestor rows, mirrored leaf rows'
            # ancestor columns) == the single-process Gram elementwise
            g1 = single.G.cpu().numpy().astype(np.float64)
            g2 = shard.G.cpu().numpy().astype(np.float64)
            gerr = float((np.abs(g2 - g1) / np.maximum(np.abs(g1), 1e-30)).max())
    torch.cuda.synchronize()
    assert shard.g_row0 == (nl // 64) * 64
    out[rank] = (np.array(l1), np.array(l2),
                 single.params["tree_params"].cpu().numpy(),
                 shard.params["tree_params"].cpu().numpy(),
                 single.params["ancestors"][:, lo:hi].cpu().numpy(),
                 shard.params["ancestors"].cpu().numpy(), gerr)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("clip,L,nl", [(None, 512, 32), (1.0, 512, 32), (None, 510, 32),
                                       (None, 510, 100), (1.0, 256, 100)])
def test_c5_site_sharding_world2_on_one_gpu(clip, L, nl):
    """L = 510: each rank holds 255 sites, K = 1 020 (K % 16 = 12, like the
    C5 shard at N = 8, K = 25 000): the x3 GEMMs run on the ragged K and the
    cached leaf x leaf Gram survives sharding (only the ancestor rows are
    all-reduced per step, then mirrored).  nl = 100 (N = 199): the cached
    leaf block ends at row 64 < n_leaf, so the per-step reduce covers rows
    [64, 199) and the mirror rewrites the leaf rows' ancestor columns; the
    first step's Gram is checked elementwise against the single process."""
    world = 2
    out = mp.Manager().dict()
    mp.spawn(_c5_worker, args=(world, _free_port(), clip, L, nl, out), nprocs=world, join=True)
    for r in range(world):
        l1, l2, tp1, tp2, an1, an2, gerr = out[r]
        assert gerr <= 1e-5, gerr
        np.testing.assert_allclose(l2, l1, rtol=1e-5)
        # Gram partial sums differ in association from the single-process
        # Gram only at fp32 rounding; Adam's ~sign(g) first steps can turn a
        # rounding-level gradient into a 2 lr difference: allow 0.1 % of them
        for a, b in ((tp2, tp1), (an2, an1)):
            close = np.isclose(a, b, rtol=1e-4, atol=1e-5)
            assert close.mean() > 0.999, close.mean()
    # the replicated tree update is bitwise identical on every rank
    assert np.array_equal(out[0][3], out[1][3])


def test_native_rccl_allreduce_one_rank(device):
    """trex_comm_* / trex_allreduce_sum (include/trex_hip.h) on a one-rank
    communicator: the sum over one rank is the identity, on torch's stream."""
    from trex_amd.distributed import NativeComm

    uid = NativeComm.new_unique_id()
    assert len(uid) == 128
    comm = NativeComm(1, 0, uid, device.index or 0)
    x = torch.arange(4 * 4 + 1, dtype=torch.float32, device=device)
    y = x.clone()
    comm.all_reduce_sum(y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    comm.close()
