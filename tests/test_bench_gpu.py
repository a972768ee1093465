"""bench.py's N > 1 path, rehearsed on one MI355X.

The driver runs ``torch.distributed.run --nproc-per-node N bench.py --gpus N``
on an 8-GPU node with RCCL; this box has one GPU, so the same command runs
with TREX_BENCH_DEVICE_SHARE=1 (both ranks on cuda:0, gloo instead of RCCL:
the code path, not the timing).  Checked:

* rc 0 and one JSON line from rank 0;
* ``value`` counts the WHOLE batch (every tree of every rank) per step;
* the all-reduced [dC, loss] rank 0 holds after the last step equals the
  single-process engine over the whole batch (the shards' sum).

Fresh child processes via torch.distributed.run; the parent only touches
the GPU after they have exited.
"""

from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from _cases import assert_grad_close

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_world2_device_share_sums_the_whole_batch(tmp_path):
    trees, taxa, sites, states, steps = 64, 32, 1000, 4, 3
    dump = tmp_path / "reduced.npy"
    env = dict(os.environ, TREX_BENCH_DEVICE_SHARE="1", TREX_BENCH_DUMP=str(dump))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", str(steps), "--warmup", "1", "--trees", str(trees),
           "--taxa", str(taxa), "--sites", str(sites), "--states", str(states), "--no-c5"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["trees"] == trees
    assert res["config"]["trees_rank0"] == trees // 2
    units = trees * sites * (taxa - 1) * states
    np.testing.assert_allclose(res["value"], units / (res["ms_per_step"] * 1e-3), rtol=1e-9)

    import torch

    sys.path.insert(0, ROOT)
    import bench

    from trex_amd import SankoffEngine

    dev = torch.device("cuda", 0)
    ch, plan, leaves, cost = bench.make_inputs(torch, dev, trees, taxa, sites, states, 0, trees)
    eng = SankoffEngine(plan, sites, states, dev)
    f, dc, _, _ = eng.fwd_bwd(leaves, cost, 0.5)
    torch.cuda.synchronize()
    red = np.load(dump)
    q2 = states * states
    # two shards' fp64-reduced dC partials summed in fp32: elementwise to
    # fp32 rounding of the sum
    assert_grad_close(red[:q2].reshape(states, states), dc.cpu().numpy(), rtol=1e-6)
    np.testing.assert_allclose(red[q2], float(f.tree_score.double().sum()), rtol=1e-6)


def test_bench_world2_c5_site_shard_matches_single_process():
    """The bench's N > 1 C5 leg (site shard, Gram all-reduce of the ancestor
    rows + mirror, MAX-reduced timer) at a small shape: 128 taxa (255 nodes,
    cached leaf block rows [0, 128)), 510 sites -> 255 per rank, K = 1 020
    (K % 16 = 12, a ragged last x3 chunk).  Rank 0 prints a c5 line with
    n_gpus == 2, and its loss after the run equals bench's own single-process
    C5 leg over all sites (same seeds, same schedule) at rtol 1e-5."""
    taxa, sites, steps, warmup = 128, 510, 4, 2
    env = dict(os.environ, TREX_BENCH_DEVICE_SHARE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--trees", "16", "--taxa", "16",
           "--sites", "256", "--c5-taxa", str(taxa), "--c5-sites", str(sites),
           "--c5-steps", str(steps), "--c5-warmup", str(warmup)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    c5 = json.loads(lines[0])["c5"]
    assert c5["n_gpus"] == 2 and c5["scaling"] == "strong"
    assert c5["taxa"] == taxa and c5["sites"] == sites and c5["sites_rank0"] == sites // 2
    assert c5["gemm"] == "x3"

    import torch

    sys.path.insert(0, ROOT)
    import bench

    single = bench.c5_line(torch, torch.device("cuda", 0), steps=steps, warmup=warmup, nl=taxa,
                           L=sites)
    assert single["n_gpus"] == 1
    np.testing.assert_allclose(c5["loss_last"], single["loss_last"], rtol=1e-5)


def test_bench_rccl_one_rank_rehearsal(tmp_path):
    """bench.py's N > 1 code path with a real RCCL
    process group ("nccl" on ROCm), forced at world 1 (TREX_BENCH_FORCE_DIST)
    because this box has one GPU: init_process_group("nccl", device_id=...),
    the side-stream all-reduce of [dC, loss] overlapped with the next step,
    the barriers and the MAX-reduced timer, then the C5 leg's Gram all-reduce
    (TreeOptimizer(group=WORLD)).  A one-rank all-reduce is the identity, so
    the dumped [dC, loss] equals the engine's own over the same batch bit for
    bit, and the C5 loss equals the single-process leg's."""
    trees, taxa, sites, states, steps = 32, 16, 700, 4, 3
    dump = tmp_path / "reduced.npy"
    env = dict(os.environ, TREX_BENCH_FORCE_DIST="1", TREX_BENCH_DUMP=str(dump))
    env.pop("TREX_BENCH_DEVICE_SHARE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--gpus", "1", "--steps", str(steps), "--warmup", "1", "--trees", str(trees),
           "--taxa", str(taxa), "--sites", str(sites), "--states", str(states),
           "--c5-taxa", "64", "--c5-sites", "300", "--c5-steps", "3", "--c5-warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 1 and res["config"]["process_group"] == "nccl"
    # the self-verifying fields of the driver's N-GPU line
    assert res["config"]["rccl_ranks"] == 1 and res["config"]["world_size"] == 1
    d = res["dist"]
    assert d["rccl_ranks"] == 1 and len(d["ms_per_step_per_rank"]) == 1
    assert d["allreduce_count"] == steps and d["allreduce_us_mean_rank0"] > 0
    assert d["allreduce_bytes"] == (states * states + 1) * 4
    ga = res["c5"]["gram_allreduce"]
    assert ga["ranks"] == 1 and ga["calls_per_step"] == 1 and ga["bytes_per_step"] > 0
    assert "RCCL all-reduce" in res["config"]["workload"]
    assert res["c5"]["scaling"] == "strong" and res["c5"]["n_gpus"] == 1

    import torch

    sys.path.insert(0, ROOT)
    import bench

    from trex_amd import SankoffEngine

    dev = torch.device("cuda", 0)
    ch, plan, leaves, cost = bench.make_inputs(torch, dev, trees, taxa, sites, states, 0, trees)
    eng = SankoffEngine(plan, sites, states, dev)
    f, dc, _, _ = eng.fwd_bwd(leaves, cost, 0.5)
    torch.cuda.synchronize()
    red = np.load(dump)
    q2 = states * states
    np.testing.assert_array_equal(red[:q2].reshape(states, states), dc.cpu().numpy())
    assert red[q2] == np.float32(f.tree_score.sum().item())
    single = bench.c5_line(torch, dev, steps=3, warmup=1, nl=64, L=300)
    np.testing.assert_allclose(res["c5"]["loss_last"], single["loss_last"], rtol=1e-6)
