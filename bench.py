#!/usr/bin/env python
"""Benchmark: batched Sankoff forward + gradient on MI355X (BASELINE.json metric).

One step = softmin Sankoff forward (writes the DP table, as trex's run_sankoff
returns it) + adjoint sweep (d score / d cost) over this rank's shard of the
C4 workload (BASELINE.json configs[3]: 1024 random 32-taxa topologies x 5000
sites x 4 states, tau = 0.5), then an RCCL all-reduce of [d_cost, loss] when
N > 1.  Strong scaling: the N ranks split C4's 1024 trees (--trees) in
contiguous blocks, so N = 1 runs the whole batch and N = 8 runs 128 trees per
rank.  Metric: site-node-state updates/s = B*L*n_int*Q per step over all
ranks.

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--trees", type=int, default=1024,
                    help="C4 batch size, split over the ranks (strong scaling)")
    ap.add_argument("--taxa", type=int, default=32)
    ap.add_argument("--sites", type=int, default=5000)
    ap.add_argument("--states", type=int, default=4)
    ap.add_argument("--tau", type=float, default=0.5)
    ap.add_argument("--no-graph", action="store_true", help="launch eagerly, no hipGraph")
    ap.add_argument("--no-settle", action="store_true",
                    help="skip the clock-settle steps before the warmup (cold-start timing)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 single-tree line")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 protein line")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 tree-cost loop line")
    ap.add_argument("--no-nk", action="store_true", help="skip the NK landscape-aware line")
    ap.add_argument("--no-ragged", action="store_true", help="skip the ragged-batch line")
    ap.add_argument("--no-shard", action="store_true", help="skip the 128-tree shard line")
    ap.add_argument("--no-e2e", action="store_true", help="skip the H2D-inclusive C4 line")
    ap.add_argument("--c5-taxa", type=int, default=256, help="C5 leaves (nodes = 2 taxa - 1)")
    ap.add_argument("--c5-sites", type=int, default=50000,
                    help="C5 sites (split over the ranks at N > 1)")
    ap.add_argument("--c5-steps", type=int, default=20)
    ap.add_argument("--c5-warmup", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (written by profiles/pmc_traffic.py)")
    return ap.parse_args()


def make_inputs(torch, device, n_trees, n, L, Q, lo, hi):
    """Trees [lo, hi) of the C4 batch (random coalescent
    topologies, seed 4; iid uniform leaf states, seed 5): the same global
    batch for every rank count, so N ranks split exactly C4's work."""
    from trex_amd import TreePlan, random_topologies

    ch = random_topologies(n_trees, n, seed=4)[lo:hi]
    plan = TreePlan(ch)
    g = torch.Generator(device=device)
    g.manual_seed(5)
    leaves = torch.randint(0, Q, (n_trees, n, L), generator=g, device=device,
                           dtype=torch.int8)[lo:hi].contiguous()
    cost = (torch.ones(Q, Q) - torch.eye(Q)).to(device=device, dtype=torch.float32)
    return ch, plan, leaves, cost


def host_cpu():
    """The host's CPU model and the cores this job may use: the affinity
    mask, capped by a cgroup CPU quota and by OMP_NUM_THREADS when the
    environment sets it (the GPU box's per-GPU CPU share)."""
    info = {"model": None, "cpus_online": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                info["cgroup_quota_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    use = info["affinity_cpus"]
    if info["cgroup_quota_cpus"]:
        use = min(use, max(1, int(info["cgroup_quota_cpus"])))
    if info["omp_num_threads"] and info["omp_num_threads"].isdigit():
        use = min(use, int(info["omp_num_threads"]))
    info["threads_used"] = use
    return info, use


class Step:
    """fused fwd + adjoint into preallocated buffers (capturable)."""

    def __init__(self, torch, eng, leaves, cost, tau):
        self.eng, self.leaves, self.cost, self.tau = eng, leaves, cost, tau
        dev = eng.device
        self.out_f = {
            "dp": torch.empty(eng.dp_shape, dtype=torch.float32, device=dev),
            "tree_score": torch.empty((eng.plan.B,), dtype=torch.float32, device=dev),
        }
        self.out_b = {"d_cost": torch.empty((eng.Q, eng.Q), dtype=torch.float32, device=dev)}
        self.out_fb = dict(self.out_f, **self.out_b)

    def fused(self):
        return self.eng.fwd_bwd(self.leaves, self.cost, self.tau, out=self.out_fb)

    def fwd(self):
        return self.eng.forward(self.leaves, self.cost, self.tau, dp=True, out=self.out_f)

    def bwd(self):
        return self.eng.backward(self.leaves, self.cost, self.tau, self.out_f["dp"],
                                 out=self.out_b)

    def __call__(self):
        self.fused()


def time_kernels(torch, step, iters=20):
    """Average device time per launch of the fused kernel and, for reference,
    of the separate fwd / adjoint kernels (HIP events on the stream they run
    on: torch's current stream)."""
    out = {}
    for name, fn in (("sankoff_fwd_bwd", step.fused), ("sankoff_fwd", step.fwd),
                     ("sankoff_bwd", step.bwd)):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters)]
        for e0, e1 in ev:
            e0.record()
            fn()
            e1.record()
        torch.cuda.synchronize()
        out[name] = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev])) * 1e-3
    return out


def shard_line(torch, device, ch, leaves, cost, tau, L, Q, n, Bs):
    """The slice of C4 each rank runs at N = 8 (128 trees), alone on one GPU:
    fused fwd + grad (hipGraph replay) and the fused kernel's event time."""
    from trex_amd import SankoffEngine, TreePlan

    eng = SankoffEngine(TreePlan(ch[:Bs]), L, Q, device)
    st = Step(torch, eng, leaves[:Bs].contiguous(), cost, tau)
    sec = _replay_seconds(torch, st, 200)
    kt = time_kernels(torch, st)["sankoff_fwd_bwd"]
    fb = Bs * L * (2 * n + 8 * Q * (n - 1))
    return {"workload": f"C4 / 8: {Bs} trees x {L} sites x {n} taxa x {Q} states, softmin "
                        f"tau={tau} fwd + grad (one rank's share at N = 8), hipGraph replay",
            "ms_per_step": sec * 1e3, "value": Bs * L * (n - 1) * Q / sec,
            "fused_kernel_us": round(kt * 1e6, 2), "algorithmic_bytes": fb,
            "hbm_frac": round(fb / kt / 1e9 / HBM_PEAK_GBS, 4)}


def e2e_line(torch, run_step, leaves, units, reps=10, make_step=None):
    """C4 end to end (SURVEY 8(d) "kernel-only and end-to-end incl. H2D of
    leaves"): each step first uploads the int8 leaves from host memory into
    the device buffer the step reads, then runs the fused fwd + grad --
    from pageable memory (a plain numpy array) and from pinned memory."""
    host = leaves.cpu()
    pinned = host.pin_memory()
    nbytes = leaves.numel() * leaves.element_size()
    out = {"workload": "C4 as the headline line, leaves uploaded from host memory every step",
           "leaf_bytes": nbytes}
    for name, src in (("pageable", host), ("pinned", pinned)):
        leaves.copy_(src, non_blocking=True)
        run_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            leaves.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        h2d = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            leaves.copy_(src, non_blocking=True)
            run_step()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / reps
        out[name] = {"ms_per_step_incl_h2d": sec * 1e3, "h2d_ms": h2d * 1e3,
                     "h2d_GBs": round(nbytes / h2d / 1e9, 1), "value": units / sec}
    if make_step is not None:
        # a stream of batches: batch k + 1's leaves upload (pinned, on a copy
        # stream) into the other of two device buffers while batch k computes
        dev = leaves.device
        bufs = [leaves, torch.empty_like(leaves)]
        steps = [make_step(b) for b in bufs]
        copy = torch.cuda.Stream(dev)
        comp = torch.cuda.current_stream(dev)
        up = [torch.cuda.Event(), torch.cuda.Event()]
        done = [torch.cuda.Event(), torch.cuda.Event()]

        def run(n):
            with torch.cuda.stream(copy):
                bufs[0].copy_(pinned, non_blocking=True)
                up[0].record(copy)
            for k in range(n):
                c, nx = k % 2, (k + 1) % 2
                if k + 1 < n:
                    if k >= 1:  # buffer nx was read by batch k - 1
                        copy.wait_event(done[nx])
                    with torch.cuda.stream(copy):
                        bufs[nx].copy_(pinned, non_blocking=True)
                        up[nx].record(copy)
                comp.wait_event(up[c])
                steps[c]()
                done[c].record(comp)
            torch.cuda.synchronize()

        run(3)
        t0 = time.perf_counter()
        run(reps)
        sec = (time.perf_counter() - t0) / reps
        out["pinned_overlapped"] = {
            "ms_per_step_incl_h2d": sec * 1e3, "value": units / sec,
            "note": "double-buffered: upload of batch k+1 on a copy stream overlaps batch k's "
                    "fused kernel; bound by PCIe (h2d_ms above)"}
    return out


def c2_line(torch, device, args, cpu_threads):
    """C2 (BASELINE.json configs[1]): one balanced 64-taxa tree x 10k sites x
    4 states, softmin fwd+grad (tau 1.0), leaves simulated along the tree."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cases import simulate_leaves

    from trex_amd import SankoffEngine, TreePlan, children_from_adjacency

    seqs, adj = simulate_leaves(64, 10000, 4, 5, seed=1)
    ch = children_from_adjacency(adj)
    eng = SankoffEngine(TreePlan(ch), 10000, 4, device)
    leaves = torch.from_numpy(np.ascontiguousarray(seqs[None, :64])).to(device)
    cost = (torch.ones(4, 4) - torch.eye(4)).to(device=device, dtype=torch.float32)
    step = Step(torch, eng, leaves, cost, 1.0)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    # one step is ~25 us of GPU work, below a graph launch's host cost: the
    # graph holds 10 consecutive steps (each a full fwd + grad), so the
    # replay rate measures the GPU, not the launch path
    per_graph = 10
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            step()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    n = 100
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / (n * per_graph)
    # one-step graph replays, launch cost included (what a caller replaying
    # a single step sees)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        step()
    for _ in range(10):
        g1.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500):
        g1.replay()
    torch.cuda.synchronize()
    single_s = (time.perf_counter() - t0) / 500
    units = 10000 * 63 * 4
    # trex-exact reconstruction of the same tree (run_sankoff(return_path=True)
    # on the device: hard forward writing the DP table + backtrack)
    rout = {"dp": torch.empty(eng.dp_shape, dtype=torch.float32, device=device),
            "tree_score": torch.empty(1, device=device)}

    def recon():
        r = eng.forward(leaves, cost, 0.0, out=rout)
        eng.backtrack(cost, r.dp)

    recon_s = _replay_seconds(torch, recon, 200)
    out = {"workload": "C2: balanced 64-taxa tree x 10000 sites x 4 states, softmin tau=1.0 "
                       "fwd+grad, hipGraph of 10 steps replayed", "ms_per_step": gpu_s * 1e3,
           "value": units / gpu_s, "ms_per_single_step_graph_replay": single_s * 1e3,
           "hard_recon_ms_per_step": recon_s * 1e3}
    from oracle.cpu_port import fwd_bwd

    fwd_bwd(ch, seqs[None, :64], cost.cpu().numpy(), 1.0, threads=cpu_threads)
    reps = []
    for _ in range(5):
        t0 = time.perf_counter()
        fwd_bwd(ch, seqs[None, :64], cost.cpu().numpy(), 1.0, threads=cpu_threads)
        reps.append(time.perf_counter() - t0)
    cpu_s = float(np.median(reps))
    out["cpu_port_ms"] = cpu_s * 1e3
    out["cpu_port_threads"] = cpu_threads
    out["speedup_vs_cpu_port"] = cpu_s / gpu_s
    # trex-structure numpy proxy at the full C2 size: run_sankoff's layout
    # (dp + bt tables, vectorised over sites, serial over nodes), hard
    # forward only (trex's run_sankoff has no gradient of its own)
    from oracle.sankoff_ref import run_sankoff_ref

    t0 = time.perf_counter()
    run_sankoff_ref(adj, (np.ones((4, 4)) - np.eye(4)).astype(np.float32),
                    seqs[:64].astype(np.float32), 127, 4, 64)
    px = time.perf_counter() - t0
    out["trex_numpy_proxy"] = {"ms": px * 1e3, "value": units / px, "cores": 1,
                               "sample": "full C2 (1 tree x 10000 sites x 64 taxa), hard "
                                         "forward only, oracle/sankoff_ref.run_sankoff_ref"}
    return out


def _replay_seconds(torch, fn, n):
    """Capture fn in a hipGraph, return mean wall seconds per replay."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def c3_line(torch, device, cpu_threads):
    """C3 (BASELINE.json configs[2]): balanced 64-taxa tree x 10 000 sites x
    20 states (protein), C symmetric integer {1..4} off-diagonal (seed 3).
    Two steps: (a) softmin tau=0.5 fwd + grad + marginals + soft ancestral
    states in one fused launch; (b) trex-exact ancestral reconstruction
    (hard forward + backtrack, run_sankoff(return_path=True))."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _cases import int_cost, simulate_leaves

    from trex_amd import SankoffEngine, TreePlan, children_from_adjacency

    nl, L, Q, tau = 64, 10000, 20, 0.5
    n_int = nl - 1
    seqs, adj = simulate_leaves(nl, L, Q, 50, seed=2)
    ch = children_from_adjacency(adj)
    eng = SankoffEngine(TreePlan(ch), L, Q, device)
    leaves = torch.from_numpy(np.ascontiguousarray(seqs[None, :nl])).to(device)
    cost_np = int_cost(Q, seed=3)
    cost = torch.from_numpy(cost_np).to(device)
    f = torch.empty(eng.dp_shape, dtype=torch.float32, device=device)
    out = {"dp": f, "tree_score": torch.empty(1, device=device),
           "d_cost": torch.empty((Q, Q), device=device),
           "marginals": torch.empty_like(f),
           "anc_states": torch.empty((1, n_int, L), dtype=torch.int8, device=device)}

    def soft():
        eng.fwd_bwd(leaves, cost, tau, marginals=True, anc_states=True, out=out)

    def hard():
        r = eng.forward(leaves, cost, 0.0, out=out)
        eng.backtrack(cost, r.dp)

    soft_s = _replay_seconds(torch, soft, 200)
    hard_s = _replay_seconds(torch, hard, 200)
    # device time of the fused kernel alone (HIP events on torch's stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for e0, e1 in ev:
        e0.record()
        soft()
        e1.record()
    torch.cuda.synchronize()
    k_s = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev])) * 1e-3
    units = L * n_int * Q
    # algorithmic bytes (SURVEY.md 8(d) fwd+grad + C3 extras): leaves in twice,
    # DP table out + adjoint re-read, marginals out (f32), anc states out (i8)
    abytes = L * (2 * nl + 8 * Q * n_int + 4 * Q * n_int + n_int)
    res = {"workload": "C3: balanced 64-taxa tree x 10000 sites x 20 states, softmin tau=0.5 "
                       "fwd+grad+marginals+soft ancestral (fused) | hard fwd + trex backtrack",
           "soft_ms_per_step": soft_s * 1e3, "soft_value": units / soft_s,
           "hard_recon_ms_per_step": hard_s * 1e3, "hard_recon_value": units / hard_s,
           "unit": "site-node-state updates/s",
           "roofline": {"bound": "hbm", "kernel": "site_prep + sankoff_site_kernel<3,20> + reduce (lane-per-site, DESIGN 5.8)",
                        "achieved": round(abytes / k_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(abytes / k_s / 1e9 / HBM_PEAK_GBS, 4),
                        "algorithmic_bytes": abytes, "launch_us": round(k_s * 1e6, 2)}}
    from oracle.cpu_port import fwd_bwd

    fwd_bwd(ch, seqs[None, :nl], cost_np, tau, threads=cpu_threads)
    reps = []
    for _ in range(3):
        t0 = time.perf_counter()
        fwd_bwd(ch, seqs[None, :nl], cost_np, tau, threads=cpu_threads)
        reps.append(time.perf_counter() - t0)
    cpu_s = float(np.median(reps))
    res["cpu_port_ms"] = cpu_s * 1e3
    res["speedup_vs_cpu_port"] = cpu_s / soft_s
    return res


MFMA_F16_DENSE_TFS = 2500.0  # MI355X dense f16/bf16 MFMA peak (MI355X_MICROARCH.md)
MFMA_F32_TFS = 157.0         # MI355X f32 matrix peak


def c5_gemm_kernels(torch, opt):
    """HIP-event time of the step's two GEMM launches on the optimiser's own
    buffers, with their algorithmic HBM bytes and (f16x3) the MFMA flops the
    tile plan issues -- executed work, not a trex-equivalent rate."""
    from trex_amd._lib import lib, stream_handle

    L_ = lib()
    st = stream_handle(opt.S.device)
    cs = torch.cuda.current_stream(opt.S.device)
    N, K, nl, na = opt.N, opt.K, opt.n_leaf, opt.n_anc
    # the step's own GEMM launches (pre-split operands on the x3 path, leaf
    # rows read as codes where the optimiser does)
    gram = lambda: opt._gram(st)  # noqa: E731
    mf = lambda: opt._mf(st)  # noqa: E731

    def timed(fn, reps=20):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for _ in range(reps):
            fn()
        e1.record(cs)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    out = {}
    nt, sk = (N + 31) // 32, opt.skip_rows // 32
    tiles = nt * (nt + 1) // 2 - sk * (sk + 1) // 2
    # MF operand bytes: the code rows as one byte per site (leaf codes) or f32 rows
    lcr = int(L_.trex_tree_leaf_code_rows(nl)) if opt.codes is not None else 0
    s_mf = (N - lcr) * K * 4 + lcr * (K // opt.Q)
    # f16x3 products issued per 32x32 tile-step: 3 (hi*hi + hi*lo + lo*hi),
    # 2 where one operand is an exact one-hot leaf row (zero lo plane: the
    # Gram's leaf strips when the codes declare them, the MF's code stages)
    lzs = lcr // 32
    g_leaf = (sum(nt - max(a, sk) for a in range(min(lzs, nt)))
              if (opt.codes is not None and getattr(opt, "presplit", False)) else 0)
    g_prod = (2 * g_leaf + 3 * (tiles - g_leaf)) / tiles if tiles else 3
    m_prod = (2 * lzs + 3 * (nt - lzs)) / nt
    # the Gram reads whole 128-row passes of code rows as bytes (pre-split path)
    gcr = (lcr // 128) * 128 if getattr(opt, "presplit", False) else 0
    s_gram = (N - gcr) * K * 4 + gcr * (K // opt.Q)
    for name, fn, abytes, flops, prod in (
            ("gram", gram, s_gram + N * N * 4, tiles * 32 * 32 * K * 2, g_prod),
            ("mf", mf, s_mf + N * N * 4 + na * K * 4, ((na + 31) // 32 * 32) * nt * 32 * K * 2,
             m_prod)):
        sec = timed(fn)
        d = {"us": round(sec * 1e6, 2), "algorithmic_bytes": abytes,
             "GBs": round(abytes / sec / 1e9, 1), "hbm_frac": round(abytes / sec / 1e9 / HBM_PEAK_GBS, 4)}
        if opt.gemm == "x3":
            issued = int(round(prod * flops))  # f16 MFMA flops actually issued
            d.update(mfma_flops_issued=issued,
                     mfma_tflops=round(issued / sec / 1e12, 1),
                     mfma_frac=round(issued / sec / 1e12 / MFMA_F16_DENSE_TFS, 4),
                     mfma_peak_tflops=MFMA_F16_DENSE_TFS)
        else:
            d.update(mfma_flops_issued=flops, mfma_tflops=round(flops / sec / 1e12, 1),
                     mfma_frac=round(flops / sec / 1e12 / MFMA_F32_TFS, 4),
                     mfma_peak_tflops=MFMA_F32_TFS)
        out[name] = d
    return out


def c5_line(torch, device, steps=20, warmup=3, rank=0, world=1, gemm="x3", nl=256, L=50000,
            dist_on=False):
    """C5 (BASELINE.json configs[4]): 256 taxa (511 nodes) x 50 000 sites x 4
    states, joint Adam optimisation step (update_seq, update_tree, surrogate
    + graph constraint, their VJPs, optax Adam) -- trex's
    tests/test_convergence.py:208-261 loop at C5 size.  With N > 1 ranks the
    sites shard: one all-reduce of the 511 x 511 Gram per step
    (strong scaling: the 50 000 sites are split).  Eager launches (Adam's bias
    correction changes every step)."""
    from trex_amd._lib import lib
    from trex_amd.datagen import generate_groundtruth
    from trex_amd.distributed import shard_bounds
    from trex_amd.tree import TreeOptimizer, gumbel_noise

    Q = 4
    n = 2 * nl - 1
    lo, hi = shard_bounds(L, rank, world)
    seqs = generate_groundtruth(nl, Q, 5, L, seed=6).all_sequences.astype(np.int8)
    S = torch.zeros((n, hi - lo, Q), dtype=torch.float32, device=device)
    S[:nl] = torch.nn.functional.one_hot(
        torch.as_tensor(seqs[:nl, lo:hi].astype(np.int64), device=device), Q).float()
    g = torch.Generator(device=device)
    g.manual_seed(7)  # identical on every rank: replicated tree params and noise
    params = {"tree_params": torch.randn((n - 1, nl - 1), generator=g, device=device),
              "ancestors": torch.randn((nl - 1, L, Q), generator=g, device=device)[:, lo:hi]
              .contiguous()}
    noise = [gumbel_noise((n - 1, nl - 1), generator=g, device=device) for _ in range(4)]
    group = None
    dist_on = dist_on or world > 1
    if dist_on:
        import torch.distributed as dist

        group = dist.group.WORLD
    opt = TreeOptimizer(S, params, lr=0.01, group=group, gemm=gemm)
    def temp(k):  # the annealing schedule of tests/test_convergence.py:260
        return max(0.1, 2.0 * (1.0 - k / 5000))

    for k in range(warmup):
        opt.step(temp(k), noise[k % 4], next_temperature=temp(k + 1))
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    red0 = (opt.reducer.calls, opt.reducer.bytes) if opt.reducer is not None else (0, 0)
    t0 = time.perf_counter()
    for k in range(steps):
        loss = opt.step(temp(warmup + k), noise[k % 4], next_temperature=temp(warmup + k + 1))
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    gram_ar = None
    if opt.reducer is not None:
        # the Gram exchange of one timed step (GramReducer's own count)
        gram_ar = {"calls_per_step": (opt.reducer.calls - red0[0]) / steps,
                   "bytes_per_step": (opt.reducer.bytes - red0[1]) // steps,
                   "ranks": dist.get_world_size(group)}
    if dist_on:
        t = torch.tensor([sec], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        sec = float(t.item())
    # algorithmic HBM bytes of one step (the step is HBM-bound overall): the
    # Gram reads S once, the MF reads S and writes the ancestor rows of dS,
    # the fused update_seq-VJP + Adam pass reads dS and the ancestors' logits
    # / moments, writes logits / moments and the next step's S rows
    Kl = (hi - lo) * Q
    na = nl - 1
    lcr = int(lib().trex_tree_leaf_code_rows(nl)) if opt.codes is not None else 0
    step_bytes = n * Kl * 4 + ((n - lcr) * Kl * 4 + lcr * (hi - lo) + na * Kl * 4) + na * Kl * 4 * 8
    gemm_desc = ("f16x3 split-product MFMA GEMMs (f32 accumulate; rtol 1e-5 vs fp64 at this "
                 "size, tests/test_configs_full_gpu.py)" if opt.gemm == "x3" else "f32 MFMA GEMMs")
    res = {"workload": f"C5: {n}-node relaxed tree x {L} sites x {Q} states, joint Adam step "
                       "(surrogate + constraint + VJPs + optax adam), " + gemm_desc
                       + (f"; sites sharded over {world} ranks, Gram all-reduce" if dist_on
                          else ""),
           "ms_per_step": sec * 1e3, "steps_per_s": 1.0 / sec, "n_gpus": world,
           "taxa": nl, "sites": L, "sites_rank0": hi - lo if rank == 0 else None,
           "scaling": "strong" if dist_on else None, "loss_last": float(loss),
           "gemm": opt.gemm, "leaf_codes": opt.codes is not None,
           "gram_allreduce": gram_ar,
           "roofline": {"bound": "hbm", "algorithmic_bytes_per_step": step_bytes,
                        "achieved": round(step_bytes / sec / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(step_bytes / sec / 1e9 / HBM_PEAK_GBS, 4)}}
    if world == 1:
        res["kernels"] = c5_gemm_kernels(torch, opt)
    return res


def ragged_line(torch, device, steps=20, warmup=3):
    """a ragged C4-like batch -- 128 random topologies
    with 8..64 taxa and 1 000..5 000 sites each, softmin tau=0.5 fwd + grad in
    one launch (trex pads such a batch to MAX_NODES / N buckets,
    padding.py:25-27)."""
    from trex_amd import random_topologies
    from trex_amd.ragged import RaggedSankoffEngine, RaggedTreePlan

    rng = np.random.default_rng(12)
    B, Q = 128, 4
    taxa = rng.integers(8, 65, size=B)
    Ls = rng.integers(1000, 5001, size=B)
    chs = [random_topologies(1, int(n), seed=1000 + b)[0] for b, n in enumerate(taxa)]
    plan = RaggedTreePlan(chs, Ls)
    leaves = [rng.integers(0, Q, size=(int(n), int(L))).astype(np.int8) for n, L in zip(taxa, Ls)]
    eng = RaggedSankoffEngine(plan, Q, device)
    lv = torch.as_tensor(plan.pack_leaves(leaves), device=device)
    cost = torch.as_tensor((np.ones((Q, Q)) - np.eye(Q)).astype(np.float32), device=device)
    for _ in range(warmup):
        eng.value_and_grad(lv, cost, 0.5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.value_and_grad(lv, cost, 0.5)
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    units = plan.row_sites * Q
    return {"workload": f"ragged batch: {B} random topologies, 8..64 taxa, 1000..5000 sites, "
                        f"{Q} states, softmin tau=0.5 fwd+grad in one launch (eager)",
            "ms_per_step": sec * 1e3, "value": units / sec, "unit": "site-node-state updates/s"}


def nk_line(torch, device, steps=50, warmup=5):
    """the NK landscape-aware objective
    (src/trex/evals/benchmark.py:235-306, 586-663) -- one Adam step of
    run_trex_landscape_aware_configurable (loss + grad + optax adam), at the
    reference's eval shape (benchmark.py:981-985: 32 leaves, N = 15 sites,
    binary states, K = 10, lambda = 3) and at a larger DNA shape."""
    from trex_amd import nk as NK
    from trex_amd.datagen import create_nk_model_landscape

    out = {}
    for name, (nl, L, Q, k, lam) in {"eval_32x15_q2_k10": (32, 15, 2, 10, 3.0),
                                     "dna_256x2000_q4_k4": (256, 2000, 4, 4, 1.0)}.items():
        n_all = 2 * nl - 1
        rng = np.random.default_rng(8)
        land_np = create_nk_model_landscape(L, k, seed=9, n_states=Q)
        inter, F = land_np["interactions"], land_np["fitness_tables"]
        A = np.zeros((n_all, n_all), np.float32)
        A[np.arange(n_all - 1), nl + np.arange(n_all - 1) // 2] = 1.0
        land = NK.NKLandscape(inter, F, Q, device)
        S0 = NK.masked_sequences_from_leaves(rng.integers(0, Q, size=(nl, L)), n_all, Q, device)
        fn = NK.LandscapeAwareLoss(A, nl, land, lam, k)
        # run_trex_landscape_aware_configurable's Adam step: loss + dS, then
        # the update_seq VJP, Adam and the next update_seq in one pass
        opt = NK.LandscapeAwareAdam(fn, rng.normal(size=(nl - 1, L, Q)).astype(np.float32), S0,
                                    1e-3)

        def step():
            opt.step()

        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / steps
        # the same step captured once in a hipGraph (the Adam step count lives
        # on the device, trex_step_advance) and replayed: the reference's
        # fori_loop body without per-step host launches
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        for _ in range(warmup):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        gsec = (time.perf_counter() - t0) / steps
        out[name] = {"workload": f"{nl} leaves x {L} sites x {Q} states, K={k}, lambda={lam}: "
                                 "landscape-aware loss + grad + adam step",
                     "ms_per_step": gsec * 1e3, "ms_per_step_eager": sec * 1e3,
                     "timing": "hipGraph replay of one captured step (eager launches beside it)",
                     "logit_macs_per_step": 2 * fn.n_parents * L * Q ** (k + 1)}
    return out


def cpu_baseline(ch, leaves_np, cost_np, tau, L, n, Q, threads):
    """OpenMP C restatement (oracle/cpu_port.c) on this host's cores, on a
    bounded sample of the same workload; plus the trex-structure numpy proxy."""
    from oracle.cpu_port import fwd_bwd

    nb = len(ch)
    fwd_bwd(ch[:2], leaves_np[:2], cost_np, tau, threads=threads)  # warm
    reps = []
    t_end = time.perf_counter() + 20.0
    while len(reps) < 5 and (not reps or time.perf_counter() < t_end):
        t0 = time.perf_counter()
        fwd_bwd(ch, leaves_np, cost_np, tau, threads=threads)
        reps.append(time.perf_counter() - t0)
    sec = float(np.median(reps))
    units = nb * L * (n - 1) * Q
    base = {"value": units / sec, "unit": "site-node-state updates/s", "cores": threads,
            "kind": "port",
            "sample": f"{nb} trees x {L} sites x {n} taxa x {Q} states softmin fwd+grad "
                      f"(oracle/cpu_port.c, OpenMP, median of {len(reps)})"}
    return base


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("launch N>1 with torch.distributed.run (one process per GPU)")
    # TREX_BENCH_DEVICE_SHARE=1 rehearses N ranks on one GPU over gloo (code
    # path check only; timings are not meaningful); the driver's runs use RCCL
    share = os.environ.get("TREX_BENCH_DEVICE_SHARE") == "1"
    # TREX_BENCH_FORCE_DIST=1 runs the N > 1 code path at N = 1 (RCCL
    # process group, side-stream all-reduce, MAX timer): a one-GPU rehearsal
    # of the backend the driver's 8-GPU run initialises
    dist_on = world > 1 or os.environ.get("TREX_BENCH_FORCE_DIST") == "1"
    device = torch.device("cuda", 0 if share else local)
    torch.cuda.set_device(device)
    if dist_on:
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
        # the group really spans N ranks: an all-reduce of ones on it (with
        # RCCL, on the device) must come back as N, the launcher's WORLD_SIZE
        ones = torch.ones(1, dtype=torch.float32, device=device)
        dist.all_reduce(ones)
        torch.cuda.synchronize()
        rccl_ranks = int(round(float(ones.item())))
        if rccl_ranks != world or dist.get_world_size() != world:
            raise SystemExit(f"process group spans {rccl_ranks} ranks (get_world_size "
                             f"{dist.get_world_size()}), WORLD_SIZE says {world}")

    from trex_amd import SankoffEngine
    from trex_amd.distributed import shard_bounds

    n, L, Q, tau = args.taxa, args.sites, args.states, args.tau
    lo, hi = shard_bounds(args.trees, rank, world)
    B = hi - lo
    ch, plan, leaves, cost = make_inputs(torch, device, args.trees, n, L, Q, lo, hi)
    eng = SankoffEngine(plan, L, Q, device)
    step = Step(torch, eng, leaves, cost, tau)
    red = torch.zeros(Q * Q + 1, dtype=torch.float32, device=device)

    # N > 1: the step's [dC, loss] all-reduce runs on a side stream and
    # overlaps the next step's kernel (double-buffered, as DDP overlaps its
    # gradient buckets with backward); every all-reduce completes inside the
    # timed region (synchronize at the end waits for both streams)
    comm = torch.cuda.Stream(device) if dist_on else None
    reds = [red, torch.zeros_like(red)]
    done = [torch.cuda.Event(), torch.cuda.Event()]
    it = [0]
    # timed steps' all-reduces: HIP events on the comm stream around each one
    ar_events = []
    ar_timing = [False]

    def fill(buf):
        # the all-reduce payload [dC, loss], written inside the step's graph
        # (eager, these were three extra launches of ~4 us each per step)
        buf[:Q * Q].copy_(step.out_b["d_cost"].view(-1))
        torch.sum(step.out_f["tree_score"], dim=0, keepdim=True, out=buf[Q * Q:])

    use_graph = not args.no_graph
    graphs = None  # [buffer 0, buffer 1] step graphs (one without dist)
    step()
    if dist_on:
        fill(reds[0])
    torch.cuda.synchronize()
    if use_graph:
        graphs = []
        for i in range(2 if dist_on else 1):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
                if dist_on:
                    fill(reds[i])
            graphs.append(g)

    def run_once():
        i = it[0] % 2
        if dist_on:
            it[0] += 1
            # the all-reduce two steps back has read this buffer
            torch.cuda.current_stream(device).wait_event(done[i])
        if graphs is not None:
            graphs[i if dist_on else 0].replay()
        else:
            step()
            if dist_on:
                fill(reds[i])
        if dist_on:
            buf = reds[i]
            cur = torch.cuda.current_stream(device)
            comm.wait_stream(cur)
            with torch.cuda.stream(comm):
                if ar_timing[0]:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record(comm)
                dist.all_reduce(buf)
                if ar_timing[0]:
                    ev[1].record(comm)
                    ar_events.append(ev)
                done[i].record(comm)

    # settle: a fresh box runs the first ~30 ms of sustained work at rising
    # clocks (per-step 1 084 -> 922 us over the first 35 steps, then flat:
    # tools/time_step.py, profiles/r06_c4_cold_ramp.txt).  Blocks of 5 steps
    # (>= 5 ms each) run until one is within 1 % of the one before (at most 20), so
    # the W warmup and K timed steps below measure the steady state; the
    # settle steps are reported in the line (config.settle_steps)
    # (N > 1: the stop decision is all-reduced, so every rank runs the same
    # steps and issues the same all-reduces)
    settle = 0
    if not args.no_settle:
        prev = None
        nblk = 5  # steps per block; after the first block, >= 5 ms of steps
        for blk in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(nblk):
                run_once()
            torch.cuda.synchronize()
            cur = (time.perf_counter() - t0) / nblk
            settle += nblk
            if blk == 0:
                nb5 = max(5, int(np.ceil(5e-3 / max(cur, 1e-6))))
                if dist_on:
                    nbt = torch.tensor([nb5], dtype=torch.int32, device=device)
                    dist.all_reduce(nbt, op=dist.ReduceOp.MAX)
                    nb5 = int(nbt.item())
                nblk = nb5
                prev = None
                continue
            stop = prev is not None and cur >= 0.99 * prev
            if dist_on:
                flag = torch.tensor([1 if stop else 0], dtype=torch.int32, device=device)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                stop = bool(flag.item())
            if stop:
                break
            prev = cur
    for _ in range(args.warmup):
        run_once()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    ar_timing[0] = dist_on
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_once()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t0
    ar_timing[0] = False
    dist_info = None
    if dist_on:
        # every rank's own time (all_gather), then the MAX the line reports
        mine = torch.tensor([el], dtype=torch.float64, device=device)
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
        t = mine.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        ar_us = [a.elapsed_time(b) * 1e3 for a, b in ar_events]
        dist_info = {"rccl_ranks": rccl_ranks, "world_size": dist.get_world_size(),
                     "ms_per_step_per_rank": [round(float(x.item()) / args.steps * 1e3, 4)
                                              for x in per_rank],
                     "allreduce_bytes": red.numel() * red.element_size(),
                     "allreduce_us_mean_rank0": round(sum(ar_us) / max(len(ar_us), 1), 2),
                     "allreduce_count": len(ar_us)}

    n_int = n - 1
    units = args.trees * L * n_int * Q  # the whole batch, all ranks
    value = units * args.steps / el
    dump = os.environ.get("TREX_BENCH_DUMP")
    if dump and rank == 0:
        # the last step's reduced [dC (Q*Q), loss] (rank 0's copy after the
        # all-reduce; at N = 1 the step's own dC and loss): tests compare it
        # with the single-process engine over the whole batch
        if dist_on:
            last = reds[(it[0] - 1) % 2]
        else:
            last = torch.cat([step.out_b["d_cost"].view(-1),
                              step.out_f["tree_score"].sum().view(1)])
        np.save(dump, last.cpu().numpy())

    # per-kernel device time (HIP events) -> roofline of the step's kernel
    kt = time_kernels(torch, step)
    nl = n
    # algorithmic HBM bytes per launch, SURVEY.md section 8(d) / DESIGN.md "Roofline":
    #   fwd:   int8 leaves in + fp32 DP table out            B*L*(n + 4*Q*n_int)
    #   bwd:   leaves + DP table in                          B*L*(n + 4*Q*n_int)
    #   fused: fwd + the adjoint's re-read of both           B*L*(2n + 8*Q*n_int)
    #   (no site scores are written in this step; dC and tree scores are O(Q^2 + B))
    fwd_bytes = B * L * (nl + 4 * Q * n_int)
    kern = {"sankoff_fwd_bwd": (kt["sankoff_fwd_bwd"], 2 * fwd_bytes),
            "sankoff_fwd": (kt["sankoff_fwd"], fwd_bytes),
            "sankoff_bwd": (kt["sankoff_bwd"], fwd_bytes)}
    dom = "sankoff_fwd_bwd"
    achieved = kern[dom][1] / kern[dom][0] / 1e9
    # measured HBM traffic per launch (rocprofv3 FETCH_SIZE / WRITE_SIZE passes,
    # calibrated: tools/pmc.sh traffic c4 -> profiles/traffic.json)
    traffic = {}
    try:
        with open(args.traffic) as f:
            tj = json.load(f)
        if tj.get("workload_key") == f"{B}x{n}x{L}x{Q}":
            traffic = {k: tj.get(k) for k in kern}
    except (OSError, ValueError):
        pass
    per_kernel = {k: {"us": round(v[0] * 1e6, 2), "algorithmic_bytes": v[1],
                      "GBs": round(v[1] / v[0] / 1e9, 1),
                      "frac": round(v[1] / v[0] / 1e9 / HBM_PEAK_GBS, 4),
                      "traffic_bytes": traffic.get(k)} for k, v in kern.items()}
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic.get(dom),
                "per_kernel": per_kernel,
                "per_kernel_us": {k: round(v[0] * 1e6, 2) for k, v in kern.items()}}

    result = {
        "metric": "site-node-state updates/sec (Sankoff fwd+grad)",
        "value": value,
        "unit": "site-node-state updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (random coalescent topologies, iid uniform leaf states, C = 1 - I)",
        "config": {"workload": f"C4: {args.trees} random {n}-taxa topologies x {L} sites x "
                               f"{Q} states, softmin tau={tau} fwd (DP table written) + grad, "
                               f"split over {world} GPU(s) ({B} trees on rank 0)"
                               + ("; RCCL all-reduce of [dC, loss] per step, overlapped with "
                                  "the next step" if dist_on else ""),
                   "trees": args.trees, "trees_rank0": B, "taxa": n, "sites": L, "states": Q,
                   "tau": tau, "hipgraph": use_graph, "parallelism": f"tree-batch x{world}",
                   "settle_steps": settle,
                   "process_group": dist.get_backend() if dist_on else None,
                   "rccl_ranks": dist_info["rccl_ranks"] if dist_info else None,
                   "world_size": dist_info["world_size"] if dist_info else None},
        "roofline": roofline,
    }
    if dist_info:
        result["dist"] = dist_info
    if rank == 0 and not dist_on:
        hinfo, threads = host_cpu()
        threads = args.cpu_threads or threads
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(ch, leaves.cpu().numpy(), cost.cpu().numpy(),
                                                  tau, L, n, Q, threads)
            result["cpu_baseline"]["host"] = hinfo
        if not args.no_e2e:
            result["c4_e2e"] = e2e_line(torch, run_once, leaves, units,
                                        make_step=lambda b: Step(torch, eng, b, cost, tau))
        if not args.no_shard:
            result["c4_shard"] = shard_line(torch, device, ch, leaves, cost, tau, L, Q, n,
                                            min(128, B))
        if not args.no_c2:
            result["c2"] = c2_line(torch, device, args, threads)
        if not args.no_c3:
            result["c3"] = c3_line(torch, device, threads)
        if not args.no_c5:
            c5kw = dict(steps=args.c5_steps, warmup=args.c5_warmup, nl=args.c5_taxa,
                        L=args.c5_sites)
            result["c5"] = c5_line(torch, device, **c5kw)
            torch.cuda.empty_cache()
            result["c5_f32"] = c5_line(torch, device, gemm="f32", **c5kw)
        if not args.no_nk:
            result["nk"] = nk_line(torch, device)
        if not args.no_ragged:
            result["ragged"] = ragged_line(torch, device)
    if dist_on and not args.no_c5:
        result["c5"] = c5_line(torch, device, steps=args.c5_steps, warmup=args.c5_warmup,
                               rank=rank, world=world, nl=args.c5_taxa, L=args.c5_sites,
                               dist_on=True)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
