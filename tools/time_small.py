"""Same-box A/B of the small-grid Sankoff kernels: C2 (64 taxa x 10 000 x 4,
softmin fwd + grad) and C3 (64 taxa x 10 000 x 20, fwd + grad + marginals +
soft ancestral) under kernel-selection environment settings, hipGraph
replay (what bench.py's c2 / c3 lines time).

  python tools/time_small.py [C2|C3|C3P|C3Q] ...   (default: C2 C3)
"""

from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _cases import int_cost, simulate_leaves  # noqa: E402

from trex_amd import SankoffEngine, TreePlan, children_from_adjacency  # noqa: E402

CONFIGS = {
    "C2": [("wave", {"TREX_WIDE_SMALLQ": "1", "TREX_STAGED": "0"}),
           ("staged", {"TREX_WIDE_SMALLQ": "1", "TREX_STAGED": "1"}),
           ("lane", {"TREX_WIDE_SMALLQ": "0", "TREX_STAGED": "0"})],
    "C3": [("wave", {"TREX_STAGED": "0"}), ("staged", {"TREX_STAGED": "1"})],
    # the lane-per-site kernel: one wave per site set vs a wave pair (sankoff_site2.hip)
    "C3P": [("one", {"TREX_SITE2": "0"}), ("pair8", {"TREX_SITE2": "8"}),
            ("pair6", {"TREX_SITE2": "6"}), ("pair4", {"TREX_SITE2": "4"}),
            ("one", {"TREX_SITE2": "0"}), ("pair8", {"TREX_SITE2": "8"}),
            ("pair6", {"TREX_SITE2": "6"}), ("pair4", {"TREX_SITE2": "4"})],
    "C3Q": [("one", {"TREX_SITE2": "0"}), ("pair8", {"TREX_SITE2": "8"}),
            ("one", {"TREX_SITE2": "0"}), ("pair8", {"TREX_SITE2": "8"})],
}


def replay_us(fn, n=100, per_graph=10):
    """GPU time per step: graphs of per_graph steps (amortises the launch)."""
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(per_graph):
            fn()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    best = []
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize()
        best.append((time.perf_counter() - t0) / n / per_graph * 1e6)
    return min(best)


def case(name, dev):
    if name == "C2":
        nl, L, Q, tau, mut, seed = 64, 10000, 4, 1.0, 5, 1
        cost = (np.ones((Q, Q)) - np.eye(Q)).astype(np.float32)
    else:
        nl, L, Q, tau, mut, seed = 64, 10000, 20, 0.5, 50, 2
        cost = int_cost(Q, seed=3)
    seqs, adj = simulate_leaves(nl, L, Q, mut, seed=seed)
    ch = children_from_adjacency(adj)
    name = name[:2]
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    lv = torch.from_numpy(np.ascontiguousarray(seqs[None, :nl])).to(dev)
    c = torch.from_numpy(cost).to(dev)
    f = torch.empty(eng.dp_shape, dtype=torch.float32, device=dev)
    out = {"dp": f, "tree_score": torch.empty(1, device=dev),
           "d_cost": torch.empty((Q, Q), device=dev)}
    extra = {}
    if name == "C3":
        out["marginals"] = torch.empty_like(f)
        out["anc_states"] = torch.empty((1, nl - 1, L), dtype=torch.int8, device=dev)
        extra = dict(marginals=True, anc_states=True)

    def step():
        eng.fwd_bwd(lv, c, tau, out=out, **extra)

    return step, out


def main():
    dev = torch.device("cuda", 0)
    names = sys.argv[1:] or ["C2", "C3"]
    for name in names:
        ref = None
        for label, env in CONFIGS[name]:
            os.environ.update(env)
            step, out = case(name, dev)
            us = replay_us(step)
            step()
            torch.cuda.synchronize()
            sc = float(out["tree_score"][0])
            dc = out["d_cost"].cpu().numpy()
            if ref is None:
                ref = (sc, dc)
            rel = float(np.abs(dc - ref[1]).max() / np.abs(ref[1]).max())
            extra_s = ""
            if "TREX_SITE2" in env:
                from trex_amd._lib import lib
                extra_s = f"  site2 launches {lib().trex_debug_site2_launches()}"
            print(f"{name} {label:7s} {us:8.1f} us  score {sc:.6f}  dC rel diff {rel:.2e}{extra_s}",
                  flush=True)


if __name__ == "__main__":
    main()
