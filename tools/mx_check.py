"""Diagnostic: the matrix-core kernel (sankoff_mx.hip) vs the state-parallel
kernel (TREX_MX=0) vs the fp64 oracle on Q = 20 cases, plus C3 timing.
Not a test (tests/ hold the parity bars); run on the GPU box:
    python tools/mx_check.py
"""
from __future__ import annotations

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

from _cases import int_cost, random_leaves, random_topologies, simulate_leaves  # noqa: E402
from oracle.softmin_ref import batched_fwd_bwd_ref  # noqa: E402
from trex_amd import SankoffEngine, TreePlan, children_from_adjacency  # noqa: E402


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-30)))


def run(eng, lv, c, tau, mx):
    os.environ["TREX_MX"] = "1" if mx else "0"
    f, dc, mg, an = eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True, site_score=True)
    torch.cuda.synchronize()
    return f, dc, mg, an


def case(name, ch, leaves, cost, tau, dev, oracle=True):
    B, n, L = leaves.shape
    Q = cost.shape[0]
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    lv = torch.as_tensor(leaves, device=dev)
    c = torch.as_tensor(cost, device=dev)
    fm, dm, mm, am = run(eng, lv, c, tau, True)
    fs, ds, ms, as_ = run(eng, lv, c, tau, False)
    out = {"case": name, "score_mx_vs_sp": rel(fm.tree_score.cpu(), fs.tree_score.cpu()),
           "dc_mx_vs_sp": rel(dm.cpu(), ds.cpu()),
           "dp_mx_vs_sp": float((fm.dp - fs.dp).abs().max()),
           "marg_mx_vs_sp": float((mm - ms).abs().max()),
           "anc_diff": int((am != as_).sum())}
    if oracle:
        ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
        out["score_mx_vs_ref"] = rel(fm.tree_score.cpu(), ref["tree_score"])
        out["dc_mx_vs_ref"] = rel(dm.cpu(), ref["d_cost"])
        out["dc_sp_vs_ref"] = rel(ds.cpu(), ref["d_cost"])
    # fused == separate launches on the mx path
    os.environ["TREX_MX"] = "1"
    f2 = eng.forward(lv, c, tau, site_score=True)
    d2, m2, a2 = eng.backward(lv, c, tau, f2.dp, marginals=True, anc_states=True)
    torch.cuda.synchronize()
    out["fused_eq_separate"] = bool(torch.equal(f2.dp, fm.dp) and torch.equal(d2, dm)
                                    and torch.equal(m2, mm) and torch.equal(a2, am)
                                    and torch.equal(f2.tree_score, fm.tree_score))
    print(out, flush=True)
    return eng, lv, c


def timing(eng, lv, c, tau, mx, n=50):
    os.environ["TREX_MX"] = "1" if mx else "0"
    f = torch.empty(eng.dp_shape, dtype=torch.float32, device=lv.device)
    Q = c.shape[0]
    out = {"dp": f, "tree_score": torch.empty(eng.plan.B, device=lv.device),
           "d_cost": torch.empty((Q, Q), device=lv.device), "marginals": torch.empty_like(f),
           "anc_states": torch.empty((eng.plan.B, eng.plan.n_int, eng.L), dtype=torch.int8,
                                     device=lv.device)}
    for _ in range(5):
        eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True, out=out)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in ev:
        e0.record()
        eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True, out=out)
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev])) * 1e3


def main():
    dev = torch.device("cuda", 0)
    ch = random_topologies(2, 16, seed=29)
    case("rand16x300 q20 tau0.5", ch, random_leaves(2, 16, 300, 20, seed=3), int_cost(20, seed=3), 0.5, dev)
    case("rand16x300 q20 missing", ch, random_leaves(2, 16, 300, 20, seed=4, missing=0.05),
         int_cost(20, seed=3), 1.0, dev)
    case("rand12x257 q7 tau0.3", random_topologies(3, 12, seed=5), random_leaves(3, 12, 257, 7, seed=6),
         int_cost(7, seed=7), 0.3, dev)
    case("rand12x100 q13 tau1", random_topologies(2, 12, seed=8), random_leaves(2, 12, 100, 13, seed=9),
         int_cost(13, seed=10, hi=2), 1.0, dev)
    # C3 at full size
    nl, L, Q, tau = 64, 10000, 20, 0.5
    seqs, adj = simulate_leaves(nl, L, Q, 50, seed=2)
    ch = children_from_adjacency(adj)
    eng, lv, c = case("C3 full", ch, np.ascontiguousarray(seqs[None, :nl]), int_cost(Q, seed=3), tau,
                      dev, oracle=False)
    t_mx = timing(eng, lv, c, tau, True)
    t_sp = timing(eng, lv, c, tau, False)
    print({"C3_fused_us_mx": t_mx, "C3_fused_us_state_parallel": t_sp}, flush=True)


if __name__ == "__main__":
    main()
