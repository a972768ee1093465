"""One workload driver for rocprofv3 kernel-trace / PMC runs (and quick
timing): runs the named workload ITERS times on cuda:0.

    python tools/prof.py WORKLOAD [--iters N] [--trees B]
    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- \
        python3 tools/prof.py c4-fused

workloads
  c4-fused | c4-fwd | c4-bwd | c4   the bench's C4 entry points (1 024 trees x
                                     32 taxa x 5 000 sites x 4, tau 0.5; --trees)
  c2 | c3                            BASELINE configs[1] / [2] under the library's
                                     kernel policy (tools/time_small.py cases)
  c5                                 the bench's C5 Adam step (x3 GEMMs)
  gemm                               the C5-shape GEMMs alone: x3 Gram (leaf block
                                     skipped) + ancestor-rows MF, then the f32 ones
  nk | nk-eval                       the NK landscape-aware step at the DNA shape
                                     (bench nk_line) / the reference's eval shape
                                     as hipGraph replays
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def c4(torch, dev, a, which):
    from bench import Step, make_inputs
    from trex_amd import SankoffEngine

    ch, plan, leaves, cost = make_inputs(torch, dev, a.trees, 32, 5000, 4, 0, a.trees)
    st = Step(torch, SankoffEngine(plan, 5000, 4, dev), leaves, cost, 0.5)
    st.fwd()
    for _ in range(a.iters):
        if which in ("c4", "c4-fused"):
            st.fused()
        if which in ("c4", "c4-fwd"):
            st.fwd()
        if which in ("c4", "c4-bwd"):
            st.bwd()


def small(torch, dev, a, which):
    from time_small import case

    step, _ = case(which.upper(), dev)
    for _ in range(a.iters):
        step()


def gemm(torch, dev, a):
    from trex_amd._lib import check, lib, ptr, stream_handle

    N, K, nl = 511, 200000, 256
    g = torch.Generator(device=dev).manual_seed(0)
    S = torch.rand((N, K), device=dev, generator=g)
    M = torch.rand((N, N), device=dev, generator=g)
    G = torch.empty((N, N), device=dev)
    dS = torch.empty((N - nl, K), device=dev)
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=dev)
    st = stream_handle(dev)
    for _ in range(a.iters):
        check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, nl, 1.0, ptr(G), ptr(ws), ws.numel(), st))
        check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, nl, N - nl, float(N + 1), 1.0,
                                         ptr(dS), st))
        check(lib().trex_tree_gram_skip(ptr(S), N, K, nl, ptr(G), ptr(ws), ws.numel(), st))
        check(lib().trex_tree_mf_rows(ptr(M), ptr(S), N, K, nl, N - nl, ptr(dS), st))


def nk_eval(torch, dev, a):
    import numpy as np

    from trex_amd import nk as NK
    from trex_amd.datagen import create_nk_model_landscape

    nl, L, Q, k, lam = 32, 15, 2, 10, 3.0
    n_all = 2 * nl - 1
    rng = np.random.default_rng(8)
    land_np = create_nk_model_landscape(L, k, seed=9, n_states=Q)
    A = np.zeros((n_all, n_all), np.float32)
    A[np.arange(n_all - 1), nl + np.arange(n_all - 1) // 2] = 1.0
    land = NK.NKLandscape(land_np["interactions"], land_np["fitness_tables"], Q, dev)
    S0 = NK.masked_sequences_from_leaves(rng.integers(0, Q, size=(nl, L)), n_all, Q, dev)
    fn = NK.LandscapeAwareLoss(A, nl, land, lam, k)
    opt = NK.LandscapeAwareAdam(fn, rng.normal(size=(nl - 1, L, Q)).astype(np.float32), S0, 1e-3)
    for _ in range(5):
        opt.step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        opt.step()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        g.replay()
    torch.cuda.synchronize()
    print("graph replay ms per step", (time.perf_counter() - t0) / a.iters * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workload")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--trees", type=int, default=1024)
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    w = a.workload
    if w.startswith("c4"):
        c4(torch, dev, a, w)
    elif w in ("c2", "c3"):
        small(torch, dev, a, w)
    elif w == "c5":
        from bench import c5_line

        print(c5_line(torch, dev, steps=a.iters, warmup=2))
    elif w == "gemm":
        gemm(torch, dev, a)
    elif w == "nk":
        from bench import nk_line

        print(nk_line(torch, dev, steps=a.iters, warmup=2))
    elif w == "nk-eval":
        nk_eval(torch, dev, a)
    else:
        raise SystemExit(f"unknown workload {w!r} (see the docstring)")
    torch.cuda.synchronize()
    print("done", w)


if __name__ == "__main__":
    main()
