"""The NK landscape-aware step at the reference's eval shape only (32 leaves,
15 sites, Q = 2, K = 10; src/trex/evals/benchmark.py:981-985), eager then as
hipGraph replays, for rocprofv3 kernel-trace collection:
    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python tools/prof_nk_eval.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import numpy as np
    import torch

    from trex_amd import nk as NK
    from trex_amd.datagen import create_nk_model_landscape

    dev = torch.device("cuda", 0)
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

    def step():
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    torch.cuda.synchronize()
    print("graph replay ms per step", (time.perf_counter() - t0) / 50 * 1e3)
