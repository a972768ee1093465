"""Debug: phase-1 (forward-only) DP table of the lane-per-site kernel vs the
fused kernel's, balanced 64-taxa, Q = 20 (TREX_SITE_CHERRY on / off)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _cases import balanced_children, int_cost, random_leaves  # noqa: E402

from trex_amd import SankoffEngine, TreePlan  # noqa: E402

dev = torch.device("cuda", 0)
B, n, L, Q, tau = 2, 64, 777, 20, 0.5
ch = balanced_children(n, B)
lv = torch.as_tensor(random_leaves(B, n, L, Q, seed=72, missing=0.03), device=dev)
c = torch.as_tensor(int_cost(Q, seed=73), device=dev)
for flag in ("1", "0"):
    os.environ["TREX_SITE_CHERRY"] = flag
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    for fill in (0.0, 7.0):
        f, _, _, _ = eng.fwd_bwd(lv, c, tau)
        dp_f = f.dp.clone()
        out = {"dp": torch.full(eng.dp_shape, fill, device=dev)}
        f2 = eng.forward(lv, c, tau, out=out)
        torch.cuda.synchronize()
        d = (f2.dp != dp_f)
        print(flag, fill, "mismatch", int(d.sum()), "of", d.numel())
        if d.any():
            idx = d.nonzero()
            rows = sorted(set(idx[:, 1].tolist()))
            sites = sorted(set(idx[:, 2].tolist()))
            print("  rows", rows[:20], "sites", sites[:10], "...", sites[-5:], "n_sites", len(sites))
            print("  got", f2.dp[tuple(idx[0].tolist())].item(), "fused", dp_f[tuple(idx[0].tolist())].item())
