"""Microbenchmarks: achievable HBM write / copy bandwidth on this GPU and the
Sankoff forward at several batch sizes and both cost modes (tuning aid)."""
import sys, os, time, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trex_amd import SankoffEngine, TreePlan, random_topologies


def t_ev(fn, n=20):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


dev = torch.device("cuda", 0)
out = {}
x = torch.empty(317 * 2**20 // 4, dtype=torch.float32, device=dev)
y = torch.empty_like(x)
s = t_ev(lambda: x.fill_(1.0)); out["fill_GBs"] = x.numel() * 4 / s / 1e9
s = t_ev(lambda: y.copy_(x)); out["copy_GBs"] = 2 * x.numel() * 4 / s / 1e9
for B in (128, 256, 512):
    n, L, Q = 32, 5000, 4
    ch = random_topologies(B, n, seed=4)
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    lv = torch.randint(0, Q, (B, n, L), device=dev, dtype=torch.int8)
    c = (torch.ones(Q, Q) - torch.eye(Q)).to(dev)
    dp = torch.empty(eng.dp_shape, device=dev)
    o = {"dp": dp, "tree_score": torch.empty(B, device=dev)}
    for tau in (0.0, 0.5):
        s = t_ev(lambda: eng.forward(lv, c, tau, out=o))
        out[f"fwd_B{B}_tau{tau}_us"] = s * 1e6
        out[f"fwd_B{B}_tau{tau}_GBs"] = B * L * (n + 4 * Q * (n - 1)) / s / 1e9
print(json.dumps(out, indent=1))
