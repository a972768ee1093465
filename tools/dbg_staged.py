"""Debug: staged vs one-wave kernel DP tables on a small case."""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from _cases import random_topologies, int_cost
from trex_amd import SankoffEngine, TreePlan
dev = torch.device("cuda", 0)
for Q, L in ((20, 1), (20, 7), (8, 7), (16, 7), (32, 7)):
    ch = random_topologies(1, 16, seed=221)
    rng = np.random.default_rng(3)
    lv = torch.as_tensor(rng.integers(0, Q, size=(1, 16, L)).astype(np.int8), device=dev)
    c = torch.as_tensor(int_cost(Q, seed=Q + L), device=dev)
    res = {}
    for st in ("0", "1"):
        os.environ["TREX_STAGED"] = st
        eng = SankoffEngine(TreePlan(ch), L, Q, dev)
        f = eng.forward(lv, c, 0.0)
        torch.cuda.synchronize()
        res[st] = f.dp.cpu().numpy()[0]  # (n_int, L, Q)
    d = res["0"] != res["1"]
    print(Q, L, "mismatch rows", sorted(set(np.argwhere(d)[:, 0].tolist())), "sites",
          sorted(set(np.argwhere(d)[:, 1].tolist())), "states", sorted(set(np.argwhere(d)[:, 2].tolist())))
