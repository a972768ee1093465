"""C2 fwd + grad a few times (for rocprofv3 --pmc passes of the staged kernel).
  python tools/prof_c2.py [iters]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _cases import simulate_leaves  # noqa: E402

from trex_amd import SankoffEngine, TreePlan, children_from_adjacency  # noqa: E402

dev = torch.device("cuda", 0)
seqs, adj = simulate_leaves(64, 10000, 4, 5, seed=1)
eng = SankoffEngine(TreePlan(children_from_adjacency(adj)), 10000, 4, dev)
lv = torch.from_numpy(np.ascontiguousarray(seqs[None, :64])).to(dev)
c = (torch.ones(4, 4) - torch.eye(4)).to(dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    eng.fwd_bwd(lv, c, 1.0)
torch.cuda.synchronize()
print("ok")
