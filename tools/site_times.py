"""Phase timestamps of the lane-per-site kernel (diagnostic build:
tools/build_ab.sh sitet sankoff_site.hip -DTREX_SITE_TIMING) on C3: per wave
and phase, mean cycles over workgroups.  --pair: the wave-pair kernel
(tools/build_ab.sh s2t sankoff_site2.hip -DTREX_SITE2_TIMING, 16 waves).

  TREX_HIP_LIB=trex_amd/libtrex_ab_sitet.so python tools/site_times.py
  TREX_HIP_LIB=trex_amd/libtrex_ab_s2t.so python tools/site_times.py --pair
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
PAIR = "--pair" in sys.argv
if PAIR:
    os.environ.setdefault("TREX_SITE2", "8")
os.environ.setdefault("TREX_HIP_LIB", os.path.join(ROOT, "trex_amd",
                                                   "libtrex_ab_s2t.so" if PAIR else "libtrex_ab_sitet.so"))
from _cases import int_cost, simulate_leaves  # noqa: E402

from trex_amd import SankoffEngine, TreePlan, children_from_adjacency  # noqa: E402
from trex_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
nl, L, Q, tau = 64, 10000, 20, 0.5
seqs, adj = simulate_leaves(nl, L, Q, 50, seed=2)
eng = SankoffEngine(TreePlan(children_from_adjacency(adj)), L, Q, dev)
lv = torch.from_numpy(np.ascontiguousarray(seqs[None, :nl])).to(dev)
c = torch.as_tensor(int_cost(Q, seed=3), device=dev)
for _ in range(10):
    eng.fwd_bwd(lv, c, tau, marginals=True, anc_states=True)
torch.cuda.synchronize()
NW = 16 if PAIR else 8
buf = np.zeros((2048, NW, 20), np.uint64)
fn = lib().trex_debug_site2_times if PAIR else lib().trex_debug_site_times
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
nwg = (L + 63) // 64
t = buf[:nwg].astype(np.int64)
names = {1: "prologue", 2: "fwd s0", 3: "fwd s1", 4: "fwd s2", 5: "fwd s3", 6: "fwd s4", 7: "fwd s5",
         8: "root", 9: "sync", 10: "adj s(S-1)", 11: "adj s(S-2)", 12: "adj s(S-3)", 13: "adj s(S-4)",
         14: "adj s(S-5)", 15: "adj s(S-6)", 16: "dC reduce"}
print("workgroups", nwg, "span cycles", int(t[:, :, 16].max() - t[:, :, 0].min()),
      "mean WG life", float((t[:, 0, 16] - t[:, 0, 0]).mean()))
prev = t[:, :, 0]
for j in range(1, 17):
    col = t[:, :, j]
    if not col.any():
        continue
    d = col - prev
    print(f"{names[j]:12s} " + " ".join(f"{d[:, w].mean():7.0f}" for w in range(NW)))
    prev = col
