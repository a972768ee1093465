"""Phase timestamps of the matrix-core kernel (diagnostic build,
tools/build_diag_mx.sh) on C3: per-phase mean cycles over workgroups.

  TREX_HIP_LIB=trex_amd/libtrex_mxtime.so python tools/mx_times.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("TREX_HIP_LIB", os.path.join(ROOT, "trex_amd", "libtrex_mxtime.so"))
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
buf = np.zeros((4096, 24), np.uint64)
fn = lib().trex_debug_mx_times
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
nwg = (L + 15) // 16
t = buf[:nwg].astype(np.int64)
names = ["prologue"] + [f"fwd stage {s}" for s in range(6)] + ["root+sync"] + \
        [f"adj stage {5 - s}" for s in range(6)] + ["dC reduce"]
cols = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15]
d = np.diff(t[:, cols], axis=1)
print("workgroups", nwg, "total mean cycles", float((t[:, 15] - t[:, 0]).mean()),
      "start spread", int(t[:, 0].max() - t[:, 0].min()), "span", int(t[:, 15].max() - t[:, 0].min()))
for k, nm in enumerate(names):
    print(f"{nm:14s} mean {d[:, k].mean():9.0f}  p90 {np.percentile(d[:, k], 90):9.0f}")
