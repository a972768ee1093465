"""Phase timestamps of the staged kernel (diagnostic build, see
tools/build_diag_staged.sh) on C2: per-phase mean cycles over workgroups and
the dispatch spread.

  TREX_HIP_LIB=trex_amd/libtrex_stagetime.so python tools/stage_times.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("TREX_HIP_LIB", os.path.join(ROOT, "trex_amd", "libtrex_stagetime.so"))
os.environ["TREX_WIDE_SMALLQ"] = "1"
os.environ["TREX_STAGED"] = "1"
from _cases import simulate_leaves  # noqa: E402

from trex_amd import SankoffEngine, TreePlan, children_from_adjacency  # noqa: E402
from trex_amd._lib import lib  # noqa: E402

dev = torch.device("cuda", 0)
seqs, adj = simulate_leaves(64, 10000, 4, 5, seed=1)
eng = SankoffEngine(TreePlan(children_from_adjacency(adj)), 10000, 4, dev)
lv = torch.from_numpy(np.ascontiguousarray(seqs[None, :64])).to(dev)
c = (torch.ones(4, 4) - torch.eye(4)).to(dev)
for _ in range(20):
    eng.fwd_bwd(lv, c, 1.0)
torch.cuda.synchronize()
buf = np.zeros((4096, 20), np.uint64)
fn = lib().trex_debug_stage_times
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
nwg = 625
t = buf[:nwg].astype(np.int64)
t0 = t[:, 0]
print("workgroups", nwg, "start spread (cycles) min 0 max", int(t0.max() - t0.min()),
      "span start->end", int(t[:, 19].max() - t0.min()))
labels = {1: "prologue"}
for s in range(6):
    labels[2 + s] = f"fwd stage {s}"
labels[10] = "root"
for s in range(6):
    labels[11 + s] = f"bwd stage {5 - s}"
labels[19] = "dC reduce"
prev = 0
for j in list(range(1, 8)) + [10] + list(range(11, 17)) + [19]:
    d = t[:, j] - t[:, prev]
    print(f"{labels[j]:14s} mean {d.mean():8.0f}  min {d.min():8d}  max {d.max():8d}")
    prev = j
tot = t[:, 19] - t[:, 0]
print(f"{'per-WG total':14s} mean {tot.mean():8.0f}  min {tot.min():8d}  max {tot.max():8d}")

rt = np.zeros((4096, 2), np.uint64)
f2 = lib().trex_debug_stage_rt
f2.argtypes = [ctypes.c_void_p]
assert f2(rt.ctypes.data) == 0
r = rt[:nwg].astype(np.int64) * 10  # ns
r0 = r[:, 0].min()
st, en = r[:, 0] - r0, r[:, 1] - r0
print("realtime (ns): start min/median/max", st.min(), int(np.median(st)), st.max(),
      " end min/median/max", en.min(), int(np.median(en)), en.max())
print("per-WG lifetime ns mean", int((en - st).mean()), "kernel span (first start -> last end)", en.max())
