"""Tuning aid: time the uniform engine vs the ragged engine on the SAME C4
shard (128 x 32 taxa x 5000 sites x 4 states): forward, adjoint, fused."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from trex_amd import SankoffEngine, TreePlan, random_topologies  # noqa: E402
from trex_amd.ragged import RaggedSankoffEngine, RaggedTreePlan  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    dev = torch.device("cuda", 0)
    B, n, L, Q, tau = 128, 32, 5000, 4, 0.5
    ch = random_topologies(B, n, seed=4)
    leaves = np.random.default_rng(5).integers(0, Q, size=(B, n, L)).astype(np.int8)
    cost = torch.as_tensor((np.ones((Q, Q)) - np.eye(Q)).astype(np.float32), device=dev)
    u = SankoffEngine(TreePlan(ch), L, Q, dev)
    lv = torch.as_tensor(leaves, device=dev)
    rp = RaggedTreePlan(list(ch), [L] * B)
    r = RaggedSankoffEngine(rp, Q, dev)
    rlv = torch.as_tensor(rp.pack_leaves(list(leaves)), device=dev)
    f = u.forward(lv, cost, tau)
    _, rdp, _ = r.forward(rlv, cost, tau)
    res = {
        "uniform fwd": timeit(lambda: u.forward(lv, cost, tau)),
        "ragged fwd": timeit(lambda: r.forward(rlv, cost, tau)),
        "uniform bwd": timeit(lambda: u.backward(lv, cost, tau, f.dp)),
        "ragged bwd": timeit(lambda: r.backward(rlv, cost, tau, rdp)),
        "uniform fused": timeit(lambda: u.fwd_bwd(lv, cost, tau)),
        "ragged fused": timeit(lambda: r.fwd_bwd(rlv, cost, tau)),
    }
    for k, v in res.items():
        print(f"{k:16s} {v:8.1f} us")


if __name__ == "__main__":
    main()
