import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from trex_amd._lib import lib, ptr, check, stream_handle
dev = torch.device("cuda", 0)
for (N, L) in [(511, 50000), (511, 5000), (200, 50000), (129, 50000)]:
    rng = np.random.default_rng(21)
    seq = torch.as_tensor(rng.integers(0, 4, size=(N, L)), device=dev)
    S = torch.nn.functional.one_hot(seq, 4).to(torch.float32).contiguous()
    A = torch.zeros(N, N, device=dev)
    K = L * 4
    loss = torch.empty(1, device=dev); Gout = torch.empty(N, N, device=dev)
    ws = torch.empty(lib().trex_tree_workspace_bytes(N, K), dtype=torch.uint8, device=dev)
    check(lib().trex_tree_surrogate(ptr(S), ptr(A), N, K, ptr(loss), None, None, ptr(Gout), ptr(ws), ws.numel(), stream_handle(dev)))
    F = S.reshape(N, -1).double()
    Gr = (F @ F.T)
    d = (Gout.double() - Gr).abs()
    bad = (d > 0).nonzero()
    print(N, L, "max err", float(d.max()), "nbad", bad.shape[0], bad[:10].tolist() if bad.shape[0] else "")
    if bad.shape[0]:
        rows = sorted(set(bad[:, 0].tolist()))
        print("  bad rows range", rows[0], rows[-1], len(rows), " cols", sorted(set(bad[:,1].tolist()))[:5])
