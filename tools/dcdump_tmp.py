import os, sys
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from _cases import int_cost, simulate_leaves
from oracle.softmin_ref import batched_fwd_bwd_ref
from trex_amd import SankoffEngine, TreePlan, children_from_adjacency
dev = torch.device("cuda", 0)
nl, Q, tau = 64, 20, 0.5
for L in (1000, 10000):
    seqs, adj = simulate_leaves(nl, L, Q, 50, seed=2)
    ch = children_from_adjacency(adj)
    lv = np.ascontiguousarray(seqs[None, :nl])
    cost = int_cost(Q, seed=3)
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    res = {}
    for mx in ("1", "0"):
        os.environ["TREX_MX"] = mx
        f, dc, _, _ = eng.fwd_bwd(torch.as_tensor(lv, device=dev), torch.as_tensor(cost, device=dev), tau, site_score=True)
        torch.cuda.synchronize()
        res[mx] = (f.tree_score.cpu().numpy().astype(np.float64), f.site_score.cpu().numpy()[0].astype(np.float64), dc.cpu().numpy())
    ss1, ss0 = res["1"][1], res["0"][1]
    d = np.abs(ss1 - ss0)
    print("L", L, "tree", res["1"][0], res["0"][0], "site-sum", ss1.sum(), ss0.sum(), "max site diff", d.max(), "argmax", d.argmax(), "n>1e-3", int((d > 1e-3).sum()))
    if L == 1000:
        ref = batched_fwd_bwd_ref(ch, lv, cost, tau)
        print(" ref tree", ref["tree_score"], "max site err mx", np.abs(ss1 - ref["site_score"][0]).max(), "sp", np.abs(ss0 - ref["site_score"][0]).max())
