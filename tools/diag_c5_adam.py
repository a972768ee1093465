"""Diagnostic: the C5 full-size TreeOptimizer loop (tests/test_configs_full_gpu.py
test_c5_full_size_step_vs_fp64) with every step's d tree_params and the final
parameters dumped for both GEMM precisions, next to the fp64 oracle's, so the
tree_params tolerance can be analysed offline.

  python tools/diag_c5_adam.py gpurun_out/c5_adam.npz
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import tree_ref as T  # noqa: E402
from test_configs_full_gpu import _c5_case, _dev  # noqa: E402


def main(out):
    from trex_amd import tree as G

    dev = torch.device("cuda", 0)
    S, params, noise = _c5_case()
    n, L, Q = S.shape
    temps = [2.0, 1.9996, 1.9992]
    res = {}
    p64 = {k: v.astype(np.float64) for k, v in params.items()}
    st = T.adam_init(p64)
    for k in range(3):
        rl, gr = T.compute_loss(noise, p64, S, temps[k], None)
        A64 = T.update_tree(p64["tree_params"], noise, 1.0)
        S64 = T.update_seq(p64["ancestors"], S, temps[k])
        _, _, dA64 = T.compute_surrogate_cost_grads(S64, A64)
        dA64 = dA64 + temps[k] * T.enforce_graph_constraints_grad(A64, 10.0)
        res[f"ref_loss{k}"] = rl
        res[f"ref_g{k}"] = gr["tree_params"]
        res[f"ref_A{k}"] = A64
        res[f"ref_dAmax{k}"] = np.abs(dA64).max(axis=1)
        upd, st = T.adam_update(gr, st, lr=0.01)
        p64 = {kk: p64[kk] + upd[kk] for kk in p64}
    res["ref_p"] = p64["tree_params"]
    del S64
    for gemm in ("x3", "f32"):
        opt = G.TreeOptimizer(_dev(S, dev), {k: _dev(v, dev) for k, v in params.items()},
                              lr=0.01, gemm=gemm)
        nz = _dev(noise, dev)
        for k in range(3):
            nxt = temps[k + 1] if k + 1 < 3 else temps[k]
            lk = float(opt.step(temps[k], nz, next_temperature=nxt))
            torch.cuda.synchronize()
            res[f"{gemm}_loss{k}"] = lk
            res[f"{gemm}_g{k}"] = opt.grads["tree_params"].cpu().numpy()
        res[f"{gemm}_p"] = opt.params["tree_params"].cpu().numpy()
        res[f"{gemm}_anc_err"] = float(np.abs(opt.params["ancestors"].cpu().numpy()
                                              - p64["ancestors"]).max())
        del opt
        torch.cuda.empty_cache()
    np.savez_compressed(out, **res)
    print("saved", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5_adam.npz")
