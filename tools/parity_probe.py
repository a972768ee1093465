"""Elementwise parity probe (diagnostic, GPU): measures the per-entry errors the
tests' bars are set from -- softmin marginals vs the fp64 oracle as a ratio of
the fp32-D conditioning bound (tests/_cases.py path_dmax), Gram entries
(elementwise relative), MF / dS / dA entries against their |terms| bounds.

python tools/parity_probe.py [marg|site|gemm|c5 ...]
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from _cases import hamming, int_cost, path_dmax, random_leaves, random_topologies  # noqa: E402
from oracle.softmin_ref import batched_fwd_bwd_ref  # noqa: E402
from trex_amd import SankoffEngine, TreePlan  # noqa: E402

EPS = 2.0 ** -24
dev = torch.device("cuda", 0)


def _d(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(dev).contiguous()


def marg_stats(tag, ch, leaves, cost, tau, env):
    for k, v in env.items():
        os.environ[k] = v
    B, n, L = leaves.shape
    Q = cost.shape[0]
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    eng = SankoffEngine(TreePlan(ch), L, Q, dev)
    f, dc, mg, _ = eng.fwd_bwd(_d(leaves), _d(cost, torch.float32), tau, marginals=True)
    got = eng.state_rows(mg).cpu().numpy().astype(np.float64)
    r = ref["marginals"]
    pd = path_dmax(ch, ref["dp"])[:, :, None, :]
    m = np.abs(r) > 1e-30
    rel = np.abs(got - r) / np.maximum(np.abs(r), 1e-300)
    cond = EPS * pd / tau
    ratio = rel / np.maximum(cond, 1e-300)
    dcr = np.abs(dc.cpu().numpy() - ref["d_cost"]) / np.abs(ref["d_cost"])
    flat_atol = max(2e-5, 8 * 1.2e-7 * np.abs(ref["dp"]).max() / tau)
    print(f"[marg] {tag} tau={tau}: max rel {rel[m].max():.3e}  n>1e-5 {int((rel[m] > 1e-5).sum())}"
          f"/{int(m.sum())}  max rel/(eps*pathD/tau) {ratio[m].max():.3f}  "
          f"max rel where cond<1e-5/4: {rel[m & (cond < 2.5e-6)].max() if (m & (cond < 2.5e-6)).any() else 0:.3e}"
          f"  (old flat atol {flat_atol:.2e}, max abs err {np.abs(got - r).max():.2e})  dC max rel {dcr.max():.2e}",
          flush=True)
    for k in env:
        del os.environ[k]


def probe_marg():
    q4k = {"lane": {"TREX_WIDE_SMALLQ": "0"},
           "state": {"TREX_WIDE_SMALLQ": "1", "TREX_STAGED": "0"},
           "staged": {"TREX_WIDE_SMALLQ": "1", "TREX_STAGED": "1"}}
    for (L, n) in [(1000, 64), (501, 32), (100, 8)]:
        ch = random_topologies(3, n, seed=n + 11)
        lv = random_leaves(3, n, L, 4, seed=L + 3)
        for tau in (1.0, 0.1, 0.02):
            for kn, env in q4k.items():
                marg_stats(f"Q4 {kn} L={L} n={n}", ch, lv, hamming(4), tau, env)
    wk = {"wave": {"TREX_STAGED": "0"}, "staged": {"TREX_STAGED": "1"}}
    for (L, n, Q) in [(100, 8, 20), (1000, 64, 20), (301, 16, 6), (257, 12, 32), (129, 10, 61)]:
        ch = random_topologies(2, n, seed=n + 13)
        lv = random_leaves(2, n, L, Q, seed=L + 5)
        for tau in (1.0, 0.1):
            for kn, env in wk.items():
                marg_stats(f"Q{Q} {kn} L={L} n={n}", ch, lv, hamming(Q), tau, env)
            if Q == 20:
                marg_stats(f"Q{Q} site=0 L={L} n={n}", ch, lv, hamming(Q), tau, {"TREX_SITE": "0"})
    # C3 full size
    ch = random_topologies(1, 64, seed=31)
    lv = random_leaves(1, 64, 10000, 20, seed=32)
    marg_stats("C3 full", ch, lv, int_cost(20, seed=3), 0.5, {})


def probe_site():
    B, n, L, Q, tau = 2, 8, 100, 20, 1.0
    ch = random_topologies(B, n, seed=19)
    leaves = random_leaves(B, n, L, Q, seed=103, missing=0.03)
    cost = hamming(Q)
    ref = batched_fwd_bwd_ref(ch, leaves, cost, tau)
    out = {}
    for site in ("1", "0"):
        os.environ["TREX_SITE"] = site
        eng = SankoffEngine(TreePlan(ch), L, Q, dev)
        f, dc, _, _ = eng.fwd_bwd(_d(leaves), _d(cost, torch.float32), tau)
        out[site] = dc.cpu().numpy().astype(np.float64)
        rel = np.abs(out[site] - ref["d_cost"]) / np.abs(ref["d_cost"])
        print(f"[site] TREX_SITE={site} missing 3%: dC max rel vs fp64 {rel.max():.3e}", flush=True)
    del os.environ["TREX_SITE"]
    rel = np.abs(out["1"] - out["0"]) / np.abs(out["0"])
    print(f"[site] site vs state-parallel dC max rel {rel.max():.3e}", flush=True)


def probe_gemm():
    from trex_amd._lib import check, lib, ptr, stream_handle

    st = stream_handle(dev)
    for N, K, skip in [(511, 4096, 256), (511, 4096, 0), (300, 160, 130), (100, 1024, 0),
                       (64, 16, 0), (511, 25000, 256), (300, 1028, 130), (64, 20, 0)]:
        rng = np.random.default_rng(N + K)
        logits = rng.normal(scale=3.0, size=(N, K // 4, 4))
        P = np.exp(logits - logits.max(-1, keepdims=True))
        P /= P.sum(-1, keepdims=True)
        P[: N // 3] = np.eye(4)[rng.integers(0, 4, size=(N // 3, K // 4))]
        S = P.reshape(N, K).astype(np.float32)
        Al = rng.normal(size=(N, N))
        A = np.exp(Al - Al.max(1, keepdims=True))
        A /= A.sum(1, keepdims=True)
        M = (np.diag(A.sum(1) + A.sum(0)) - (A + A.T)).astype(np.float32)
        St, Mt = _d(S), _d(M)
        ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=dev)
        S64 = S.astype(np.float64)
        Gref = S64 @ S64.T
        t0 = (skip // 64) * 64
        mask = np.ones((N, N), bool)
        mask[:t0, :t0] = False
        Gx = torch.zeros((N, N), device=dev)
        check(lib().trex_tree_gram_skip_x3(ptr(St), N, K, skip, 1.0, ptr(Gx), ptr(ws), ws.numel(), st))
        Gf = torch.zeros((N, N), device=dev)
        check(lib().trex_tree_gram_skip(ptr(St), N, K, skip, ptr(Gf), ptr(ws), ws.numel(), st))
        torch.cuda.synchronize()
        for tag, Gt in (("x3", Gx), ("f32", Gf)):
            g = Gt.cpu().numpy().astype(np.float64)
            rel = np.abs(g - Gref)[mask] / np.maximum(Gref[mask], 1e-300)
            k = int(np.argmax(rel))
            print(f"[gram] {tag} N={N} K={K} skip={skip}: max elementwise rel {rel.max():.3e} "
                  f"(entry {Gref[mask][k]:.4e}; min entry {Gref[mask].min():.3e})", flush=True)
        absb = np.abs(M.astype(np.float64)) @ np.abs(S64)
        for r0 in (N // 2, 0):
            out = torch.empty((N - r0, K), device=dev)
            check(lib().trex_tree_mf_rows_x3(ptr(Mt), ptr(St), N, K, r0, N - r0, float(N + 1), 1.0,
                                             ptr(out), st))
            outf = torch.empty((N, K), device=dev)
            check(lib().trex_tree_mf(ptr(Mt), ptr(St), N, K, ptr(outf), st))
            torch.cuda.synchronize()
            ref = M.astype(np.float64)[r0:] @ S64
            for tag, o in (("x3", out.cpu().numpy()), ("f32", outf.cpu().numpy()[r0:])):
                rb = np.abs(o - ref) / np.maximum(absb[r0:], 1e-300)
                print(f"[mf] {tag} N={N} K={K} r0={r0}: max |err|/(|M||S|) {rb.max():.3e}",
                      flush=True)


def probe_c5():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_configs_full_gpu import _c5_case

    from oracle import tree_ref as T
    from trex_amd import tree as G

    S, params, noise = _c5_case()
    n, L, Q = S.shape
    nl = (n + 1) // 2
    for gemm in ("x3", "f32"):
        opt = G.TreeOptimizer(_d(S), {k: _d(v) for k, v in params.items()}, lr=0.01, gemm=gemm)
        nz = _d(noise)
        p64 = {k: v.cpu().numpy().astype(np.float64) for k, v in opt.params.items()}
        opt.step(2.0, nz, next_temperature=2.0)
        torch.cuda.synchronize()
        S64 = T.update_seq(p64["ancestors"], S, 2.0)
        A64 = T.update_tree(p64["tree_params"], noise, 1.0)
        F = S64.reshape(n, -1)
        Gr = F @ F.T
        g = opt.G.cpu().numpy().astype(np.float64)
        rel = np.abs(g - Gr) / np.maximum(Gr, 1e-300)
        print(f"[c5] {gemm} Gram max elementwise rel {rel.max():.3e} (min entry {Gr.min():.3e})",
              flush=True)
        E = np.diag(Gr)
        cg = 2.0 * T.enforce_graph_constraints_grad(A64, 10.0)
        dA = 0.5 * (E[:, None] + E[None, :]) - Gr + cg
        bA = 0.5 * (E[:, None] + E[None, :]) + Gr + np.abs(cg)
        ea = np.abs(opt.dA.cpu().numpy() - dA) / bA
        print(f"[c5] {gemm} dA max |err|/(|terms|) {ea.max():.3e}", flush=True)
        rc = A64.sum(1) + A64.sum(0)
        AA = A64 + A64.T
        dF = rc[:, None] * F - AA @ F
        bF = np.abs(rc)[:, None] * np.abs(F) + np.abs(AA) @ np.abs(F)
        ds = opt.dS.cpu().numpy().reshape(n, -1).astype(np.float64)
        e = np.abs(ds[nl:] - dF[nl:]) / bF[nl:]
        print(f"[c5] {gemm} dS max |err|/(|terms|) {e.max():.3e}", flush=True)
        del opt, F, Gr, S64, dF, bF, ds, e
        torch.cuda.empty_cache()


if __name__ == "__main__":
    what = sys.argv[1:] or ["site", "marg", "gemm", "c5"]
    for w in what:
        {"marg": probe_marg, "site": probe_site, "gemm": probe_gemm, "c5": probe_c5}[w]()
