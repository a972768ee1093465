"""GPU parity of the tree-cost path (trex tree.py) vs the fp64 oracle.

Tolerances: f32 kernels vs fp64 oracle, rtol 1e-5 on losses; elementwise on
the GEMM outputs -- the Gram G = S S^T (a sum of non-negative terms) at rtol
1e-5 per entry, the mixed-sign products dS = M S and the surrogate's dS / dA
at 1e-5 times the sum of their terms' magnitudes per entry (|M| |S|,
tests/_cases.py surrogate_grad_bounds) -- for the f32 and the f16x3
split-product GEMMs alike; 1e-6 on elementwise softmaxes; exact for
integer-valued results (compute_cost, one-hot surrogate = edge Hamming
count).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from _cases import assert_bound_close, assert_grad_close, loss_grad_bounds, surrogate_grad_bounds
from oracle import tree_ref as T
from trex_amd import tree as G

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _t(x, device):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=torch.float32, device=device)


def _n(x):
    return x.detach().cpu().numpy().astype(np.float64)


def _tree_case(nl, L, Q, seed):
    rng = np.random.default_rng(seed)
    n = 2 * nl - 1
    n_anc = nl - 1
    params = {"tree_params": rng.normal(size=(n - 1, n_anc)).astype(np.float32),
              "ancestors": rng.normal(size=(n_anc, L, Q)).astype(np.float32)}
    noise = rng.gumbel(size=(n - 1, n_anc)).astype(np.float32)
    seqs = np.zeros((n, L, Q), np.float32)
    seqs[:nl] = np.eye(Q, dtype=np.float32)[rng.integers(0, Q, size=(nl, L))]
    return params, noise, seqs


def test_reference_tree_fixtures(device):
    """tests/test_tree.py:18-87 fixtures, exact values."""
    soft = np.array([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.3, 0.3, 0.4]], np.float32)
    oh = G.discretize_tree_topology(_t(soft, device), 3)
    np.testing.assert_array_equal(_n(oh), T.discretize_tree_topology(soft, 3))
    A = G.update_tree(_t(np.zeros((2, 1)), device), {"tree_params": _t(np.ones((2, 1)), device)})
    np.testing.assert_allclose(_n(A), T.update_tree(np.ones((2, 1))), rtol=1e-6)
    eye = G.update_tree(None, {"tree_params": torch.ones((1, 0), device=device)})
    np.testing.assert_array_equal(_n(eye), np.eye(2))
    assert float(G.enforce_graph_constraints(_t(np.eye(5), device), 10.0)) == 50.0
    seqs = np.eye(4, dtype=np.float32)[np.array([[0, 1, 2], [3, 2, 1]])]
    assert float(G.compute_surrogate_cost(_t(seqs, device), _t(np.eye(2), device))) == 0.0
    s3 = np.eye(2, dtype=np.float32)[np.array([[0, 1], [1, 0], [0, 0]])]
    c = float(G.compute_cost(_t(s3, device), _t(np.eye(3), device), _t(1 - np.eye(2), device)))
    assert c == 0.0


@pytest.mark.parametrize("T_", [1.0, 0.3, 2.0])
def test_update_seq_and_vjp(device, T_):
    params, _, seqs = _tree_case(8, 37, 4, 1)
    S = G.update_seq({"ancestors": _t(params["ancestors"], device)}, _t(seqs, device), T_)
    np.testing.assert_allclose(_n(S), T.update_seq(params["ancestors"], seqs, T_), rtol=1e-6,
                               atol=1e-7)


@pytest.mark.parametrize("nl,T_", [(4, 1.0), (16, 0.5), (100, 1.7)])
def test_update_tree(device, nl, T_):
    params, noise, _ = _tree_case(nl, 2, 4, nl)
    gates = (np.random.default_rng(3).random(noise.shape) > 0.2).astype(np.float32)
    for gt in (None, gates):
        A = G.update_tree(_t(noise, device), {"tree_params": _t(params["tree_params"], device)},
                          T_, None if gt is None else _t(gt, device))
        ref = T.update_tree(params["tree_params"], noise, T_, gt)
        np.testing.assert_allclose(_n(A), ref, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("N,L,Q", [(7, 3, 4), (15, 50, 4), (100, 33, 3), (129, 200, 4),
                                   (64, 1000, 20)])
def test_surrogate_value_and_grads(device, N, L, Q):
    rng = np.random.default_rng(N + L)
    S = rng.random((N, L, Q)).astype(np.float32)
    A = rng.random((N, N)).astype(np.float32)
    val, dS, dA = G.surrogate_cost_and_grads(_t(S, device), _t(A, device))
    rv, rdS, rdA = T.compute_surrogate_cost_grads(S, A)
    np.testing.assert_allclose(float(val), rv, rtol=RTOL)
    bS, bA = surrogate_grad_bounds(S, A)
    assert_bound_close(_n(dS), rdS, bS, what="dS")
    assert_bound_close(_n(dA), rdA, bA, what="dA")
    np.testing.assert_allclose(float(G.compute_surrogate_cost(_t(S, device), _t(A, device))), rv,
                               rtol=RTOL)


@pytest.mark.parametrize("nl,L", [(64, 2000), (16, 30)])  # (16, 30): the one-launch small path
def test_surrogate_onehot_is_edge_hamming_exact(device, nl, L):
    rng = np.random.default_rng(5)
    Q = 4
    n = 2 * nl - 1
    seq = rng.integers(0, Q, size=(n, L))
    S = np.eye(Q, dtype=np.float32)[seq]
    parent = np.concatenate([nl + np.arange(nl) // 2, nl + (np.arange(nl - 2) + nl) // 2, [n - 1]])
    A = np.eye(n, dtype=np.float32)[parent]
    A[-1] = 0
    ham = sum((seq[i] != seq[parent[i]]).sum() for i in range(n - 1))
    assert float(G.compute_surrogate_cost(_t(S, device), _t(A, device))) == ham
    A2 = np.eye(n, dtype=np.float32)[parent]
    C = (1 - np.eye(Q)).astype(np.float32)
    assert float(G.compute_cost(_t(S, device), _t(A2, device), _t(C, device))) == ham


@pytest.mark.parametrize("ckind", ["none", "diag", "matrix"])
def test_soft_cost(device, ckind):
    rng = np.random.default_rng(7)
    N, L, Q = 37, 41, 4
    S = rng.random((N, L, Q)).astype(np.float32)
    A = rng.random((N, N)).astype(np.float32)
    C = {"none": None, "diag": rng.random(Q).astype(np.float32),
         "matrix": rng.random((Q, Q)).astype(np.float32)}[ckind]
    got = G.compute_soft_cost(_t(S, device), _t(A, device), None if C is None else _t(C, device))
    np.testing.assert_allclose(float(got), T.compute_soft_cost(S, A, C), rtol=RTOL)


def test_compute_cost_random_labels(device):
    rng = np.random.default_rng(8)
    N, L, Q = 31, 500, 4
    S = rng.random((N, L, Q)).astype(np.float32)
    A = rng.random((N, N)).astype(np.float32)
    C = rng.integers(0, 5, size=(Q, Q)).astype(np.float32)
    assert float(G.compute_cost(_t(S, device), _t(A, device), _t(C, device))) == \
        T.compute_cost(S, A, C)


@pytest.mark.parametrize("fix", ["none", "seqs", "tree"])
def test_loss_and_grad_vs_oracle(device, fix):
    params, noise, seqs = _tree_case(16, 60, 4, 11)
    adj = T.discretize_tree_topology(T.update_tree(params["tree_params"], noise), 31)
    Tt = 0.8
    if fix == "seqs":
        seqs = T.update_seq(params["ancestors"], seqs, Tt).astype(np.float32)
    kw = dict(fix_seqs=fix == "seqs", fix_tree=fix == "tree")
    loss, grads = G.loss_and_grad(_t(noise, device),
                                  {k: _t(v, device) for k, v in params.items()},
                                  _t(seqs, device), Tt, _t(adj, device), **kw)
    rloss, rgrads = T.compute_loss(noise, params, seqs, Tt, adj, **kw)
    np.testing.assert_allclose(float(loss), rloss, rtol=RTOL)
    # per entry: 1e-5 of each gradient's terms' magnitudes, carried through
    # update_tree's / update_seq's softmax VJPs (tests/_cases.py loss_grad_bounds)
    bounds = loss_grad_bounds(noise, params, seqs, Tt, adj, rtol=RTOL, **kw)
    for k in ("tree_params", "ancestors"):
        assert_bound_close(_n(grads[k]), rgrads[k], bounds[k], what=k)


@pytest.mark.parametrize("clip", [None, 1.0])
def test_adam_matches_optax_semantics(device, clip):
    params, noise, seqs = _tree_case(8, 20, 4, 13)
    p_dev = {k: _t(v, device) for k, v in params.items()}
    p_ref = {k: v.astype(np.float64) for k, v in params.items()}
    opt = G.Adam(p_dev, lr=0.01, clip_norm=clip)
    st = T.adam_init(p_ref)
    for step in range(5):
        Tt = max(0.1, 2.0 * (1.0 - step / 5000))
        _, g = G.loss_and_grad(_t(noise, device), p_dev, _t(seqs, device), Tt, None)
        _, gr = T.compute_loss(noise, p_ref, seqs, Tt, None)
        opt.step(p_dev, g)
        upd, st = T.adam_update(gr, st, lr=0.01, clip_norm=clip)
        p_ref = {k: p_ref[k] + upd[k] for k in p_ref}
        for k in p_ref:
            np.testing.assert_allclose(_n(p_dev[k]), p_ref[k], rtol=2e-5, atol=2e-6)


def test_c5_scale_gram_properties(device):
    """C5 shape (256 taxa -> 511 nodes, 50 000 sites, 4 states): the Gram-based
    surrogate on one-hot sequences over a tree equals the edge Hamming count
    (every Gram entry is an exact integer; the 19 M total is returned as the
    correctly rounded f32), deterministic across runs."""
    rng = np.random.default_rng(21)
    nl, L, Q = 256, 50000, 4
    n = 2 * nl - 1
    seq = rng.integers(0, Q, size=(n, L)).astype(np.int64)
    S = torch.nn.functional.one_hot(torch.as_tensor(seq, device=device), Q).to(torch.float32)
    parent = np.concatenate([nl + np.arange(nl) // 2, nl + (np.arange(nl - 2) + nl) // 2, [n - 1]])
    A = np.eye(n, dtype=np.float32)[parent]
    A[-1] = 0
    ham = int(sum((seq[i] != seq[parent[i]]).sum() for i in range(n - 1)))
    v1, dS1, dA1 = G.surrogate_cost_and_grads(S, _t(A, device))
    v2, dS2, dA2 = G.surrogate_cost_and_grads(S, _t(A, device))
    assert float(v1) == float(np.float32(ham))
    assert torch.equal(dS1, dS2) and torch.equal(dA1, dA2)
    # dA_ij = (E_i + E_j)/2 - G_ij with one-hot rows: E = L, G_ij = #agreements
    i, j = 3, parent[3]
    agree = int((seq[i] == seq[j]).sum())
    assert float(dA1[i, j]) == L - agree


@pytest.mark.parametrize("gemm,L", [("x3", 52), ("f32", 52), ("x3", 51)])
def test_tree_optimizer_matches_oracle_loop(device, gemm, L):
    """The fused device loop == oracle compute_loss + adam, step by step
    (both GEMM precisions: f16x3 split products and f32 MFMA).  K = 208 is a
    multiple of 16; K = 204 leaves a ragged last 16-column chunk, which the
    x3 Gram masks (no silent fall back to f32)."""
    params, noise, seqs = _tree_case(16, L, 4, 17)
    opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01, gemm=gemm)
    assert opt.gemm == gemm
    p_ref = {k: v.astype(np.float64) for k, v in params.items()}
    st = T.adam_init(p_ref)
    nz = _t(noise, device)
    for step in range(6):
        Tt = max(0.1, 2.0 * (1.0 - step / 50))
        loss = opt.step(Tt, nz)
        rloss, gr = T.compute_loss(noise, p_ref, seqs, Tt, None)
        np.testing.assert_allclose(float(loss), rloss, rtol=RTOL)
        upd, st = T.adam_update(gr, st, lr=0.01)
        p_ref = {k: p_ref[k] + upd[k] for k in p_ref}
    for k in p_ref:
        np.testing.assert_allclose(_n(opt.params[k]), p_ref[k], rtol=5e-5, atol=5e-6)


def test_tree_optimizer_x3_needs_aligned_rows_and_says_so(device):
    """K = L*Q % 4 != 0 cannot feed the x3 GEMMs' 16-B row loads: the
    optimiser warns and runs the f32 GEMMs (never silently)."""
    params, noise, seqs = _tree_case(16, 33, 5, 3)  # K = 165
    with pytest.warns(RuntimeWarning, match="multiple of 4"):
        opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                              lr=0.01, gemm="x3")
    assert opt.gemm == "f32"


@pytest.fixture(params=["5", "3", "6"])
def gram_version(request, monkeypatch):
    """Every Gram / MF kernel version: v5 (one wave per SIMD; the f32 default),
    v3 (the x3 default), v6 (the x3 Gram at two waves per SIMD, A/B)."""
    monkeypatch.setenv("TREX_GRAM", request.param)
    monkeypatch.setenv("TREX_MF", request.param)
    return request.param


@pytest.mark.parametrize("N,L,r0", [(511, 1001, 256), (300, 257, 0), (64, 5, 0)])
def test_mf_v5_is_bitwise_v3(device, N, L, r0, monkeypatch):
    """MF v5 (one wave per SIMD) keeps v3's per-tile MFMA order (stages,
    then the two k-steps, f16x3 products in the same order): dS bitwise
    equal, with and without leaf codes."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    S_np, nl = _onehot_case(N, L, N + L)
    K = L * 4
    rng = np.random.default_rng(L)
    M = _t(rng.normal(size=(N, N)) * 20, device)
    S = _t(S_np, device)
    st = stream_handle(torch.device(device))
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, L)), dtype=torch.uint8, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    check(lib().trex_tree_leaf_codes(ptr(S), nl, L, 4, ptr(cb), cb.numel(), ptr(status), st))
    mx = float(M.abs().max()) * 1.01
    outs = {}
    for ver in ("3", "5"):
        monkeypatch.setenv("TREX_MF", ver)
        a = torch.empty((N - r0, K), device=device)
        b = torch.empty((N - r0, K), device=device)
        check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, r0, N - r0, mx, 1.0, ptr(a), st))
        check(lib().trex_tree_mf_rows_x3_codes(ptr(M), ptr(S), N, K, r0, N - r0, mx, 1.0, ptr(cb),
                                               cb.numel(), nl, 4, ptr(b), st))
        outs[ver] = (a, b)
    assert torch.equal(outs["5"][0], outs["3"][0])
    assert torch.equal(outs["5"][1], outs["3"][1])
    assert torch.equal(outs["5"][0], outs["5"][1])


@pytest.mark.parametrize("N,K,skip", [(511, 4096, 256), (511, 4096, 0), (300, 8192, 128),
                                      (511, 25000, 256), (511, 200000, 256), (64, 20, 0)])
def test_gram_x3_stays_inside_its_workspace(device, N, K, skip, gram_version):
    """The split-K Gram writes its partials only inside
    trex_tree_workspace_bytes(N, K) (a guard page of canary bytes after the
    workspace stays untouched) -- for the skipped and un-skipped tile plans,
    whose split counts differ, and both kernel versions (K = 200 000: C5)."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(K + skip)
    S = _t(rng.random((N, K)), device)
    nbytes = int(lib().trex_tree_workspace_bytes(N, K))
    guard = 1 << 20
    buf = torch.full((nbytes + guard,), 0xA5, dtype=torch.uint8, device=device)
    G = torch.zeros((N, N), device=device)
    check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, skip, 1.0, ptr(G), ptr(buf), nbytes,
                                       stream_handle(torch.device(device))))
    torch.cuda.synchronize()
    assert bool(torch.all(buf[nbytes:] == 0xA5))
    S64 = _n(S).astype(np.float64)
    t0 = (skip // 64) * 64
    ref = S64[t0:] @ S64.T
    assert_grad_close(_n(G)[t0:], ref, rtol=1e-5, what="G")  # non-negative sums: per entry


@pytest.mark.parametrize("Q", [4, 5])
def test_tree_optimizer_next_temperature_hint_is_bitwise_neutral(device, Q):
    """update_seq folded into the Adam kernel (trex_adam_seq_update_step,
    used when step() knows the next temperature) gives bitwise the same
    losses and parameters as recomputing S at the start of every step --
    including a wrong hint, which must only cost a recompute."""
    L = 48 if Q == 4 else 32  # K = 192 / 160
    params, noise, seqs = _tree_case(16, L, Q, 5)
    nz = _t(noise, device)
    temps = [2.0, 1.5, 1.5, 1.2, 0.9, 0.9]
    runs = []
    for mode in ("hint", "none", "wrong"):
        opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                              lr=0.01)
        losses = []
        for i, Tt in enumerate(temps):
            nxt = temps[i + 1] if i + 1 < len(temps) else Tt
            hint = {"hint": nxt, "none": None, "wrong": nxt + 0.25}[mode]
            losses.append(float(opt.step(Tt, nz, next_temperature=hint)))
        runs.append((losses, {k: v.clone() for k, v in opt.params.items()}))
    for losses, prm in runs[1:]:
        assert losses == runs[0][0]
        for k in prm:
            assert torch.equal(prm[k], runs[0][1][k])


@pytest.mark.parametrize("N,K,row0", [(511, 4096, 256), (100, 132, 37), (64, 64, 0)])
def test_mf_rows_equals_full_dS_slice(device, N, K, row0):
    """trex_tree_mf_rows (the optimiser's ancestor-rows-only dS = M S) is
    bit-identical to the corresponding rows of the full product."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(N + K)
    M = _t(rng.normal(size=(N, N)), device)
    S = _t(rng.normal(size=(N, K)), device)
    full = torch.empty((N, K), device=device)
    part = torch.empty((N - row0, K), device=device)
    st = stream_handle(torch.device(device))
    check(lib().trex_tree_mf(ptr(M), ptr(S), N, K, ptr(full), st))
    check(lib().trex_tree_mf_rows(ptr(M), ptr(S), N, K, row0, N - row0, ptr(part), st))
    assert torch.equal(part, full[row0:])
    M64, S64 = _n(M).astype(np.float64), _n(S)
    ref = M64 @ S64
    # f32 MFMA dS: per entry within 1e-5 of the sum of its terms' magnitudes
    assert_bound_close(_n(full), ref, 1e-5 * (np.abs(M64) @ np.abs(S64)), what="dS (f32 MF)")


@pytest.mark.parametrize("N,row0", [(199, 64), (511, 256), (130, 128), (64, 0), (64, 64)])
def test_gram_mirror_restores_symmetry(device, N, row0):
    """trex_tree_gram_mirror: after a site-sharded all-reduce of rows
    [row0, N) only, G[i][j] = G[j][i] for i < row0 <= j; the leaf x leaf
    block [0, row0)^2 and rows [row0, N) are untouched.  Starting from a full
    symmetric Gram whose upper-right block is garbage, the result equals the
    full Gram bitwise."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(N + row0)
    S = rng.random((N, 40))
    full = _t(S @ S.T, device)
    G = full.clone()
    G[:row0, row0:] = -3.0
    check(lib().trex_tree_gram_mirror(ptr(G), N, row0, stream_handle(torch.device(device))))
    assert torch.equal(G, full)


def test_gram_skip_keeps_cached_block(device):
    """trex_tree_gram_skip recomputes every tile except the leading constant
    block, which keeps its previous contents (the optimiser's cached
    leaf x leaf Gram); the other entries equal the full Gram bitwise."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(3)
    N, K, skip = 300, 1024, 130  # tiles 0-1 (rows < 128) skipped
    S = _t(rng.random((N, K)), device)
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=device)
    st = stream_handle(torch.device(device))
    full = torch.empty((N, N), device=device)
    check(lib().trex_tree_gram(ptr(S), N, K, ptr(full), ptr(ws), ws.numel(), st))
    G = torch.full((N, N), -7.0, device=device)
    check(lib().trex_tree_gram_skip(ptr(S), N, K, skip, ptr(G), ptr(ws), ws.numel(), st))
    t0 = (skip // 64) * 64
    assert torch.all(G[:t0, :t0] == -7.0)
    mask = torch.ones((N, N), dtype=torch.bool, device=device)
    mask[:t0, :t0] = False
    assert torch.equal(G[mask], full[mask])


@pytest.mark.parametrize("N,K,skip", [(511, 4096, 256), (511, 4096, 0), (300, 160, 130),
                                      (100, 1024, 0), (64, 16, 0), (511, 25000, 256),
                                      (300, 1028, 130), (64, 20, 0)])
def test_split_gram_and_mf_vs_fp64(device, N, K, skip, gram_version):
    """f16x3 split-product Gram / MF (trex_tree_gram_skip_x3 /
    trex_tree_mf_rows_x3) vs fp64 at the f32 path's bar: softmax-like S
    (values spanning 1e-6 .. 1, one-hot rows) and M = diag(r+c) - (A+A^T)
    with softmax rows of A.  K = 25 000 is one rank's C5 site shard at N = 8
    (6 250 sites x 4): K % 16 = 8, a ragged last chunk, like 1 028 and 20."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(N + K)
    logits = rng.normal(scale=3.0, size=(N, K // 4, 4))
    P = np.exp(logits - logits.max(-1, keepdims=True))
    P /= P.sum(-1, keepdims=True)
    P[: N // 3] = np.eye(4)[rng.integers(0, 4, size=(N // 3, K // 4))]  # one-hot leaf rows
    S = P.reshape(N, K).astype(np.float32)
    Al = rng.normal(size=(N, N))
    A = np.exp(Al - Al.max(1, keepdims=True))
    A /= A.sum(1, keepdims=True)
    M = (np.diag(A.sum(1) + A.sum(0)) - (A + A.T)).astype(np.float32)
    St, Mt = _t(S, device), _t(M, device)
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=device)
    st = stream_handle(torch.device(device))
    Gx = torch.zeros((N, N), device=device)
    check(lib().trex_tree_gram_skip_x3(ptr(St), N, K, skip, 1.0, ptr(Gx), ptr(ws), ws.numel(), st))
    S64 = S.astype(np.float64)
    Gref = S64 @ S64.T
    t0 = (skip // 64) * 64
    mask = np.ones((N, N), bool)
    mask[:t0, :t0] = False
    # every Gram entry is a sum of non-negative terms: rtol 1e-5 per entry
    assert_grad_close(_n(Gx)[mask], Gref[mask], rtol=1e-5, what="G (x3)")
    absb = np.abs(M.astype(np.float64)) @ np.abs(S64)
    for r0 in (N // 2, 0):  # 0: more than 256 output rows for N = 511 / 300
        out = torch.empty((N - r0, K), device=device)
        check(lib().trex_tree_mf_rows_x3(ptr(Mt), ptr(St), N, K, r0, N - r0, float(N + 1), 1.0,
                                         ptr(out), st))
        ref = M.astype(np.float64)[r0:] @ S64
        assert_bound_close(_n(out), ref, 1e-5 * absb[r0:], what="dS (x3 MF)")


@pytest.mark.parametrize("Q,L", [(4, 300), (5, 33)])
def test_adam_seq_step_fused_is_bitwise_separate(device, Q, L):
    """trex_adam_seq_step == trex_tree_update_seq_bwd + trex_adam_step, bitwise."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(Q * L)
    n_anc, T_ = 7, 1.3
    x = rng.normal(size=(n_anc, L, Q))
    s_anc = _t(np.exp(x) / np.exp(x).sum(-1, keepdims=True), device)
    ds = _t(rng.normal(size=(n_anc, L, Q)), device)
    p0 = _t(rng.normal(size=(n_anc, L, Q)), device)
    m0 = _t(rng.normal(size=(n_anc, L, Q)) * 0.1, device)
    v0 = _t(rng.random((n_anc, L, Q)) * 0.1, device)
    st = stream_handle(torch.device(device))
    L_ = lib()
    pa, ma, va = p0.clone(), m0.clone(), v0.clone()
    g = torch.empty_like(p0)
    check(L_.trex_tree_update_seq_bwd(ptr(s_anc), ptr(ds), n_anc, L, Q, T_, ptr(g), st))
    check(L_.trex_adam_step(ptr(pa), ptr(g), ptr(ma), ptr(va), pa.numel(), 3, 0.01, 0.9, 0.999,
                            1e-8, None, 0, 0.0, st))
    pb, mb, vb = p0.clone(), m0.clone(), v0.clone()
    gb = torch.empty_like(p0)
    check(L_.trex_adam_seq_step(ptr(s_anc), ptr(ds), n_anc, L, Q, T_, ptr(pb), ptr(mb), ptr(vb),
                                3, 0.01, 0.9, 0.999, 1e-8, ptr(gb), st))
    assert torch.equal(g, gb) and torch.equal(pa, pb) and torch.equal(ma, mb)
    assert torch.equal(va, vb)


@pytest.mark.parametrize("N,K,skip,x3", [(511, 4096, 0, True), (300, 8192, 128, True),
                                         (511, 4096, 0, False), (200, 1024, 0, False),
                                         (511, 200000, 256, True)])
def test_gram_is_run_to_run_deterministic(device, N, K, skip, x3):
    """The split-K Grams give bitwise the same symmetric G on every run: the
    reduce writes each mirrored pair of a diagonal tile from one thread only
    (two threads holding the (i, j) and (j, i) partial sums used to race)."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    rng = np.random.default_rng(N + K)
    x = rng.normal(size=(N, K // 4, 4)) * 3
    e = np.exp(x - x.max(-1, keepdims=True))
    S = _t((e / e.sum(-1, keepdims=True)).reshape(N, K), device)
    st = stream_handle(torch.device(device))
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=device)
    runs = []
    for _ in range(4):
        G = torch.empty((N, N), device=device)
        if x3:
            check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, skip, 1.0, ptr(G), ptr(ws),
                                               ws.numel(), st))
        else:
            check(lib().trex_tree_gram_skip(ptr(S), N, K, skip, ptr(G), ptr(ws), ws.numel(), st))
        runs.append(G)
    t0 = (skip // 64) * 64
    for G in runs[1:]:
        assert torch.equal(G[t0:], runs[0][t0:])
    assert torch.equal(runs[0][t0:, t0:], runs[0][t0:, t0:].T)


def _onehot_case(N, L, seed, Q=4):
    rng = np.random.default_rng(seed)
    nl = (N + 1) // 2
    x = rng.normal(size=(N, L, Q)) * 3
    S = np.exp(x - x.max(-1, keepdims=True))
    S /= S.sum(-1, keepdims=True)
    S[:nl] = np.eye(Q)[rng.integers(0, Q, size=(nl, L))]
    return S.reshape(N, L * Q).astype(np.float32), nl


@pytest.mark.parametrize("N,L,skip", [(511, 1001, 256), (511, 2048, 0), (300, 257, 128),
                                      (101, 77, 0), (127, 50, 64)])
def test_leaf_code_gram_is_bitwise_the_x3p_gram(device, N, L, skip):
    """trex_tree_gram_skip_x3p_codes (the leaf strips' zero lo-plane
    products skipped) == trex_tree_gram_skip_x3p bit for bit -- skipped and
    un-skipped leaf x leaf tiles, n_leaf not a multiple of 32 (N = 101: 51
    leaves, one code strip), a ragged last K chunk -- and vs fp64."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    Sn, nl = _onehot_case(N, L, 3 * N + L)
    K = L * 4
    S = _t(Sn, device)
    st = stream_handle(torch.device(device))
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, L)), dtype=torch.uint8, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    check(lib().trex_tree_leaf_codes(ptr(S), nl, L, 4, ptr(cb), cb.numel(), ptr(status), st))
    assert int(status.item()) == 0
    S16 = torch.empty_like(S)
    check(lib().trex_tree_split_x3(ptr(S), N, K, K, 1.0, ptr(S16), K, st))
    nbytes = int(lib().trex_tree_workspace_bytes(N, K))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
    Ga = torch.zeros((N, N), device=device)
    Gb = torch.zeros((N, N), device=device)
    check(lib().trex_tree_gram_skip_x3p(ptr(S16), N, K, skip, 1.0, ptr(Ga), ptr(ws), nbytes, st))
    check(lib().trex_tree_gram_skip_x3p_codes(ptr(S16), N, K, skip, 1.0, ptr(cb), cb.numel(), nl,
                                              4, ptr(Gb), ptr(ws), nbytes, st))
    torch.cuda.synchronize()
    assert torch.equal(Ga, Gb)
    t0 = (skip // 64) * 64
    S64 = Sn.astype(np.float64)
    assert_grad_close(_n(Gb)[t0:], S64[t0:] @ S64.T, rtol=1e-5, what="G")


@pytest.mark.parametrize("N,L", [(511, 1001), (511, 2048), (255, 333), (383, 64), (127, 50),
                                 (101, 77)])
def test_leaf_code_mf_is_bitwise_the_x3_mf(device, N, L):
    """trex_tree_mf_rows_x3_codes (leaf rows read as codes, one-hot x scale
    exact in f16) == trex_tree_mf_rows_x3 on the f32 rows bit for bit --
    ragged last column tile, both column-tile widths, n_leaf not a multiple
    of 32 (N = 101: 51 leaves, 32 code rows) -- and both vs fp64."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    Sn, nl = _onehot_case(N, L, N + L)
    K = L * 4
    S = _t(Sn, device)
    st = stream_handle(torch.device(device))
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, L)), dtype=torch.uint8, device=device)
    status = torch.full((1,), 7, dtype=torch.int32, device=device)
    check(lib().trex_tree_leaf_codes(ptr(S), nl, L, 4, ptr(cb), cb.numel(), ptr(status), st))
    Mn = np.random.default_rng(N).normal(size=(N, N)) * 20
    M = _t(Mn, device)
    n_anc = N - nl
    d0 = torch.empty((n_anc, K), device=device)
    d1 = torch.empty((n_anc, K), device=device)
    mx = float(np.abs(_n(M)).max())
    check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, nl, n_anc, mx, 1.0, ptr(d0), st))
    check(lib().trex_tree_mf_rows_x3_codes(ptr(M), ptr(S), N, K, nl, n_anc, mx, 1.0, ptr(cb),
                                           cb.numel(), nl, 4, ptr(d1), st))
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    assert torch.equal(d0, d1)
    ref = _n(M)[nl:].astype(np.float64) @ Sn.astype(np.float64)
    assert_bound_close(_n(d1), ref, 1e-5 * (np.abs(_n(M)[nl:]) @ np.abs(Sn.astype(np.float64))),
                       what="dS (leaf codes)")


def test_leaf_codes_flag_rows_that_are_not_one_hot(device):
    """A leaf row that is not exactly one-hot sets the status word, and the
    optimiser then keeps the f32-row GEMMs."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    Sn, nl = _onehot_case(127, 40, 3)
    Sn[5, 7] = 0.5  # site 1 of leaf 5: not one-hot
    S = _t(Sn, device)
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, 40)), dtype=torch.uint8, device=device)
    status = torch.zeros(1, dtype=torch.int32, device=device)
    check(lib().trex_tree_leaf_codes(ptr(S), nl, 40, 4, ptr(cb), cb.numel(), ptr(status),
                                     stream_handle(torch.device(device))))
    torch.cuda.synchronize()
    assert int(status.item()) == 1
    params, _, _ = _tree_case(nl, 40, 4, 1)
    opt = G.TreeOptimizer(S.reshape(127, 40, 4), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01)
    assert opt.gemm == "x3" and opt.codes is None


def test_tree_optimizer_leaf_codes_are_bitwise_neutral(device, monkeypatch):
    """TreeOptimizer with leaf codes (the default for one-hot leaves, Q = 4)
    == TREX_LEAF_CODES=0 (f32 leaf rows) bit for bit, loss and parameters."""
    params, noise, seqs = _tree_case(100, 50, 4, 9)  # 96 code rows + 4 f32 leaf rows
    nz = _t(noise, device)
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TREX_LEAF_CODES", flag)
        opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                              lr=0.01)
        assert (opt.codes is not None) == (flag == "1")
        losses = [float(opt.step(max(0.2, 1.5 - 0.2 * i), nz)) for i in range(4)]
        runs.append((losses, {k: v.clone() for k, v in opt.params.items()}))
    assert runs[0][0] == runs[1][0]
    for k in runs[0][1]:
        assert torch.equal(runs[0][1][k], runs[1][1][k])


@pytest.mark.parametrize("gemm,capture", [("x3", True), ("f32", True), ("x3", False)])
def test_tree_device_loop_is_bitwise_eager(device, gemm, capture):
    """TreeOptimizer.device_loop (count, annealed temperature and Gumbel noise
    on the device; one step captured in a hipGraph and replayed) == eager
    step(T_k, gumbel_noise_step(seed, k), T_{k+1}) for k = 1..5, bitwise:
    losses, tree params and ancestor logits -- including after 2 eager steps
    (the device count continues the host one)."""
    params, _, seqs = _tree_case(16, 52, 4, 19)
    temps = [max(0.1, 2.0 * (1.0 - k / 50)) for k in range(12)]
    seed = 1234
    ref = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01, gemm=gemm)
    dut = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01, gemm=gemm)
    shape = (ref.N - 1, ref.n_anc)
    for k in range(1, 3):  # both start with two eager steps
        for o in (ref, dut):
            o.step(temps[k - 1], G.gumbel_noise_step(seed, k, shape, device), temps[k])
    loop = dut.device_loop(temps, seed, capture=capture)
    losses = []
    for k in range(3, 8):
        losses.append(float(ref.step(temps[k - 1], G.gumbel_noise_step(seed, k, shape, device),
                                     temps[k])))
        assert float(loop.run(1)) == losses[-1], k
    torch.cuda.synchronize()
    assert dut.opt.count == ref.opt.count == 7
    for k in ref.params:
        assert torch.equal(dut.params[k], ref.params[k]), k
    # the device noise is trex_gumbel_noise's restatement (oracle/datagen_ref.py)
    from oracle.datagen_ref import gumbel_noise

    np.testing.assert_allclose(_n(G.gumbel_noise_step(seed, 3, shape, device)).ravel(),
                               gumbel_noise(seed, 3, shape[0] * shape[1]), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("gemm", ["x3", "f32"])
def test_tree_optimizer_checkpoint_resume_is_bitwise(device, gemm, tmp_path):
    """save_checkpoint after 3 steps, load into a fresh TreeOptimizer (same
    leaves), 3 more steps: losses and parameters bitwise those of the
    uninterrupted 6-step run (SURVEY.md §5 checkpoint / resume: params and
    the Adam state; S and the Gram are recomputed)."""
    params, noise, seqs = _tree_case(16, 52, 4, 23)
    nz = _t(noise, device)
    temps = [2.0, 1.8, 1.6, 1.4, 1.2, 1.0, 0.9]

    def make():
        return G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                               lr=0.02, gemm=gemm)

    ref = make()
    ref_losses = [float(ref.step(temps[i], nz, temps[i + 1])) for i in range(6)]
    first = make()
    for i in range(3):
        first.step(temps[i], nz, temps[i + 1])
    path = tmp_path / "c5.npz"
    first.save_checkpoint(path)
    resumed = make()
    resumed.load_checkpoint(path)
    assert resumed.opt.count == 3
    losses = [float(resumed.step(temps[i], nz, temps[i + 1])) for i in range(3, 6)]
    assert losses == ref_losses[3:]
    for k in ref.params:
        assert torch.equal(resumed.params[k], ref.params[k]), k
    for k in ref.opt.mu:
        assert torch.equal(resumed.opt.mu[k], ref.opt.mu[k]) and torch.equal(resumed.opt.nu[k],
                                                                            ref.opt.nu[k]), k



@pytest.mark.parametrize("dev_state", [False, True])
def test_fused_step_entries_are_bitwise_separate(device, dev_state):
    """trex_tree_surrogate_constraint == trex_tree_surrogate_combine +
    trex_tree_constraint[_dev] (accumulate), and trex_tree_update_tree_bwd_adam
    == trex_tree_update_tree_bwd + trex_adam_step[_dev], bit for bit (loss,
    dA, M; gradient, params, moments), with host or device-state counts."""
    from trex_amd._lib import check, lib, ptr, stream_handle

    nl = 40
    N, na = 2 * nl - 1, nl - 1
    g = torch.Generator(device=device).manual_seed(3)
    A = torch.softmax(torch.randn((N, N), device=device, generator=g) * 2, dim=1).contiguous()
    Gm = torch.rand((N, N), device=device, generator=g) * 100
    Gm = (Gm + Gm.T).contiguous()
    dA0 = torch.randn((N, N), device=device, generator=g)
    th0 = torch.randn((N - 1, na), device=device, generator=g)
    mu0 = torch.randn((N - 1, na), device=device, generator=g) * 1e-2
    nu0 = torch.rand((N - 1, na), device=device, generator=g) * 1e-3
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=device)
    st = stream_handle(device)
    T, count, scale = 0.7, 4, 10.0
    state = s_ptr = None
    if dev_state:
        state = torch.zeros(8, dtype=torch.int32, device=device)
        state[0] = count - 1
        check(lib().trex_step_advance(ptr(state), 0.9, 0.999, ptr(torch.tensor([T] * 8, device=device)),
                                      8, st))
        s_ptr = ptr(state)
    out = []
    for fused in (False, True):
        loss = torch.zeros(1, device=device)
        dA = torch.empty_like(dA0)
        M = torch.empty_like(dA0)
        if fused:
            check(lib().trex_tree_surrogate_constraint(ptr(A), ptr(Gm), N, scale, T, s_ptr,
                                                       ptr(loss), ptr(dA), ptr(M), 0.0, None, 0,
                                                       ptr(ws), st))
        else:
            check(lib().trex_tree_surrogate_combine(ptr(A), ptr(Gm), N, ptr(loss), ptr(dA), ptr(M),
                                                    ptr(ws), st))
            if dev_state:
                check(lib().trex_tree_constraint_dev(ptr(A), N, scale, s_ptr, ptr(loss), 1,
                                                     ptr(dA), ptr(ws), st))
            else:
                check(lib().trex_tree_constraint(ptr(A), N, scale, T, ptr(loss), 1, ptr(dA),
                                                 ptr(ws), st))
        th, mu, nu = th0.clone(), mu0.clone(), nu0.clone()
        gr = torch.empty_like(th0)
        if fused:
            check(lib().trex_tree_update_tree_bwd_adam(ptr(A), ptr(dA0), None, N, na, 1.3, ptr(gr),
                                                       ptr(th), ptr(mu), ptr(nu), count, s_ptr,
                                                       0.01, 0.9, 0.999, 1e-8, st))
        else:
            check(lib().trex_tree_update_tree_bwd(ptr(A), ptr(dA0), None, N, na, 1.3, ptr(gr), st))
            if dev_state:
                check(lib().trex_adam_step_dev(ptr(th), ptr(gr), ptr(mu), ptr(nu), th.numel(),
                                               s_ptr, 0.01, 0.9, 0.999, 1e-8, None, 0, 0.0, st))
            else:
                check(lib().trex_adam_step(ptr(th), ptr(gr), ptr(mu), ptr(nu), th.numel(), count,
                                           0.01, 0.9, 0.999, 1e-8, None, 0, 0.0, st))
        torch.cuda.synchronize()
        out.append((loss, dA, M, gr, th, mu, nu))
    for a, b, name in zip(out[0], out[1], ("loss", "dA", "M", "grad", "params", "mu", "nu")):
        assert torch.equal(a, b), name


def test_tree_device_loop_after_more_eager_steps(device):
    """A captured device loop, then eager steps (which count on the host
    only), then the same loop again: bitwise the all-eager run (the loop
    re-syncs the device step record in place before replaying)."""
    params, _, seqs = _tree_case(16, 52, 4, 31)
    temps = [max(0.1, 2.0 * (1.0 - k / 50)) for k in range(14)]
    seed = 99
    ref = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01)
    dut = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                          lr=0.01)
    shape = (ref.N - 1, ref.n_anc)

    def eager(o, k):
        return float(o.step(temps[k - 1], G.gumbel_noise_step(seed, k, shape, device), temps[k]))

    loop = dut.device_loop(temps, seed, capture=True)
    for k in range(1, 4):
        assert float(loop.run(1)) == eager(ref, k), k
    for k in range(4, 6):
        assert eager(dut, k) == eager(ref, k), k
    for k in range(6, 9):
        assert float(loop.run(1)) == eager(ref, k), k
    torch.cuda.synchronize()
    for k in ref.params:
        assert torch.equal(dut.params[k], ref.params[k]), k


@pytest.mark.parametrize("gemm", ["x3", "f32"])
def test_tree_device_loop_after_load_checkpoint(device, gemm, tmp_path):
    """a captured loop replays with S's (S16's) ancestor rows as
    the previous replay left them.  Load an earlier checkpoint into the
    looping optimiser, and then take an eager step whose next temperature
    leaves the schedule: each time run() must first refresh the rows, so
    the replays stay bitwise an uninterrupted eager run from that state."""
    params, _, seqs = _tree_case(16, 52, 4, 37)
    temps = [max(0.1, 2.0 * (1.0 - k / 40)) for k in range(16)]
    seed = 7

    def make():
        return G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                               lr=0.02, gemm=gemm)

    shape = None

    def eager(o, k, t_next=None):
        return float(o.step(temps[k - 1], G.gumbel_noise_step(seed, k, shape, device),
                            temps[k] if t_next is None else t_next))

    ref = make()
    shape = (ref.N - 1, ref.n_anc)
    dut = make()
    loop = dut.device_loop(temps, seed, capture=True)
    loop.run(2)
    path = tmp_path / "c5.npz"
    dut.save_checkpoint(path)  # after step 2
    loop.run(3)  # steps 3..5: the rows now belong to step 6
    dut.load_checkpoint(path)  # back to step 2's state
    for k in (1, 2):
        eager(ref, k)
    for k in (3, 4):
        assert float(loop.run(1)) == eager(ref, k), k
    # an eager step announcing a temperature off the schedule
    assert eager(dut, 5, 0.77) == eager(ref, 5, 0.77)
    for k in (6, 7):
        assert float(loop.run(1)) == eager(ref, k), k
    torch.cuda.synchronize()
    for k in ref.params:
        assert torch.equal(dut.params[k], ref.params[k]), k


def test_tree_optimizer_sequences_accessor(device, monkeypatch):
    """TreeOptimizer.sequences(): the current softmaxes in every mode.  In
    pre-split mode S's ancestor rows go stale (only S16's are kept); the
    accessor recomputes them, equal bit for bit to the f32-operand mode's S."""
    params, noise, seqs = _tree_case(16, 52, 4, 43)
    nz = _t(noise, device)
    temps = [1.5, 1.2, 1.0, 0.8]
    got = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TREX_PRESPLIT", flag)
        opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                              lr=0.02)
        for i in range(3):
            opt.step(temps[i], nz, temps[i + 1])
        got.append(opt.sequences())
        if flag == "0":
            assert torch.equal(got[-1], opt.S)
    assert torch.equal(got[0], got[1])


@pytest.mark.parametrize("nl,L,loop", [(100, 50, False), (256, 1001, False), (16, 52, True),
                                       (40, 33, False)])
def test_tree_optimizer_presplit_operands_are_bitwise_neutral(device, monkeypatch, nl, L, loop):
    """x3 with pre-split GEMM operands (S16 / M16: trex_tree_split_x3,
    trex_tree_gram_skip_x3p, trex_tree_mf_rows_x3p, the ancestors' pass
    writing S16; the default) == TREX_PRESPLIT=0 (the GEMMs split f32
    operands) bit for bit: losses, parameters and moments, eager or in the
    captured device loop, with leaf codes (nl = 100: 96 code rows + 4 f32
    rows), a ragged last column chunk (L = 1001) and no code rows (nl = 16)."""
    params, noise, seqs = _tree_case(nl, L, 4, 41)
    nz = _t(noise, device)
    temps = [max(0.1, 2.0 * (1.0 - k / 20)) for k in range(12)]
    runs = []
    for flag in ("1", "0"):
        monkeypatch.setenv("TREX_PRESPLIT", flag)
        opt = G.TreeOptimizer(_t(seqs, device), {k: _t(v, device) for k, v in params.items()},
                              lr=0.02)
        assert opt.presplit == (flag == "1")
        if loop:
            opt.step(temps[0], nz, temps[1])
            lp = opt.device_loop(temps, 5, capture=True)
            losses = [float(lp.run(1)) for _ in range(4)]
            losses.append(float(opt.step(temps[5], nz, temps[7])))  # a temperature jump
        else:
            losses = [float(opt.step(temps[i], nz, temps[i + 1])) for i in range(3)]
            losses.append(float(opt.step(temps[5], nz, temps[6])))
        torch.cuda.synchronize()
        runs.append((losses, {k: v.clone() for k, v in opt.params.items()},
                     {k: v.clone() for k, v in opt.opt.mu.items()},
                     {k: v.clone() for k, v in opt.opt.nu.items()}))
    a, b = runs
    assert a[0] == b[0]
    for i in (1, 2, 3):
        for k in a[i]:
            assert torch.equal(a[i][k], b[i][k]), (i, k)


def test_update_tree_and_compute_loss_take_a_key(device):
    """The reference's key arguments (update_tree tree.py:71, compute_loss
    tree.py:337): a PRNGKey draws the Gumbel noise on the device; the same
    key gives the same adjacency, compute_loss splits the key as the
    reference does (the second half draws update_tree's noise)."""
    params, _, seqs = _tree_case(16, 20, 4, 3)
    p = {k: _t(v, device) for k, v in params.items()}
    key = G.PRNGKey(42)
    shape = (params["tree_params"].shape[0], params["tree_params"].shape[1])
    a1 = G.update_tree(key, p)
    a2 = G.update_tree(G.gumbel(key, shape, device), p)
    a3 = G.update_tree(G.PRNGKey(42), p)
    assert torch.equal(a1, a2) and torch.equal(a1, a3)
    assert not torch.equal(a1, G.update_tree(G.PRNGKey(43), p))
    noise = G.gumbel(G.split(key)[1], shape, device)
    l_key = float(G.compute_loss(key, p, _t(seqs, device), None, 0.7, None))
    l_noise = float(G.compute_loss(noise, p, _t(seqs, device), None, 0.7, None))
    assert l_key == l_noise
    rl, _ = T.compute_loss(_n(noise), params, seqs, 0.7, None)
    np.testing.assert_allclose(l_key, rl, rtol=RTOL)
