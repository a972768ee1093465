"""C5 MF with and without leaf codes (trex_tree_leaf_codes): bitwise
equality of dS, HIP-event times of both paths (and of the Gram)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    from trex_amd._lib import check, lib, ptr, stream_handle

    N, L, Q, nl = 511, 50000, 4, 256
    K = L * Q
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    S = torch.softmax(torch.randn((N, L, Q), device=dev, generator=g) * 3, dim=-1)
    codes = torch.randint(0, Q, (nl, L), device=dev, generator=g)
    S[:nl] = torch.nn.functional.one_hot(codes, Q).float()
    S = S.reshape(N, K).contiguous()
    M = torch.randn((N, N), device=dev, generator=g) * 50
    G0 = torch.zeros((N, N), device=dev)
    d0, d1 = torch.empty((N - nl, K), device=dev), torch.empty((N - nl, K), device=dev)
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=dev)
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, L)), dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    st = stream_handle(dev)
    cs = torch.cuda.current_stream(dev)
    check(lib().trex_tree_leaf_codes(ptr(S), nl, L, Q, ptr(cb), cb.numel(), ptr(status), st))
    torch.cuda.synchronize()
    assert int(status.item()) == 0, "leaf rows not one-hot?"

    def timed(fn, reps=20):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for _ in range(reps):
            fn()
        e1.record(cs)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    mx = float(N + 1) * 50

    def setv(gram=None, mf=None):
        for key, v in (("TREX_GRAM", gram), ("TREX_MF", mf)):
            if v is None:
                os.environ.pop(key, None)
            else:
                os.environ[key] = v

    # x3 Gram: every kernel version (v3 default, v5 one wave per SIMD, v6 two)
    gx = {}
    for ver in ("3", "5", "6"):
        setv(gram=ver)
        Gv = torch.zeros((N, N), device=dev)
        tv = timed(lambda: check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, nl, 1.0, ptr(Gv),
                                                              ptr(ws), ws.numel(), st)))
        gx[ver] = (tv, Gv)
    G3 = gx["3"][1]
    for ver in ("5", "6"):
        gd = ((gx[ver][1] - G3).abs()[nl:] / G3.abs()[nl:].clamp_min(1e-30)).max().item()
        print(f"x3 gram v{ver} {gx[ver][0]:.1f} us vs v3 {gx['3'][0]:.1f} us (max rel diff {gd:.3g})")
    # x3 MF (f32 rows, leaf codes): v3 default, v5
    mfx = {}
    for ver in ("3", "5"):
        setv(mf=ver)
        tm0 = timed(lambda: check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, nl, N - nl, mx,
                                                             1.0, ptr(d0), st)))
        tm1 = timed(lambda: check(lib().trex_tree_mf_rows_x3_codes(ptr(M), ptr(S), N, K, nl,
                                                                   N - nl, mx, 1.0, ptr(cb),
                                                                   cb.numel(), nl, 4, ptr(d1),
                                                                   st)))
        mfx[ver] = (tm0, tm1, torch.equal(d0, d1), d1.clone())
    print(f"x3 mf v3 {mfx['3'][0]:.1f} us (codes {mfx['3'][1]:.1f}), v5 {mfx['5'][0]:.1f} us "
          f"(codes {mfx['5'][1]:.1f}); codes bitwise rows {mfx['3'][2]} / {mfx['5'][2]}; "
          f"v5 == v3 {torch.equal(mfx['3'][3], mfx['5'][3])}")
    # exact f32 GEMMs (TreeOptimizer(gemm="f32")): v5 default against the older kernels
    f32 = {}
    for ver in ("5", "3"):
        setv(gram=ver, mf=ver)
        Gf = torch.zeros((N, N), device=dev)
        df = torch.empty((N - nl, K), device=dev)
        tg = timed(lambda: check(lib().trex_tree_gram_skip(ptr(S), N, K, nl, ptr(Gf), ptr(ws),
                                                           ws.numel(), st)))
        tm = timed(lambda: check(lib().trex_tree_mf_rows(ptr(M), ptr(S), N, K, nl, N - nl,
                                                         ptr(df), st)))
        f32[ver] = (tg, tm, Gf, df)
    setv()
    gr = ((f32["5"][2] - f32["3"][2]).abs()[nl:] / f32["3"][2].abs()[nl:].clamp_min(1e-30)).max()
    mr = ((f32["5"][3] - f32["3"][3]).abs() / (M[nl:].abs() @ S.abs()).clamp_min(1e-30)).max()
    print(f"f32 gram v5 {f32['5'][0]:.1f} us  v3 {f32['3'][0]:.1f} us (max rel diff {gr.item():.3g}); "
          f"f32 mf v5 {f32['5'][1]:.1f} us  old {f32['3'][1]:.1f} us (max diff / |M||S| {mr.item():.3g})")
