"""C5-shape ancestors' pass (trex_adam_seq_update_step: update_seq VJP +
Adam + next update_seq) alone and after the MF (v3 / v5, x3 with leaf codes
and f32): HIP-event times."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    from trex_amd._lib import check, lib, ptr, stream_handle

    N, L, Q, nl = 511, 50000, 4, 256
    na = N - nl
    K = L * Q
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    S0 = torch.softmax(torch.randn((N, L, Q), device=dev, generator=g) * 3, dim=-1)
    codes = torch.randint(0, Q, (nl, L), device=dev, generator=g)
    S0[:nl] = torch.nn.functional.one_hot(codes, Q).float()
    S0 = S0.reshape(N, K).contiguous()
    M = torch.randn((N, N), device=dev, generator=g) * 50
    P0 = torch.randn((na, L, Q), device=dev, generator=g)
    mu0 = torch.randn((na, L, Q), device=dev, generator=g) * 1e-3
    nu0 = torch.rand((na, L, Q), device=dev, generator=g) * 1e-5
    cb = torch.empty(int(lib().trex_tree_leaf_codes_bytes(nl, L)), dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    st = stream_handle(dev)
    cs = torch.cuda.current_stream(dev)
    check(lib().trex_tree_leaf_codes(ptr(S0), nl, L, Q, ptr(cb), cb.numel(), ptr(status), st))
    torch.cuda.synchronize()
    mx = float(N + 1) * 50
    lr, b1, b2, eps, T, Tn = 0.01, 0.9, 0.999, 1e-8, 1.3, 1.2

    def state():
        return dict(S=S0.clone(), p=P0.clone(), mu=mu0.clone(), nu=nu0.clone(),
                    dS=torch.empty((na, K), device=dev))

    def pair(x3, ver, s):
        if ver:
            os.environ["TREX_MF"] = ver
        else:
            os.environ.pop("TREX_MF", None)
        if x3:
            check(lib().trex_tree_mf_rows_x3_codes(ptr(M), ptr(s["S"]), N, K, nl, na, mx, 1.0,
                                                   ptr(cb), cb.numel(), nl, Q, ptr(s["dS"]), st))
        else:
            check(lib().trex_tree_mf_rows(ptr(M), ptr(s["S"]), N, K, nl, na, ptr(s["dS"]), st))
        adam(s)

    def adam(s):
        check(lib().trex_adam_seq_update_step(ptr(s["dS"]), na, L, Q, T, Tn, ptr(s["p"]),
                                              ptr(s["mu"]), ptr(s["nu"]), 3, lr, b1, b2, eps,
                                              ptr(s["S"][nl:]), st))

    def timed(fn, reps=10):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for _ in range(reps):
            fn()
        e1.record(cs)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    sa = state()
    print(f"ancestors' pass: {timed(lambda: adam(sa), reps=20):.1f} us", flush=True)
    for x3 in (True, False):
        s = state()
        t_v3 = timed(lambda: pair(x3, "3", s)) if x3 else float("nan")
        t_v5 = timed(lambda: pair(x3, "5", s))
        os.environ.pop("TREX_MF", None)
        print(f"{'x3' if x3 else 'f32'}: MF v3 + pass {t_v3:.1f} us, MF v5 + pass {t_v5:.1f} us",
              flush=True)
