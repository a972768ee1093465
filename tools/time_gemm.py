"""HIP-event times of the C5 GEMM kernels (tools/prof.py gemm shapes) for the
library TREX_HIP_LIB points at: one line 'gram_us mf_us'."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    from trex_amd._lib import check, lib, ptr, stream_handle

    N, K, nl = 511, 200000, 256
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    S = torch.rand((N, K), device=dev, generator=g)
    M = torch.rand((N, N), device=dev, generator=g)
    G = torch.empty((N, N), device=dev)
    dS = torch.empty((N - nl, K), device=dev)
    ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=dev)
    st = stream_handle(dev)
    cs = torch.cuda.current_stream(dev)

    def timed(fn, reps=20):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cs)
        for _ in range(reps):
            fn()
        e1.record(cs)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    tg = timed(lambda: check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, nl, 1.0, ptr(G), ptr(ws),
                                                          ws.numel(), st)))
    tm = timed(lambda: check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, nl, N - nl,
                                                        float(N + 1), 1.0, ptr(dS), st)))
    print(os.environ.get("TREX_HIP_LIB", "default"), "gram %.1f us  mf %.1f us" % (tg, tm))
