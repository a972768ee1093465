"""C5-shape GEMM kernels alone (for rocprofv3 --pmc passes): the f16x3 Gram
(trex_tree_gram_skip_x3, leaf block skipped) and ancestor-rows MF
(trex_tree_mf_rows_x3), then the f32 ones (trex_tree_gram_skip /
trex_tree_mf_rows), at N = 511, K = 50 000 x 4, a few launches each."""
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
    for _ in range(int(os.environ.get("ITERS", "3"))):
        check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, nl, 1.0, ptr(G), ptr(ws), ws.numel(), st))
        check(lib().trex_tree_mf_rows_x3(ptr(M), ptr(S), N, K, nl, N - nl, float(N + 1), 1.0,
                                         ptr(dS), st))
        # the exact f32 GEMMs (TreeOptimizer(gemm="f32"))
        check(lib().trex_tree_gram_skip(ptr(S), N, K, nl, ptr(G), ptr(ws), ws.numel(), st))
        check(lib().trex_tree_mf_rows(ptr(M), ptr(S), N, K, nl, N - nl, ptr(dS), st))
    torch.cuda.synchronize()
    print("ok")
