"""C5-size split Gram launches (gram_kernel3 + reduce) for rocprofv3
kernel-trace / PMC runs:  python tools/prof_gram.py [iters]"""
import sys

import torch

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trex_amd._lib import check, lib, ptr, stream_handle  # noqa: E402

N, L, skip = 511, 50000, 256
K = 4 * L
dev = torch.device("cuda", 0)
st = stream_handle(dev)
g = torch.Generator(device=dev)
g.manual_seed(0)
S = torch.softmax(torch.randn((N, L, 4), generator=g, device=dev) * 3, -1).reshape(N, K).contiguous()
ws = torch.empty(int(lib().trex_tree_workspace_bytes(N, K)), dtype=torch.uint8, device=dev)
G = torch.empty((N, N), device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    check(lib().trex_tree_gram_skip_x3(ptr(S), N, K, skip, 1.0, ptr(G), ptr(ws), ws.numel(), st))
torch.cuda.synchronize()
print("done")
