"""C2 / C3 fwd + grad a few times under the library's kernel policy (for
rocprofv3 --pmc passes).   python tools/prof_small.py C2|C3 [iters]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from time_small import case  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
step, _ = case(name, torch.device("cuda", 0))
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 5):
    step()
torch.cuda.synchronize()
print("ok")
