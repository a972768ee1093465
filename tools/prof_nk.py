"""Run the NK landscape-aware step (bench.py nk_line) for rocprofv3
kernel-trace collection:
    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python tools/prof_nk.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    from bench import nk_line

    print(nk_line(torch, torch.device("cuda", 0), steps=10, warmup=2))
