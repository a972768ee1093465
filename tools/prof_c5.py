"""Run the C5 Adam step (bench.py c5_line) for rocprofv3 kernel-trace:
    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- python tools/prof_c5.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    import torch

    from bench import c5_line

    print(c5_line(torch, torch.device("cuda", 0), steps=10, warmup=2))
