"""Run each Sankoff entry point ITERS times on the bench workload (C4, 1024 trees),
for rocprofv3 kernel-trace / PMC collection.

    rocprofv3 --kernel-trace --stats -d OUT -o run --output-format csv -- \
        python tools/prof_kernels.py [--which fused|fwd|bwd|all]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="all")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--trees", type=int, default=1024)
    ap.add_argument("--taxa", type=int, default=32)
    ap.add_argument("--sites", type=int, default=5000)
    ap.add_argument("--tau", type=float, default=0.5)
    a = ap.parse_args()
    import torch

    from bench import Step, make_inputs
    from trex_amd import SankoffEngine

    dev = torch.device("cuda", 0)
    ch, plan, leaves, cost = make_inputs(torch, dev, a.trees, a.taxa, a.sites, 4, 0, a.trees)
    eng = SankoffEngine(plan, a.sites, 4, dev)
    st = Step(torch, eng, leaves, cost, a.tau)
    st.fwd()
    for _ in range(a.iters):
        if a.which in ("all", "fused"):
            st.fused()
        if a.which in ("all", "fwd"):
            st.fwd()
        if a.which in ("all", "bwd"):
            st.bwd()
    torch.cuda.synchronize()
    print("done", plan.n_slots)


if __name__ == "__main__":
    main()
