"""C4 step timing forms: hipGraph replay vs eager launches vs the per-launch
event bracket (where do the step's microseconds past the fused kernel go).

    python tools/time_step.py [--trees 1024] [--steps 20]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from trex_amd import SankoffEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trees", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ch, plan, leaves, cost = bench.make_inputs(torch, dev, a.trees, 32, 5000, 4, 0, a.trees)
    eng = SankoffEngine(plan, 5000, 4, dev)
    st = bench.Step(torch, eng, leaves, cost, 0.5)
    st()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        st()
    g5 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g5):
        for _ in range(5):
            st()

    def wall(fn, n):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    def events(fn, n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e-3 / n

    # cold start: consecutive blocks of 5 graph replays, per-step time each
    blocks = []
    torch.cuda.synchronize()
    for b in range(16):
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        blocks.append((time.perf_counter() - t0) / 5 * 1e6)
    print("cold graph replay, per-step us in blocks of 5:", " ".join(f"{x:.0f}" for x in blocks))
    out = {}
    for rep in range(2):
        out[f"graph_wall_us_{rep}"] = wall(g.replay, a.steps) * 1e6
        out[f"graph5_wall_us_{rep}"] = wall(g5.replay, a.steps // 5) / 5 * 1e6
        out[f"eager_wall_us_{rep}"] = wall(st, a.steps) * 1e6
        out[f"graph_events_us_{rep}"] = events(g.replay, a.steps) * 1e6
        out[f"eager_events_us_{rep}"] = events(st, a.steps) * 1e6
    kt = bench.time_kernels(torch, st)
    out["time_kernels_fused_us"] = kt["sankoff_fwd_bwd"] * 1e6
    for k, v in out.items():
        print(f"{k:28s} {v:9.1f}")


if __name__ == "__main__":
    main()
