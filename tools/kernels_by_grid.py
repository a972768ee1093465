"""Split a rocprofv3 kernel trace (CSV) by kernel and grid size.

  python tools/kernels_by_grid.py gpurun_out/.../run_kernel_trace.csv [name-filter]

Prints count, mean / min / max duration (us), VGPRs, scratch and grid per
(kernel, grid) pair: the C4 bench launches the same kernel on the 1 024-tree
batch and on the 128-tree shard, which the plain --stats summary averages.
`late_us` is the mean over the second half of the launches in time order:
a fresh box runs its first ~30 ms of work at rising clocks, and the bench's
HIP-event timings are taken after its settle / warmup steps.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else "trex"
    groups = defaultdict(list)
    meta = {}
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if flt not in name:
                continue
            key = (name, int(r["Grid_Size_X"]))
            groups[key].append((int(r["Start_Timestamp"]),
                                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
            meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"])
    print(f"{'count':>6} {'mean_us':>9} {'late_us':>9} {'min_us':>9} {'max_us':>9} {'grid':>9} "
          f"{'vgpr':>5} {'agpr':>5} {'scr':>5} {'lds':>6}  kernel")
    for key in sorted(groups, key=lambda k: -sum(x[1] for x in groups[k])):
        d = [x[1] for x in sorted(groups[key])]
        late = d[len(d) // 2:]
        v, a, s, l = meta[key]
        short = key[0].replace("trex::(anonymous namespace)::", "").replace("void ", "")[:110]
        print(f"{len(d):6d} {sum(d) / len(d):9.2f} {sum(late) / len(late):9.2f} {min(d):9.2f} "
              f"{max(d):9.2f} {key[1]:9d} {v:>5} {a:>5} {s:>5} {l:>6}  {short}")


if __name__ == "__main__":
    main()
