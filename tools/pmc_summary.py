"""Summarise rocprofv3 --pmc passes per kernel (mean over dispatches).

    python tools/pmc_summary.py gpurun_out/pmc1
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(sankoff_\w+|to_trex_layout\w*)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pass*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = short(row["Kernel_Name"])
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    durs = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pass*", "run_kernel_trace.csv"))):
        for row in csv.DictReader(open(f)):
            durs[short(row["Kernel_Name"])].append(
                (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    out = {}
    for k, cs in vals.items():
        if "sankoff" not in k:
            continue
        # counters are reported per dispatch (summed over XCD/SE instances by rocprofv3)
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        m["duration_us"] = sum(durs[k]) / max(1, len(durs[k]))
        out[k] = m
    for k, m in out.items():
        print(k)
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:.4g}")
    return out


if __name__ == "__main__":
    main(sys.argv[1])
