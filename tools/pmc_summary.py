"""Summarise rocprofv3 --pmc passes (tools/pmc.sh output directories).

    python tools/pmc_summary.py OUTDIR                 per Sankoff kernel, the mean
                                                        over dispatches + duration
    python tools/pmc_summary.py OUTDIR --kernel FILTER  kernels whose name contains
                                                        FILTER: the totals of the last
                                                        dispatch, per wave where
                                                        SQ_WAVES was collected
"""
import argparse
import collections
import csv
import glob
import os
import re
from collections import defaultdict


def short(name):
    m = re.search(r"(sankoff_\w+|to_trex_layout\w*)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:40]


def csvs(d, what):
    return sorted(glob.glob(os.path.join(d, "**", f"run_{what}.csv"), recursive=True))


def by_kernel(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in csvs(d, "counter_collection"):
        for row in csv.DictReader(open(f)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    durs = defaultdict(list)
    for f in csvs(d, "kernel_trace"):
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


def last_dispatch(d, flt):
    tot = {}
    for f in csvs(d, "counter_collection"):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if flt in r["Kernel_Name"]:
                agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        if agg:
            tot.update(agg[max(agg)])
    for k, v in tot.items():
        print(f"{k:24s} {v:16.0f}")
    if "SQ_WAVES" in tot:
        w = tot["SQ_WAVES"]
        for k in ("SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM"):
            if k in tot:
                print(f"per wave {k:16s} {tot[k] / w:10.0f}")
    return tot


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default=None)
    a = ap.parse_args()
    if a.kernel:
        last_dispatch(a.dir, a.kernel)
    else:
        by_kernel(a.dir)
