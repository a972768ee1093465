"""Sum PMC counters of the last dispatch of kernels matching a filter:
  python tools/pmc_sum.py gpurun_out/pmc_C3 wide_kernel"""
import collections
import csv
import glob
import sys

d, flt = sys.argv[1], sys.argv[2]
tot = {}
for f in sorted(glob.glob(f"{d}/pass*/run_counter_collection.csv")):
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
