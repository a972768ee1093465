"""Per-launch HBM traffic of the Sankoff kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py PMCDIR CALIBDIR [--out profiles/traffic.json]

PMCDIR holds two rocprofv3 runs of tools/prof.py c4, pass_fetch
(--pmc FETCH_SIZE) and pass_write (--pmc WRITE_SIZE), counters reported in
KiB per dispatch.  CALIBDIR holds the same two passes over
tools/micro/load_pattern and tools/micro/store_pattern, whose byte counts are
known (MI355X_MICROARCH.md "HBM": FETCH_SIZE reads 1/2 of wide streaming
reads on gfx950, other widths must be calibrated on the access pattern
itself).  traffic = FETCH_SIZE * fetch_corr + WRITE_SIZE * write_corr.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def counters(d):
    v = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            v[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(x) / len(x) for c, x in cs.items()} for k, cs in v.items()}


def short(name):
    m = re.search(r"(sankoff_kernel|rows_load|stream_load|rows_kernel|stream_kernel|"
                  r"sitemajor_kernel|wide_reduce_kernel)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("calib")
    ap.add_argument("--out", default=None)
    ap.add_argument("--workload-key", default="1024x32x5000x4")
    a = ap.parse_args()
    known = 128 * 31 * 4 * 5000 * 4  # bytes per calibration launch
    cal = {short(k): v for k, v in counters(a.calib).items()}
    fetch_rows = cal["rows_load"]["FETCH_SIZE"] * 1024
    fetch_stream = cal["stream_load"]["FETCH_SIZE"] * 1024
    write_rows = cal["rows_kernel<1>"]["WRITE_SIZE"] * 1024 if "rows_kernel<1>" in cal else None
    write_sm = cal["sitemajor_kernel"]["WRITE_SIZE"] * 1024 if "sitemajor_kernel" in cal else None
    corr = {"fetch_4B_rows": known / fetch_rows, "fetch_16B_stream": known / fetch_stream,
            "write_4B_rows": (known / write_rows) if write_rows else 1.0,
            "write_16B_sitemajor": (known / write_sm) if write_sm else 1.0}
    # the site-major DP table (trex_version >= 4) is read and written 16 B per
    # lane: the 16-B stream / site-major store corrections apply
    fetch_corr = corr["fetch_16B_stream"]
    write_corr = corr["write_16B_sitemajor"] if write_sm else corr["write_4B_rows"]
    res = {"workload_key": a.workload_key, "calibration": corr, "kernels": {}}
    for k, v in counters(a.pmc).items():
        s = short(k)
        if "sankoff_kernel" not in s:
            continue
        f = v.get("FETCH_SIZE", 0.0) * 1024 * fetch_corr
        w = v.get("WRITE_SIZE", 0.0) * 1024 * write_corr
        res["kernels"][s] = {"fetch_bytes": f, "write_bytes": w, "traffic_bytes": f + w}
    # phase -> bench kernel name (sankoff_kernel<Q, SPT, SOFT, PHASE, RAGGED>)
    for s, e in res["kernels"].items():
        args = [x.strip() for x in s.split("<", 1)[1].rstrip(">").split(",")]
        if len(args) > 4 and args[4] == "true":
            continue  # ragged instantiation
        ph = args[3]
        name = {"1": "sankoff_fwd", "2": "sankoff_bwd", "3": "sankoff_fwd_bwd"}.get(ph)
        if name:
            res[name] = e["traffic_bytes"]
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
