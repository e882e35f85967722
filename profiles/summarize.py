#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/<tag>_summary.json.

  python profiles/summarize.py TAG WORKLOAD KSTATS_DIR FETCH_DIR WRITE_DIR [MODE]

Per kernel: calls, average duration (kernel-trace --stats), and HBM bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes (both reported in KB;
gfx950 FETCH_SIZE counts wide coalesced reads at half their bytes
(MI355X_MICROARCH.md, HBM section), so reads are doubled; WRITE_SIZE is exact
for 16-B-per-lane stores).
"""
import collections
import csv
import json
import os
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    return n.split("(")[0].replace("void ", "").strip()


def main():
    tag, workload, kdir, fdir, wdir = sys.argv[1:6]
    mode = sys.argv[6] if len(sys.argv) > 6 else "rollout"
    out = {"tag": tag, "workload": workload, "mode": mode, "kernels": {}}
    for r in csv.DictReader(open(os.path.join(kdir, "run_kernel_stats.csv"))):
        out["kernels"][short(r["Name"])] = {"calls": int(r["Calls"]),
                                           "avg_us": float(r["AverageNs"]) / 1e3,
                                           "pct_time": float(r["Percentage"])}
    for key, d, mult in (("fetch_bytes", fdir, 2.0), ("write_bytes", wdir, 1.0)):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0 * mult)
        for k, v in agg.items():
            out["kernels"].setdefault(k, {})[key] = sum(v) / len(v)
    for k, v in out["kernels"].items():
        if "fetch_bytes" in v and "write_bytes" in v:
            v["hbm_bytes"] = v["fetch_bytes"] + v["write_bytes"]
            if "avg_us" in v:
                v["hbm_GBps"] = v["hbm_bytes"] / (v["avg_us"] * 1e-6) / 1e9
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{tag}_summary.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path)


if __name__ == "__main__":
    main()
