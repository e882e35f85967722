"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (mean per dispatch).
usage: python tools/pmc_summary.py <dir containing run_counter_collection.csv> [filter]"""
import csv, glob, os, re, sys
from collections import defaultdict
d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for row in csv.DictReader(open(f)):
    k = re.sub(r"\(anonymous namespace\)::|^void ", "", row["Kernel_Name"]).split("(")[0]
    if flt not in k:
        continue
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    disp[k].add(row["Dispatch_Id"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    n = len(disp[k])
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    parts = [f"{name}={v / n:.3g}" for name, v in sorted(c.items())]
    frac = " ".join(f"{nm[3:]}/WC={c[nm] / wc:.2f}" for nm in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if nm in c)
    print(f"{k[:48]:48s} n={n:4d} {frac}\n    " + " ".join(parts))
