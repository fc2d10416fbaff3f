#!/usr/bin/env python3
"""Print per-dispatch counter averages for each kernel path of pmc_quick.sh."""
import csv, glob, json, os, sys
from collections import defaultdict
root = sys.argv[1]
chain_steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for path in sorted(os.listdir(root)):
    d = os.path.join(root, path)
    if not os.path.isdir(d):
        continue
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "leapfrog" in row["Kernel_Name"]:
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    b = os.path.join(root, "bench_%s.log" % path)
    ms = None
    try:
        ms = json.loads(open(b).read().strip().splitlines()[-1])["roofline"]["kernel_ms"]
    except Exception:
        pass
    print("==", path, "kernel_ms", ms)
    for k in sorted(vals):
        v = sum(vals[k]) / len(vals[k])
        print("   %-24s %14.1f  per chain-step %10.2f" % (k, v, v / chain_steps))
