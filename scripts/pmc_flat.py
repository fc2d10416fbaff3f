#!/usr/bin/env python3
"""Merge the rocprofv3 PMC passes under DIR for kernels matching FILTER and
print per-dispatch averages, per chain-step and per wave-step values.
usage: pmc_flat.py DIR [FILTER] [CHAIN_STEPS] [STEPS_PER_WAVE]"""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "leapfrog"
cs = float(sys.argv[3]) if len(sys.argv) > 3 else 4096 * 500.0
spw = float(sys.argv[4]) if len(sys.argv) > 4 else 500.0
vals = defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if filt in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in vals.items()}
waves = avg.get("SQ_WAVES", 0) or 1
for k in sorted(avg):
    print("%-26s %16.1f  /chain-step %9.2f  /wave-step %9.2f" % (k, avg[k], avg[k] / cs,
                                                               avg[k] / waves / spw))
