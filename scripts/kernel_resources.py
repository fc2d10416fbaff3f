#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (stdin or a log file)."""
import re
import subprocess
import sys

fields = ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]")
text = open(sys.argv[1]).read() if len(sys.argv) > 1 else sys.stdin.read()
rows, cur = [], None
for line in text.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for f in fields:
        m = re.search(r"remark:\s+" + re.escape(f) + r": (\d+)", line)
        if m and cur is not None:
            cur[f] = int(m.group(1))
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), text=True,
                       capture_output=True).stdout.splitlines()
for r, n in zip(rows, names):
    n = n.replace("rhmc::", "")
    print("%-90s vgpr %3s agpr %3s scratch %4s occ %s" % (
        n[:90], r.get("VGPRs"), r.get("AGPRs"), r.get(fields[2]), r.get(fields[3])))
