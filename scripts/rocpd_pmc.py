#!/usr/bin/env python3
"""Per-kernel PMC counter averages from a rocprofv3 SQLite output
(run_results.db): usage rocpd_pmc.py DB [kernel_substring]."""
import sqlite3
import sys
from collections import defaultdict

db = sqlite3.connect(sys.argv[1])
sub = sys.argv[2] if len(sys.argv) > 2 else "leapfrog"
q = """select s.kernel_name, p.name, e.value, d.id, d.end - d.start
       from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id
       join rocpd_kernel_dispatch d on d.event_id = e.event_id
       join rocpd_info_kernel_symbol s on s.id = d.kernel_id"""
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for kname, cname, val, did, dur in db.execute(q):
    if sub in kname:
        acc[kname][cname] += val
        disp[kname].add(did)
for k, cs in acc.items():
    n = len(disp[k])
    print(k[:90], "dispatches", n)
    for c, v in sorted(cs.items()):
        print("  %-28s %.6g" % (c, v / n))
