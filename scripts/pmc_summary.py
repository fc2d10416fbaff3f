#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (scripts/profile_pmc.sh) for the dominant
kernel into profiles/pmc_<workload>.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE counts half the bytes of a coalesced read (MI355X_MICROARCH.md
§HBM); WRITE_SIZE is taken as is.  Our reads/writes are 8-B per lane, an
uncalibrated width, so the number is an estimate (the point is its size next
to the algorithmic bytes)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import source_hash  # noqa: E402  (the hash bench.py checks)

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_c2"
wl = sys.argv[2] if len(sys.argv) > 2 else "c2"
kernel_sub = sys.argv[3] if len(sys.argv) > 3 else "leapfrog"
chain_steps = float(sys.argv[4]) if len(sys.argv) > 4 else 4096 * 500.
head = sys.argv[5] if len(sys.argv) > 5 else None      # source revision measured

vals = defaultdict(list)
names = set()
for path in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    with open(path) as fh:
        for row in csv.DictReader(fh):
            if kernel_sub not in row.get("Kernel_Name", ""):
                continue
            names.add(row["Kernel_Name"])
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))

avg = {k: sum(v) / len(v) for k, v in vals.items() if v}
out = {"workload": wl, "kernel_filter": kernel_sub, "kernel": " | ".join(sorted(names)),
       "head": head, "src_hash": source_hash(), "counters_avg_per_dispatch": avg}
if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
    out["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
f64 = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64")
if all(k in avg for k in f64):
    # executed fp64 flops (FMA = 2) over all 64 lanes, per chain-leapfrog-step
    flops = (2 * avg[f64[0]] + avg[f64[1]] + avg[f64[2]]) * 64
    out["chain_steps_per_dispatch"] = chain_steps
    out["fp64_flops_per_chain_step"] = flops / chain_steps
    out["valu_insts_per_chain_step"] = avg.get("SQ_INSTS_VALU", 0) / chain_steps
    out["fp64_insts_per_chain_step"] = sum(avg[k] for k in f64) / chain_steps
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
    # fraction of the waves' lifetime with a VALU instruction issuing (both in
    # quad-cycles); with one wave per SIMD this is the SIMD's VALU busy share
    out["valu_active_frac"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
if "GRBM_GUI_ACTIVE" in avg:
    out["note_clock"] = "effective clock = GRBM_GUI_ACTIVE / 8 / kernel time"
    if "SQ_INSTS_VALU" in avg and "SQ_INSTS_VALU_TRANS_F64" in avg:
        # the SIMDs' VALU issue share: 4 cycles per wave64 VALU instruction plus
        # ~12 more per v_rcp_f64 (tools/isa_bench.hip), per SIMD (256 CUs x 4),
        # over the kernel's cycles (GRBM_GUI_ACTIVE summed over the 8 XCDs).
        # Unlike valu_active_frac it does not depend on the waves per SIMD.
        kcyc = avg["GRBM_GUI_ACTIVE"] / 8
        issue = (4 * avg["SQ_INSTS_VALU"] + 12 * avg["SQ_INSTS_VALU_TRANS_F64"]) / 1024
        out["simd_valu_issue_frac"] = issue / kcyc
        out["waves_per_simd_resident"] = (avg["SQ_WAVE_CYCLES"] / avg["SQ_BUSY_CYCLES"]) / 7.77
        out["note_waves"] = ("waves_per_simd_resident: SQ_WAVE_CYCLES / SQ_BUSY_CYCLES "
                             "normalised by C2's 7.77 (exactly one wave per SIMD)")
dst = os.path.join("profiles", "pmc_%s.json" % wl)
with open(dst, "w") as fh:
    json.dump(out, fh, indent=1, sort_keys=True)
print(json.dumps(out, indent=1, sort_keys=True))
