#!/usr/bin/env python3
"""Per-phase model of the register-window kernel's step at C2 (tools only;
DESIGN.md section 4.0).

Inputs: the marked disassembly tools/isa_regions.sh leaves (/tmp/isa/m.s: the
kernel split by rhmc_k1step.hpp's RHMC_MARKS `s_setprio n` markers; static
counts, every instruction of a region once) and the measured cycles per step
of tools/phase_prof.py (fenced s_memtime marks, profiles/r06_c2_phase/
phase_c2.txt).  At C2 every SIMD holds ONE wave (4,096 chains x 16 lanes), so
a phase is either issue-bound — its instructions issue about every 4.6
cycles, the pixel loop's rate (1,794 cycles for 392 instructions) — or
latency-bound: a dependent chain at ~9 cycles per fp64 link (tools/
isa_bench.hip: 8.9), 21.6 per v_rcp_f64 and ~63 per dependent ds_bpermute,
which no second wave hides.  Prints per region: the instruction classes, the
measured cycles, cycles per VALU instruction, the issue-bound floor (4.6 per
instruction) and the cross-lane latency (dependent ds_bpermute / swizzle).
usage: python tools/phase_model.py [m.s] [phase_c2.txt]"""
import re
import sys
from collections import Counter

ISSUE = 4.6        # cycles per VALU instruction, issue-bound (pixel loop)
XLANE = 63.1       # dependent ds_bpermute at one wave per SIMD (isa_bench)

NAMES = {"s_setprio 1": "gradient", "s_setprio 2": "kicks + p-loop",
         "s_setprio 3": "q-loop", "s_setprio 4": "flux metric + closing update",
         "s_setprio 5": "loop tail"}


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt") or op.startswith("s_nop"):
        return "wait"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op in ("ds_bpermute_b32", "ds_permute_b32", "ds_swizzle_b32"):
        return "xlane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("v_rcp_f64"):
        return "rcp64"
    if op.startswith("v_"):
        if re.search(r"quad_perm|row_|wave_|bank_mask|bound_ctrl", ins):
            return "dpp"
        return "fp64" if "_f64" in op else "valu32"
    return "other"


def measured(path):
    t = open(path).read()
    g = lambda k: float(re.search(k + r"\s+(\d+)", t).group(1))
    return {"s_setprio 1": g("gradient"), "s_setprio 2": g("kicks\\+p-loop"),
            "s_setprio 3": g("q-loop"), "s_setprio 4": g("flux\\+tail")}


def main():
    isa = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa/m.s"
    ph = sys.argv[2] if len(sys.argv) > 2 else "profiles/r06_c2_phase/phase_c2.txt"
    seg, counts = "start", {}
    for line in open(isa):
        ins = line.strip()
        if not ins:
            continue
        if ins.startswith("s_setprio"):
            seg = ins
            continue
        counts.setdefault(seg, Counter())[classify(ins)] += 1
    meas = measured(ph)
    # phase_prof's "flux+tail" bucket covers markers 4 and 5 (closing update + loop tail)
    counts["s_setprio 4"] = counts.get("s_setprio 4", Counter()) + counts.get("s_setprio 5", Counter())
    print("%-30s %8s %6s %8s %8s %8s  %s" % ("phase", "measured", "VALU", "cyc/VALU", "issue",
                                            "xlane", "classes"))
    for seg in ("s_setprio 1", "s_setprio 2", "s_setprio 3", "s_setprio 4"):
        c = counts.get(seg, Counter())
        valu = sum(c[k] for k in ("fp64", "valu32", "dpp", "rcp64"))
        print("%-30s %8.0f %6d %8.2f %8.0f %8.0f  %s" % (
            NAMES[seg], meas[seg], valu, meas[seg] / max(valu, 1), ISSUE * valu,
            XLANE * c["xlane"], dict(c)))
    print("total measured %.0f cycles per step" % sum(meas.values()))


if __name__ == "__main__":
    main()
