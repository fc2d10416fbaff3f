#!/bin/bash
# Phase split of the C2 register-window kernel (cycles per step per wave,
# fenced s_memtime; tools/phase_prof.py) and stall-related SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/phase
RHMC_KERNEL=profr timeout -k 10 120 python3 tools/phase_prof.py 4096 > gpurun_out/phase/profr.log 2>&1 || exit $?
cat gpurun_out/phase/profr.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS -d gpurun_out/phase/stall -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/phase/stall.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_IFETCH -d gpurun_out/phase/stall2 -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/phase/stall2.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for d in ("stall", "stall2"):
    f = glob.glob("gpurun_out/phase/%s/**/*counter_collection.csv" % d, recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "leapfrog" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    wc = avg["SQ_WAVE_CYCLES"]
    print(d, {k: "%.4g (%.3f)" % (v, v / wc) for k, v in sorted(avg.items())})
PY
