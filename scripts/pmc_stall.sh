#!/bin/bash
# Where a workload's dominant kernel waits: two PMC passes (issue-active and
# wait counters of the SQ), short launches.
#   pmc_stall.sh [WORKLOAD=C5] [KERNEL_SUBSTRING=leapfrog] [LEAP=20]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
WL=${1:-C5}; KSUB=${2:-leapfrog}; LEAP=${3:-20}
OUT=gpurun_out/pmc_stall_$(echo "$WL" | tr 'A-Z' 'a-z')
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  -d $OUT/p1 -o run --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --no-e2e --leap $LEAP > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_LDS SQ_INSTS_VALU \
  -d $OUT/p2 -o run --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --no-e2e --leap $LEAP > $OUT/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU \
  -d $OUT/p3 -o run --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --no-e2e --leap $LEAP > $OUT/p3.log 2>&1 || exit $?
for p in p1 p2 p3; do
  python3 - "$OUT/$p" "$KSUB" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if sys.argv[2] not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc):
    print("%-22s %.4g" % (k, acc[k]))
PY
done
