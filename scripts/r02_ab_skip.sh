#!/bin/bash
# Corner-block skip A/B on C2: GPU suite on the working tree (corners first),
# then new / skiplast (corners last) / noskip / base alternating, and one
# SQ_INSTS_VALU pass per library (dynamic VALU count: is the skip taken?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=3 bash scripts/ab_multi.sh "skiplast noskip base" --no-e2e || exit $?
mkdir -p gpurun_out/pmcv
for lib in new noskip; do
  if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
  RHMC_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS -d gpurun_out/pmcv/$lib -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/pmcv/$lib.log 2>&1 || exit $?
  python3 - gpurun_out/pmcv/$lib <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "leapfrog" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1], {k: sum(v) / len(v) for k, v in acc.items()})
PY
done
