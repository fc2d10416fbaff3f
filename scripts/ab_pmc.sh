#!/bin/bash
# One GPU session for a kernel change: GPU suite on the working tree, then the
# default bench alternating between the working tree and build/variants/lib_<V>.so
# (3 rounds), then one PMC pass (VALU / LDS / SALU instruction counts) per library.
#   ab_pmc.sh V [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
V=$1; shift
mkdir -p gpurun_out/ab gpurun_out/pmcab
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash scripts/ab_lib.sh "$V" "$@" || exit $?
for lib in new $V; do
  if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
  RHMC_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES \
    SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d gpurun_out/pmcab/$lib -o run --output-format csv \
    -- python3 bench.py --no-cpu --steps 2 --warmup 1 "$@" > gpurun_out/pmcab/$lib.log 2>&1 || exit $?
done
python3 - "$V" <<'PY'
import csv, glob, sys
for lib in ("new", sys.argv[1]):
    tot = {}
    for f in glob.glob("gpurun_out/pmcab/%s/**/*counter_collection.csv" % lib, recursive=True):
        for r in csv.DictReader(open(f)):
            if "leapfrog" not in r["Kernel_Name"] and "mh_k1" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    w = tot.get("SQ_WAVES", 1.0)
    print(lib, {k: round(v / w, 1) for k, v in sorted(tot.items())},
          "valu_active %.3f" % (tot.get("SQ_ACTIVE_INST_VALU", 0) / max(tot.get("SQ_WAVE_CYCLES", 1), 1)))
PY
echo done
