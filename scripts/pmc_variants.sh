#!/bin/bash
# VALU instruction count and VALU-active share of the dominant kernel for the
# in-tree library and each build/variants/lib_<name>.so (one PMC pass each).
#   pmc_variants.sh "name1 name2 ..." [WORKLOAD=C2] [KERNEL_SUBSTRING=leapfrog]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
VS=$1; WL=${2:-C2}; KSUB=${3:-leapfrog}
OUT=gpurun_out/pmcv
mkdir -p $OUT
for lib in new $VS; do
  if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
  RHMC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU \
    -d $OUT/$lib -o run --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --no-e2e > $OUT/$lib.log 2>&1 || exit $?
  python3 - "$OUT/$lib" "$KSUB" "$lib" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if sys.argv[2] not in r["Kernel_Name"]:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
a = {k: acc[k] / n[k] for k in acc}
print(sys.argv[3], "VALU/wave %.1f" % (a["SQ_INSTS_VALU"] / a["SQ_WAVES"]),
      "LDS/wave %.1f" % (a["SQ_INSTS_LDS"] / a["SQ_WAVES"]),
      "SALU/wave %.1f" % (a["SQ_INSTS_SALU"] / a["SQ_WAVES"]),
      "valu_active %.3f" % (a["SQ_ACTIVE_INST_VALU"] / a["SQ_WAVE_CYCLES"]))
PY
done
