#!/bin/bash
# Quick PMC comparison of kernel paths on a small workload.
# usage: pmc_quick.sh WORKLOAD CHAINS LEAP [PATHS...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
WL=$1; N=$2; L=$3; shift 3
PATHS=${*:-auto generic windowed}
OUT=gpurun_out/pmcq_$(echo $WL | tr A-Z a-z)
mkdir -p $OUT
for path in $PATHS; do
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F64"; do
    tag=$path_$(echo $grp | cut -c1-12 | tr ' ' _)
    RHMC_KERNEL=$path timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/$path/$(echo $grp | md5sum | cut -c1-6) -o run --output-format csv -- python3 bench.py --workload $WL --chains $N --leap $L --steps 2 --warmup 1 --no-cpu > $OUT/$path.log 2>&1 || exit $?
  done
  RHMC_KERNEL=$path timeout -k 10 300 python3 bench.py --workload $WL --chains $N --leap $L --steps 3 --warmup 1 --no-cpu > $OUT/bench_$path.log 2>&1 || exit $?
done
echo done
