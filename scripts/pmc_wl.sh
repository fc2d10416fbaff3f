#!/bin/bash
# PMC passes (one counter group per pass, no tracing domains) for a bench
# workload's dominant kernel: scripts/pmc_wl.sh <WL> [extra bench args...].
# Writes gpurun_out/pmc_<wl>/; scripts/pmc_summary.py summarises.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
WL=${1:-C2}; shift
TAG=$(echo "$WL" | tr 'A-Z' 'a-z')
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {
  local name=$1; shift
  echo "=== pmc pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-e2e $EXTRA > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== pass $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
EXTRA="$*"
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass valu SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass f64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64
pass stall SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
echo pmc done
