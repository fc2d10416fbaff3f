#!/bin/bash
# rocprofv3 PMC passes for the bench workload (one counter group per pass,
# --pmc never combined with tracing domains).  Writes gpurun_out/pmc_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
WL=${1:-C2}
TAG=$(echo "$WL" | tr 'A-Z' 'a-z')
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="python3 bench.py --workload $WL --steps 3 --warmup 1 --no-cpu --no-e2e ${PMC_ARGS:-}"
TAG=${PMC_TAG:-$TAG}
OUT=gpurun_out/pmc_$TAG
mkdir -p "$OUT"
pass() {
  local name=$1; shift
  echo "=== pmc pass $name: $*"
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- $BENCH > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== pass $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass valu SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE
pass f64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64
echo pmc done
