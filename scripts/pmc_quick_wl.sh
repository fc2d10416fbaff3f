#!/bin/bash
# One VALU/LDS PMC pass per workload (short launches): instructions per
# chain-step and VALU-active share of the dominant kernel.
# usage: pmc_quick_wl.sh WL [WL...]   (env LEAP = leapfrog steps per launch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for WL in "$@"; do
  TAG=$(echo "$WL" | tr 'A-Z' 'a-z')
  OUT=gpurun_out/pmcq_$TAG
  mkdir -p "$OUT"
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -d "$OUT/valu" -o run --output-format csv -- python3 bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --leap ${LEAP:-50} > "$OUT/valu.log" 2>&1 || exit $?
  tail -1 "$OUT/valu.log" | cut -c1-300
done
