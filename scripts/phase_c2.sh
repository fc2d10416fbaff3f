#!/bin/bash
# Phase split (gradient vs rest cycles per step) of the windowed single-star
# kernel, and the 16/32 lanes-per-chain throughput at 4096 / 16384 chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/phase
for k in profw16 profw32; do
  RHMC_KERNEL=$k timeout -k 10 120 python3 tools/phase_prof.py 4096 >> gpurun_out/phase/phase.log 2>&1 || exit $?
done
bash scripts/c2_variants.sh tiledw tiledw32 || exit $?
