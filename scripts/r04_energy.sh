#!/bin/bash
# Energy-kernel check after the potential-only windowed tables: the parity
# tests that reach V on the windowed path, then the C5 MH trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_energy.log 2>&1 || { tail -30 gpurun_out/pytest_energy.log; exit 1; }
tail -2 gpurun_out/pytest_energy.log
bash scripts/r04_mh_trace.sh
