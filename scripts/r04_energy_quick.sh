#!/bin/bash
# Quick energy check: the V parity tests, then the C5 MH trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bigk or energy or mh" > gpurun_out/pytest_energy.log 2>&1 || { tail -30 gpurun_out/pytest_energy.log; exit 1; }
tail -1 gpurun_out/pytest_energy.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_mh_C5 -o run --output-format csv -- python3 bench.py --workload C5 --mode mh --mh-iter 5 --leap 50 --steps 2 --warmup 1 --no-cpu --mh-unfused --f-pos 0 > gpurun_out/trace_mh_C5.log 2>&1 || exit $?
