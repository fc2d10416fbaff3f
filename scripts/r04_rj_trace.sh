#!/bin/bash
# Kernel trace of the native RJ driver at big-sim4 geometry (4096 chains):
# per-launch start/end times show whether a phase's groups overlap.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_rj
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r04_rj/trace -o run --output-format csv -- python3 scripts/rj_batched_bench.py --engine native --chains 4096 --niter 4 --nsteps 20 > gpurun_out/r04_rj/trace.log 2>&1 || { tail -20 gpurun_out/r04_rj/trace.log; exit 1; }
find gpurun_out/r04_rj/trace -name "*.csv" | head
echo done
