#!/bin/bash
# rocprofv3 kernel-trace summary of the on-device MH bench (C2, 10 x 50).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/mh
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mh/prof -o run --output-format csv \
  -- python3 bench.py --no-cpu --mode mh --mh-iter 10 --leap 50 --steps 5 --warmup 1 \
  > gpurun_out/mh/bench.log 2>&1 || exit $?
cut -d, -f1-8 gpurun_out/mh/prof/run_kernel_stats.csv | head -12
