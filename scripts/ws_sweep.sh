#!/bin/bash
# C5 window-split sweep: chains per GPU x RHMC_OPT_WINDOW_SPLIT (1, 2, 4),
# HIP-event time of 500-step launches (tools/kernel_ab.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ws
for n in ${CHAINS:-1024 2048 4096 8192 16384}; do
  timeout -k 10 300 python3 tools/kernel_ab.py C5 auto --chains $n --window-split 1 2 4 --reps 2 --launches 2 \
    > gpurun_out/ws/c5_$n.txt 2>&1 || exit $?
  grep rep gpurun_out/ws/c5_$n.txt
done
