#!/bin/bash
# GPU suite, then C3 A/B of the in-tree library against build/variants/lib_$1.so
# (alternating on one box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_lib.sh "$1" --workload C3 --steps 3 --warmup 1
