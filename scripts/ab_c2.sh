#!/bin/bash
# GPU suite, then C2 A/B of the in-tree library against build/variants/lib_<v>.so
# for each v in "$1" (alternating on one box); extra args go to bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
VS=$1; shift
bash scripts/ab_libs.sh "$VS" --steps 20 --warmup 3 "$@"
