#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
echo "=== dense tests ($(date +%T))"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bigk.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "dense or bigk or auto" > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/r04_dense_ab.sh || exit $?
bash scripts/r04_mh_c5.sh || exit $?
bash scripts/pmc_stall.sh B4 leapfrog_win 20 > gpurun_out/stall_b4.txt 2>&1; tail -30 gpurun_out/stall_b4.txt
echo session done
