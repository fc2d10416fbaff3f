#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
echo "=== dense tests ($(date +%T))"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bigk.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "dense or bigk or auto" > gpurun_out/pytest_dense.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dense.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/dense_ab2.txt
for wl in B4 B3 S32K12 S32K24 S48K12 S48K24 S48K40; do
  timeout -k 10 240 python3 tools/kernel_ab.py $wl dense --chains 4096 --reps 2 --launches 2 >> gpurun_out/dense_ab2.txt 2>&1 || exit $?
done
grep "rep 1" gpurun_out/dense_ab2.txt
bash scripts/pmc_stall.sh B4 leapfrog_win 20 > gpurun_out/stall_b4.txt 2>&1; grep -E "BANK|IDX_ACTIVE|INSTS_LDS|INSTS_VALU|WAVE_CYCLES|ACTIVE_INST_VALU" gpurun_out/stall_b4.txt
echo done
