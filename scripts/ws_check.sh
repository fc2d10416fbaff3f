#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_window_split.py tests/test_gpu_fullsize_multistar.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ws_tests.log 2>&1
rc=$?; tail -15 gpurun_out/ws_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 1024 2048 4096 8192; do
  timeout -k 10 200 python3 tools/kernel_ab.py C5 auto --chains $n --reps 1 --launches 2 --window-split 1 0 || exit $?
done > gpurun_out/ws_perf.log 2>&1
rc=$?; cat gpurun_out/ws_perf.log; exit $rc
