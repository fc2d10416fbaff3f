#!/bin/bash
# Multi-star kernels: parity tests, then C3/C5 bench lines per kernel family.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/kr
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampler.py -x -q --timeout 300 > gpurun_out/kr/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/kr/pytest.log; [ $rc -eq 0 ] || exit $rc
for wl in C3 C5; do
  for k in auto tiledk windowed; do
    if [ "$k" = auto ]; then unset RHMC_KERNEL; else export RHMC_KERNEL=$k; fi
    [ "$wl" = C5 ] && [ "$k" = tiledk ] && continue
    timeout -k 10 300 python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu --leap ${LEAP:-100} > gpurun_out/kr/${wl}_$k.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], d['fixed_point_iters_per_step'])" gpurun_out/kr/${wl}_$k.log $wl $k
  done
done
unset RHMC_KERNEL
