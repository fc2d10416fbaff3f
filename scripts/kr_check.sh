#!/bin/bash
# Multi-star kernels: parity tests, then bench lines per kernel family.
# usage: kr_check.sh [WL:KERNEL ...]   (default: C3 and C5 on each family)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/kr
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampler.py -x -q --timeout 300 > gpurun_out/kr/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/kr/pytest.log; [ $rc -eq 0 ] || exit $rc
SPECS=${*:-"C3:auto C3:tiledk C3:tiledrk C3:tiledrk_notab C5:auto"}
for spec in $SPECS; do
  wl=${spec%%:*}; k=${spec#*:}
  if [ "$k" = auto ]; then unset RHMC_KERNEL; else export RHMC_KERNEL=$k; fi
  timeout -k 10 300 python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu --leap ${LEAP:-100} > gpurun_out/kr/${wl}_$k.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], d['fixed_point_iters_per_step']['q_loop_mean'])" gpurun_out/kr/${wl}_$k.log $spec
done
unset RHMC_KERNEL
