#!/bin/bash
# Quick C2 iteration: GPU parity tests, then bench + phase split per kernel.
# usage: quick_c2.sh [KERNELS...]  (RHMC_KERNEL values; "auto" = unset)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/q
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/q/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/q/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in ${*:-auto}; do
  for n in 4096 16384; do
    if [ "$k" = auto ]; then unset RHMC_KERNEL; else export RHMC_KERNEL=$k; fi
    timeout -k 10 120 python3 bench.py --chains $n --steps 5 --warmup 1 --no-cpu > gpurun_out/q/${k}_$n.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" gpurun_out/q/${k}_$n.log $k $n
  done
done
unset RHMC_KERNEL
for k in ${PROF:-}; do
  RHMC_KERNEL=$k timeout -k 10 120 python3 tools/phase_prof.py 4096 2>&1 | grep cycles
done
