#!/bin/bash
# samplers.HMC_random: parity tests, then bench lines for the register-window
# (default) and windowed kernels at C2 and C3 geometry.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/next
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_samplers.py > gpurun_out/next/hr_tests.log 2>&1
rc=$?; tail -n 12 gpurun_out/next/hr_tests.log
[ $rc -ne 0 ] && exit $rc
run() {
  local name=$1; shift
  timeout -k 10 120 python3 bench.py --no-cpu --mode hmc_random "$@" \
    > gpurun_out/next/$name.json 2>> gpurun_out/next/hr_bench.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/next/$name.json')); print('$name', '%.4g' % d['value'], d['roofline']['kernel_ms'], d['nonfinite_chains'])"
}
run c2_hmc_random --steps 5 --warmup 1
RHMC_KERNEL=windowed run c2_hmc_random_windowed --steps 5 --warmup 1
run c3_hmc_random --workload C3 --leap 100 --steps 3 --warmup 1
RHMC_KERNEL=windowed run c3_hmc_random_windowed --workload C3 --leap 100 --steps 3 --warmup 1
echo done
