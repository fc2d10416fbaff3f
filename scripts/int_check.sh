#!/bin/bash
# Explicit integrators on the register-window kernel: parity tests, then the
# C2 bench lines (gpurun_out/next/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/next
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_integrators.py tests/test_gpu_sampler.py -k "explicit or integrators" \
  > gpurun_out/int_tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/int_tests.log
[ $rc -ne 0 ] && exit $rc
for s in hmc naive leap_frog; do
  timeout -k 10 300 python3 bench.py --no-cpu --mode integrate --solver $s --steps 5 --warmup 1 \
    > gpurun_out/next/c2_int_$s.json 2> gpurun_out/next/c2_int_$s.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/next/c2_int_$s.json')); print('$s', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
for s in hmc naive leap_frog; do
  timeout -k 10 300 python3 bench.py --no-cpu --workload C3 --mode integrate --solver $s --leap 100 --steps 3 --warmup 1 \
    > gpurun_out/next/c3_int_$s.json 2> gpurun_out/next/c3_int_$s.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/next/c3_int_$s.json')); print('C3 $s', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
echo done
