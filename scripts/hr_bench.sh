#!/bin/bash
# samplers.HMC_random bench lines: register-window (default) and windowed kernels, C2 geometry.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/next
timeout -k 10 120 python3 bench.py --no-cpu --mode hmc_random --steps 5 --warmup 1 \
  > gpurun_out/next/c2_hmc_random.json 2> gpurun_out/next/c2_hmc_random.err || exit $?
RHMC_KERNEL=windowed timeout -k 10 120 python3 bench.py --no-cpu --mode hmc_random --steps 5 --warmup 1 \
  > gpurun_out/next/c2_hmc_random_windowed.json 2>> gpurun_out/next/c2_hmc_random.err || exit $?
for f in c2_hmc_random c2_hmc_random_windowed; do
  python3 -c "import json; d=json.load(open('gpurun_out/next/$f.json')); print('$f', '%.4g' % d['value'], d['roofline']['kernel_ms'], d['nonfinite_chains'])"
done
