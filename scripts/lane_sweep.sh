#!/bin/bash
# Single-star kernels against the chain count: register-window (tiledr) vs the
# lane-group kernel (tiledl1 / tiledl4, rhmc_tiledl.hpp), C2 geometry, 500
# steps per launch.  One bench line per (kernel, chains) under gpurun_out/lane/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/lane
for n in ${CHAINS:-16384 65536 131072}; do
  for k in ${KERNELS:-tiledr tiledl1 tiledl4}; do
    RHMC_KERNEL=$k timeout -k 10 120 python3 bench.py --chains "$n" --no-cpu --steps 5 --warmup 1 \
      > gpurun_out/lane/${k}_${n}.json || exit 1
    python3 -c "
import json; r = json.load(open('gpurun_out/lane/${k}_${n}.json'))
print('%-8s %7d %.3e chain-steps/s  kernel_ms %.3f' % ('$k', $n, r['value'], r['roofline']['kernel_ms']))"
  done
done
