#!/bin/bash
# A/B of build/variants/lib_*.so on the lane-group kernel (C2 geometry, N chains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/lane_ab
for lib in build/variants/lib_*.so; do
  for n in ${CHAINS:-131072}; do
    t=$(basename $lib .so)_$n
    RHMC_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --chains $n --no-cpu --steps 5 --warmup 1 > gpurun_out/lane_ab/$t.json || exit 1
    python3 -c "
import json; r = json.load(open('gpurun_out/lane_ab/$t.json'))
print('%-24s %.3e chain-steps/s  kernel_ms %.3f' % ('$t', r['value'], r['roofline']['kernel_ms']))"
  done
done
