#!/bin/bash
# A/B of build/variants/lib_*.so on a multi-star workload (default C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/kr_ab
for lib in build/variants/lib_*.so; do
  for wl in ${WLS:-C3}; do
    t=$(basename $lib .so)_$wl
    RHMC_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $wl --no-cpu --steps ${STEPS:-3} --warmup 1 > gpurun_out/kr_ab/$t.json || exit 1
    python3 -c "
import json; r = json.load(open('gpurun_out/kr_ab/$t.json'))
print('%-24s %.3e chain-steps/s  kernel_ms %.3f' % ('$t', r['value'], r['roofline']['kernel_ms']))"
  done
done
