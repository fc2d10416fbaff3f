#!/bin/bash
# Register-window kernel at C2: LDS request padded so that one workgroup
# (4 waves) fits per CU (82 KB) vs the natural 9.9 KB request.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ldscap
for pad in 0 82000 0 82000; do
  RHMC_LDS_MIN=$pad timeout -k 10 120 python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ldscap/p$pad.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ldscap/p$pad.json')); print('pad $pad', '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])"
done
