#!/bin/bash
# C2 windowed single-star kernel: lanes per chain 32 vs 16 at two chain counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c2v
for l in 32 16; do
  for n in 4096 16384; do
    RHMC_WIN_LPC=$l timeout -k 10 120 python3 bench.py --chains $n --steps 5 --warmup 1 --no-cpu > gpurun_out/c2v/w${l}_$n.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('win lpc', sys.argv[2], sys.argv[3], '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" gpurun_out/c2v/w${l}_$n.log $l $n
  done
done
