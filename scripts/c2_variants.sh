#!/bin/bash
# C2 throughput of the single-star kernel variants at several chain counts.
# usage: c2_variants.sh [KERNELS...]   (RHMC_KERNEL values; default tiled2 tiled4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c2v
for k in ${*:-tiled2 tiled4}; do
  for n in 4096 16384; do
    RHMC_KERNEL=$k timeout -k 10 120 python3 bench.py --chains $n --steps 5 --warmup 1 --no-cpu > gpurun_out/c2v/${k}_$n.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" gpurun_out/c2v/${k}_$n.log $k $n
  done
done
