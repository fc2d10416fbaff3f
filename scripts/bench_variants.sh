#!/bin/bash
# C2 throughput of each build/variants/lib_*.so at 4096 and 16384 chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/v
for lib in build/variants/lib_*.so; do
  name=$(basename $lib .so)
  for n in ${CHAINS:-4096 16384}; do
    RHMC_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --chains $n --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/v/${name}_$n.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.3e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" gpurun_out/v/${name}_$n.log $name $n
  done
done
