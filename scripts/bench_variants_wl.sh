#!/bin/bash
# Throughput of each build/variants/lib_*.so on the given workloads.
# usage: bench_variants_wl.sh WL[:KERNEL] ...   (env LEAP, CHAINS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/vw
for lib in build/variants/lib_*.so; do
  name=$(basename $lib .so)
  for spec in "$@"; do
    wl=${spec%%:*}; k=${spec#*:}; [ "$k" = "$spec" ] && k=auto
    if [ "$k" = auto ]; then unset RHMC_KERNEL; else export RHMC_KERNEL=$k; fi
    ch=""; [ -n "$CHAINS" ] && ch="--chains $CHAINS"
    RHMC_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py --workload $wl $ch --steps 3 --warmup 1 --no-cpu --leap ${LEAP:-100} > gpurun_out/vw/${name}_${wl}_$k.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" gpurun_out/vw/${name}_${wl}_$k.log $name $spec
  done
done
unset RHMC_KERNEL
