#!/bin/bash
# Kernel traces of the RJ bench lines (flagship BIGSIM4 and B4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_rjtrace}
mkdir -p $O
for wl in BIGSIM4 B4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_$wl -o run --output-format csv -- python3 bench.py --workload $wl --mode rj --steps 3 --warmup 1 > $O/trace_$wl.log 2>&1 || exit 1
  tail -1 $O/trace_$wl.log | cut -c1-200
done
echo rjtrace done
