#!/bin/bash
# Where the MH loop's time goes (kernel trace), f_pos = 0 so that V(q') is
# finite (with f_pos = 1 every C5 chain starts below the flux wall: V = inf,
# every proposal rejected, the energy kernel returns at once).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for wl in C5 B4; do
  echo "=== $wl"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_mh_$wl -o run --output-format csv -- python3 bench.py --workload $wl --mode mh --mh-iter 5 --leap 50 --steps 2 --warmup 1 --no-cpu --mh-unfused --f-pos 0 > gpurun_out/trace_mh_$wl.log 2>&1 || exit $?
  grep '^{' gpurun_out/trace_mh_$wl.log | cut -c1-200
  timeout -k 10 300 python3 bench.py --workload $wl --leap 50 --steps 5 --warmup 1 --no-cpu --no-e2e > gpurun_out/leap50_$wl.json 2>/dev/null || exit $?
  cut -c1-200 gpurun_out/leap50_$wl.json
done
