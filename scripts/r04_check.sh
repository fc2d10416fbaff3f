#!/bin/bash
# Round-4 GPU session: smoke, the GPU suite, the C2 bench line, PMC passes for
# the bench workload (profiles/pmc_<wl>.json at HEAD: scripts/pmc_summary.py
# runs afterwards in the build container) and a kernel trace.  Each GPU step
# has its own time limit; the script stops at the first crash or timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
WL=${2:-C2}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
  step 1000 pytest_gpu python3 -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step 600 bench_$WL python3 bench.py --workload $WL
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ] || [ "$MODE" = pmc ]; then
  step 900 pmc_$WL bash scripts/profile_pmc.sh $WL
  step 600 trace_$WL rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$WL -o run --output-format csv -- python3 bench.py --workload $WL --no-cpu
fi
echo done
