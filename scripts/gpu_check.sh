#!/bin/bash
# One GPU session: smoke, parity tests, bench (N=1 and a 2-rank rehearsal on
# the one GPU), rocprofv3 kernel trace.  Each GPU step has its own time limit;
# stop at the first crash/timeout (rc >= 2 other than pytest's "tests failed").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
  step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
  step 1000 pytest_gpu python3 -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step 600 bench python3 bench.py
  step 300 bench_2ranks env RHMC_BENCH_DEVICE=0 python3 bench.py --gpus 2 --no-cpu --steps 10
  step 600 rocprof rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu
fi
echo done
