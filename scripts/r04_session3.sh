#!/bin/bash
# Full GPU suite, the one-GPU rehearsal of the 8-rank bench (C2, C4, C5) and a
# kernel trace of the C5 MH loop (where its time goes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_rehearsal
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step 900 pytest_gpu python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
for wl in C2 C4 C5; do
  step 600 r04_rehearsal/$wl env RHMC_BENCH_DEVICE=0 python3 bench.py --gpus 8 --workload $wl --no-cpu --steps 3 --warmup 1 --timeout 500
done
step 600 trace_c5_mh rocprofv3 --kernel-trace --stats -d gpurun_out/trace_c5_mh -o run --output-format csv -- python3 bench.py --workload C5 --mode mh --mh-iter 5 --leap 50 --steps 2 --warmup 1 --no-cpu --mh-unfused
echo done
