#!/bin/bash
# HEAD check after the batched-RJ host changes: the sampler GPU tests, the
# batched reversible-jump throughput at big-sim4 geometry, then (FULL=1) the
# whole GPU suite and smoke.  Logs under gpurun_out/r04_s4/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r04_s4
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step 600 pytest_sampler python3 -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_rj_native.py -m gpu -v --timeout 300 --timeout-method thread
for n in 64 256 1024 4096; do
  step 400 rj_native_$n python3 -u scripts/rj_batched_bench.py --engine native --chains $n --niter 6 --nsteps 20
done
for n in 64 256; do
  step 400 rj_python_$n python3 -u scripts/rj_batched_bench.py --engine python --chains $n --niter 6 --nsteps 20
done
if [ -n "$FULL" ]; then
  step 900 pytest_gpu python3 -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread
  step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke()"
fi
echo done
