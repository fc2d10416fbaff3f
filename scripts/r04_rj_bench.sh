#!/bin/bash
# Native vs NumPy-loop reversible-jump throughput at big-sim4 geometry, with
# the native driver's per-phase wall times.  Logs under gpurun_out/r04_rj/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r04_rj
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E "chain_leap|passed|failed" "$O/$name.log" | tail -1
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; exit $rc; fi
}
step 300 pytest_rj python3 -u -m pytest tests/test_gpu_rj_native.py tests/test_gpu_sampler.py tests/test_gpu_energy_device.py -m gpu -q -k "rj or reversible or energy_device" --timeout 200 --timeout-method thread
for n in 256 1024 4096 16384; do
  step 300 native_$n python3 -u scripts/rj_batched_bench.py --engine native --chains $n --niter 10 --nsteps 20
done
step 300 python_256 python3 -u scripts/rj_batched_bench.py --engine python --chains 256 --niter 10 --nsteps 20
step 300 native_4096_t1 python3 -u scripts/rj_batched_bench.py --engine native --chains 4096 --niter 10 --nsteps 20 --threads 1
step 300 native_4096_p1 python3 -u scripts/rj_batched_bench.py --engine native --chains 4096 --niter 10 --nsteps 20 --pipes 1
step 300 native_16384_p1 python3 -u scripts/rj_batched_bench.py --engine native --chains 16384 --niter 10 --nsteps 20 --pipes 1
echo done
