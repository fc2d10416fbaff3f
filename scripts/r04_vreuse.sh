#!/bin/bash
# The native RJ driver reusing the end-of-iteration V: its GPU tests (every
# recorded V recomputed alone, checkpoint, goldens), then throughput at
# big-sim4 geometry and the bench --mode rj line.  Logs under gpurun_out/r04_vreuse/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${OUT:-gpurun_out/r04_vreuse}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E "chain_leap|passed|failed|\"value\"" "$O/$name.log" | tail -1 | cut -c1-400
  if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
step 400 pytest_rj python3 -u -m pytest tests/test_gpu_rj_native.py tests/test_rj_asan_host.py tests/test_gpu_sampler.py -m gpu -v --timeout 120 --timeout-method thread
for n in 4096 16384; do
  step 200 native_$n python3 -u scripts/rj_batched_bench.py --engine native --chains $n --niter 10 --nsteps 20
done
step 200 native_4096_p1 python3 -u scripts/rj_batched_bench.py --engine native --chains 4096 --niter 10 --nsteps 20 --pipes 1
step 300 bench_rj_b4 python3 -u bench.py --mode rj --workload B4 --no-cpu --steps 5 --warmup 1
echo done
