#!/bin/bash
# The checkpoint GPU tests, then native RJ throughput at big-sim4 geometry for
# 1-4 pipes at 4,096 and 16,384 chains.  Logs under gpurun_out/r04_pipes/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${OUT:-gpurun_out/r04_pipes}
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E "chain_leap|passed|failed" "$O/$name.log" | tail -1
  if [ $rc -ne 0 ]; then tail -5 "$O/$name.log"; exit $rc; fi
}
step 400 pytest_rj python3 -u -m pytest tests/test_gpu_rj_native.py tests/test_rj_asan_host.py tests/test_gpu_sampler.py -m gpu -v --timeout 120 --timeout-method thread
for n in 4096 16384; do
  for p in 1 2 3 4; do
    step 200 native_${n}_p$p python3 -u scripts/rj_batched_bench.py --engine native --chains $n --niter 10 --nsteps 20 --pipes $p
  done
done
echo done
