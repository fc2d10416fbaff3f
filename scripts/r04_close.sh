#!/bin/bash
# Session close: the whole GPU suite and smoke at the final sources, the
# pipe counts around the 16,384-chain default repeated, and the RJ bench
# line.  Logs under gpurun_out/r04_close/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r04_close
mkdir -p $O
export TMPDIR=/tmp
step() {
  local lim=$1 name=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E "chain_leap|passed|failed|smoke ok|\"value\"" "$O/$name.log" | tail -1 | cut -c1-300
  if [ $rc -ne 0 ]; then tail -30 "$O/$name.log"; exit $rc; fi
}
step 900 pytest_gpu python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step 300 smoke python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
for p in 2 3 4 2 3 4; do
  step 200 native_16384_p${p}_$SECONDS python3 -u scripts/rj_batched_bench.py --engine native --chains 16384 --niter 10 --nsteps 20 --pipes $p
done
step 200 native_4096 python3 -u scripts/rj_batched_bench.py --engine native --chains 4096 --niter 10 --nsteps 20
step 300 bench_rj_b4 python3 -u bench.py --mode rj --workload B4 --no-cpu --steps 5 --warmup 1
RHMC_BENCH_DEVICE=0 step 400 bench_rj_b4_2ranks python3 bench.py --mode rj --workload B4 --steps 3 --warmup 1 --gpus 2 --chains 2048 --timeout 350
echo done
