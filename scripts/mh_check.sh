#!/bin/bash
# Fused one-star MH loop: parity tests, then the C2 MH bench line and its
# kernel-trace summary (gpurun_out/mh/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/mh
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_mh_fused.py tests/test_gpu_sampler.py > gpurun_out/mh/tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/mh/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --mode mh --mh-iter 10 --leap 50 --steps 5 --warmup 1 \
  > gpurun_out/mh/c2_mh_10x50.json 2> gpurun_out/mh/c2_mh.err || exit $?
timeout -k 10 300 env RHMC_MH=unfused python3 bench.py --no-cpu --mode mh --mh-iter 10 --leap 50 --steps 5 --warmup 1 \
  > gpurun_out/mh/c2_mh_10x50_unfused.json 2>> gpurun_out/mh/c2_mh.err || exit $?
for f in c2_mh_10x50 c2_mh_10x50_unfused; do
  python3 -c "import json; d=json.load(open('gpurun_out/mh/$f.json')); print('$f', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/mh/prof -o run --output-format csv \
  -- python3 bench.py --no-cpu --mode mh --mh-iter 10 --leap 50 --steps 5 --warmup 1 \
  > gpurun_out/mh/rocprof.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/mh/prof/run_kernel_stats.csv | head -5
echo done
