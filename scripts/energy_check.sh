#!/bin/bash
# Register-window energy kernel: parity tests, then MH at a lane-group batch
# size (131,072 chains: the four-kernel loop) with its kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/energy
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_energy_k1.py tests/test_gpu_parity.py tests/test_gpu_mh_fused.py tests/test_gpu_sampler.py \
  tests/test_gpu_samplers.py tests/test_gpu_datagen.py > gpurun_out/energy/tests.log 2>&1
rc=$?; tail -n 15 gpurun_out/energy/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/energy/prof -o run --output-format csv \
  -- python3 bench.py --no-cpu --mode mh --chains 131072 --mh-iter 10 --leap 50 --steps 3 --warmup 1 \
  > gpurun_out/energy/mh_131072.json 2> gpurun_out/energy/mh.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/energy/mh_131072.json').read().strip().splitlines()[-1]); print('mh 131072', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
cut -d, -f1-4 gpurun_out/energy/prof/run_kernel_stats.csv | head -6
echo done
