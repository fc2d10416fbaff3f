#!/bin/bash
# Full GPU suite, then the C3 bench line with its kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wl_c3
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wl_c3/prof -o run --output-format csv \
  -- python3 bench.py --workload C3 --steps 3 --warmup 1 --no-cpu > gpurun_out/wl_c3/bench.json 2> gpurun_out/wl_c3/bench.log || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/wl_c3/bench.json').read().strip().splitlines()[-1]); print('C3', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
cut -d, -f1-4 gpurun_out/wl_c3/prof/run_kernel_stats.csv | head -3
