#!/bin/bash
# Run-to-run determinism of the windowed global-table path: the S256K100 MH bench
# three times (separate processes) must report one acceptance rate; then the
# table-determinism and K > 256 GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r05_det; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --workload S256K100 --chains 4096 --mode mh --mh-iter 5 \
    --leap 10 --f-pos 0 --no-cpu --steps 2 --warmup 1 > $O/mh_$r.json 2> $O/mh_$r.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/mh_$r.json').read().strip().splitlines()[-1]); print('r$r', '%.4g' % d['value'], d.get('mh_accept_rate_last_launch'))" | tee -a $O/summary.txt
done
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tables_determinism.py tests/test_gpu_hugek.py tests/test_gpu_bigk.py \
  tests/test_gpu_ragged.py tests/test_gpu_rj_native.py tests/test_gpu_window_split.py \
  > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; exit $rc
