#!/bin/bash
# WinGG factor-table modes (RHMC_OPT_TABLES): the S256K100 MH bench, twice per
# mode in separate processes, then the table-determinism tests.  Usage:
#   scripts/det_tables.sh [out_dir] [modes...]     (default: all four modes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-gpurun_out/det_tables}; shift; mkdir -p "$O"
MODES=${*:-0 1 2 3}
for m in $MODES; do
  for r in 1 2; do
    timeout -k 10 300 python3 bench.py --workload S256K100 --chains 4096 --mode mh --mh-iter 5 \
      --leap 10 --f-pos 0 --no-cpu --steps 2 --warmup 1 --tables $m \
      > $O/mh_t${m}_$r.json 2> $O/mh_t${m}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/mh_t${m}_$r.json').read().strip().splitlines()[-1]); print('tables=$m run $r', '%.4g' % d['value'], repr(d.get('mh_accept_rate_last_launch')), d['nonfinite_chains'])" | tee -a $O/summary.txt
  done
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tables_determinism.py > $O/pytest.log 2>&1; rc=$?; tail -12 $O/pytest.log; exit $rc
