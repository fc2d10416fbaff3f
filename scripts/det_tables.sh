#!/bin/bash
# WinGG factor-table evidence: the S256K100 MH bench
# (4,096 chains, 5 x 10 steps, three launches) twice per mode in separate
# processes on the product library (RHMC_OPT_TABLES 0: per-stream buffer,
# 1: the same NaN-filled before every launch), then — when the diagnostic
# build exists (scripts/build_variants.sh canary="-DRHMC_TABLE_CANARY") — on
# that build with per-launch pool allocation (2) and the per-stream buffer (0),
# reporting the table regions written by others during a gradient or
# potential and the values found there; then the table-determinism tests.
#   scripts/det_tables.sh [out_dir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=${1:-gpurun_out/det_tables}; mkdir -p "$O"
run() { # tag lib mode
  RHMC_LIB=$2 timeout -k 10 300 python3 bench.py --workload S256K100 --chains 4096 --mode mh \
    --mh-iter 5 --leap 10 --f-pos 0 --no-cpu --steps 2 --warmup 1 --tables $3 \
    > "$O/$1.json" 2> "$O/$1.err" || return 1
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', 'tables', $3, '%.4g' % d['value'], 'accept', repr(d.get('mh_accept_rate_last_launch')), 'conflicts', d.get('table_conflicts'), 'foreign', [v['hex'] for v in d.get('table_foreign_values', [])][:4])" | tee -a "$O/summary.txt"
}
L=hmc-stellar-toy-model_amd/librhmc.so
C=build/variants/lib_canary.so
run stream_1 $L 0 && run stream_2 $L 0 && run poison_1 $L 1 && run poison_2 $L 1 || exit 1
if [ -f $C ]; then
  run canary_pool_1 $C 2 && run canary_pool_2 $C 2 && run canary_stream $C 0 || exit 1
fi
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_tables_determinism.py > "$O/pytest.log" 2>&1; rc=$?; tail -3 "$O/pytest.log"; exit $rc
