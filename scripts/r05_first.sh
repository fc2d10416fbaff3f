#!/bin/bash
# Round 5, first GPU contact: the new reference-run tests (mh_bigk, rj_big,
# flagship), the de-vacuumed many-star MH tests, the C5 f_pos MH test, the
# bench contract; then the new bench lines (C5 MH with f_pos 1, the
# flagship RJ) beside B4 RJ and C2.  Results under gpurun_out/r05_first/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_first
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_reference_runs.py tests/test_gpu_bigk.py \
  "tests/test_gpu_fullsize_multistar.py::test_c5_mh_f_pos_vs_oracle" \
  tests/test_gpu_bench_contract.py tests/test_gpu_rj_native.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="python3 bench.py"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 $B "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', '%.4g' % d['value'], r.get('kernel_ms'), r.get('frac'), d.get('mh_accept_rate_last_launch'), (d.get('rj') or {}).get('phase_ms_per_iteration'))"
}
run c2_bench --no-cpu
run c5_mh_fpos1 --workload C5 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 1
run c5_mh_fpos1_unfused --workload C5 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 1 --mh-unfused
run c5_leap50 --workload C5 --leap 50 --no-cpu --no-e2e --steps 5 --warmup 1
run rj_b4 --workload B4 --mode rj --steps 5 --warmup 1
run rj_bigsim4 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5mh -o run --output-format csv -- python3 bench.py --workload C5 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 1 > $O/trace_c5mh.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_rj_bigsim4 -o run --output-format csv -- python3 bench.py --workload BIGSIM4 --mode rj --steps 3 --warmup 1 > $O/trace_rj.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_rj_b4 -o run --output-format csv -- python3 bench.py --workload B4 --mode rj --steps 2 --warmup 1 > $O/trace_rj_b4.log 2>&1 || exit 1
echo first done
