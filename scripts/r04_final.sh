#!/bin/bash
# Round-4 closing measurements at the final sources: GPU suite, smoke, the
# bench lines of every BASELINE config and the MH modes, rocprof kernel-trace
# summaries of the C2 and C5 bench commands.  Results under gpurun_out/r04_head/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04_head
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
B="python3 bench.py"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 $B "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', '%.4g' % d['value'], r.get('kernel_ms'), r.get('frac'), r.get('pmc_stale'))"
}
run c2_bench
run c3_bench --workload C3 --no-cpu
run c4_bench --workload C4 --no-cpu
run c5_bench --workload C5 --no-cpu --steps 5 --warmup 1
run b4_bench --workload B4 --no-cpu --no-e2e
run b3_bench --workload B3 --no-cpu --no-e2e --steps 5 --warmup 1
run c5_mh_5x50 --workload C5 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 0
run c5_leap50 --workload C5 --leap 50 --no-cpu --no-e2e --steps 5 --warmup 1
run c3_mh_5x50 --workload C3 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 4 --warmup 1
run c2_mh_10x50 --mode mh --mh-iter 10 --leap 50 --no-cpu --steps 4 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 > $O/trace_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --workload C5 --no-cpu --no-e2e --steps 3 --warmup 1 > $O/trace_c5.log 2>&1 || exit 1
echo final done
