#!/bin/bash
# Round 5 evidence at the current sources: the bench lines of every BASELINE
# config and of the next rows (MH with f_pos, the reversible-jump driver incl.
# the big-sim4 flagship), rocprof kernel-trace summaries of the C2 and C5
# bench commands.  Results under gpurun_out/r05_head/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_head}
mkdir -p $O
B="python3 bench.py"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 $B "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', '%.4g' % d['value'], r.get('kernel_ms'), r.get('frac'), r.get('frac_of_issue_ceiling'), d.get('mh_accept_rate_last_launch'))"
}
run c2_bench
run c1_bench --workload C1 --no-cpu
run c3_bench --workload C3 --no-cpu
run c4_bench --workload C4 --no-cpu
run c4_shard --workload C4 --chains 131072 --no-cpu --no-e2e
run c5_bench --workload C5 --no-cpu --steps 5 --warmup 1
run c5_shard --workload C5 --chains 1024 --no-cpu --no-e2e --steps 5 --warmup 1
run b4_bench --workload B4 --no-cpu --no-e2e
run b3_bench --workload B3 --no-cpu --no-e2e --steps 5 --warmup 1
run c2_mh_10x50 --mode mh --mh-iter 10 --leap 50 --no-cpu --steps 4 --warmup 1
run c3_mh_5x50 --workload C3 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 4 --warmup 1
run c5_mh_5x10_fpos1 --workload C5 --mode mh --mh-iter 5 --leap 10 --no-cpu --steps 2 --warmup 1 --f-pos 1
run c5_mh_5x50_fpos1 --workload C5 --mode mh --mh-iter 5 --leap 50 --no-cpu --steps 2 --warmup 1 --f-pos 1
run rj_b4 --workload B4 --mode rj --steps 5 --warmup 1
run rj_bigsim4 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c2 -o run --output-format csv -- python3 bench.py --no-cpu --no-e2e --steps 10 --warmup 2 > $O/trace_c2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --workload C5 --no-cpu --no-e2e --steps 3 --warmup 1 > $O/trace_c5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5mh -o run --output-format csv -- python3 bench.py --workload C5 --mode mh --mh-iter 5 --leap 10 --no-cpu --steps 2 --warmup 1 --f-pos 1 > $O/trace_c5mh.log 2>&1 || exit 1
echo head done
