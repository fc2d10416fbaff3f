#!/bin/bash
# MH (four-kernel loop) on the windowed global-table path: per-launch table
# allocation inside the loop, against the bare leapfrog rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_winmh}
mkdir -p $O
run() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --no-e2e "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['value'], d.get('mh_accept_rate_last_launch'))"
}
run s256k100_leap --workload S256K100 --chains 4096 --leap 10 --steps 3 --warmup 1
run s256k100_mh --workload S256K100 --chains 4096 --mode mh --mh-iter 5 --leap 10 --f-pos 0 --steps 2 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-allocation-trace --stats -d $O/trace_mh -o run --output-format csv -- python3 bench.py --workload S256K100 --chains 4096 --mode mh --mh-iter 5 --leap 10 --f-pos 0 --steps 2 --warmup 1 --no-cpu --no-e2e > $O/trace_mh.log 2>&1 || exit 1
echo winmh done
