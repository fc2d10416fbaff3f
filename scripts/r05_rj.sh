#!/bin/bash
# Round 5: the device-resident reversible-jump driver (librhmc_rj.so on the
# ragged-set entry points of librhmc.so ABI 4): its parity tests, the ragged
# entry points' tests, then the RJ bench lines (B4 and the big-sim4 flagship)
# with kernel + copy traces.  Results under gpurun_out/r05_rj/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_rj}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rj_native.py tests/test_gpu_reference_runs.py \
  tests/test_gpu_sampler.py tests/test_rj_asan_host.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="python3 bench.py"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 $B "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['value'], d['ms_per_step'], (d.get('rj') or {}).get('phase_ms_per_iteration'), (d.get('rj') or {}).get('accept_rate_jumps'))"
}
run rj_b4 --workload B4 --mode rj --steps 5 --warmup 1
run rj_bigsim4 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
run rj_b4_16k --workload B4 --mode rj --chains 16384 --steps 3 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace_rj_b4 -o run --output-format csv -- python3 bench.py --workload B4 --mode rj --steps 2 --warmup 1 > $O/trace_rj_b4.log 2>&1 || exit 1
echo rj done
