#!/bin/bash
# Round 5: ragged sets on the pixel-major kernel (2-10 stars, 32/48-px images)
# — the ragged and RJ tests, C3 A/B against the round's final line (2.59e8),
# then the RJ lines (flagship BIGSIM4, B4) with a kernel trace of BIGSIM4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_pkragged}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rj_native.py tests/test_gpu_reference_runs.py \
  tests/test_gpu_sampler.py tests/test_gpu_parity.py tests/test_gpu_energy_device.py \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; j=d.get('rj') or {}; print('$n', '%.4g' % d['value'], r.get('kernel_ms'), d['ms_per_step'], j.get('native_call_s_last'))"
}
run c3_r1 --workload C3 --no-cpu --no-e2e
run c3_r2 --workload C3 --no-cpu --no-e2e
run rj_bigsim4_r1 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
run rj_bigsim4_r2 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
run rj_b4 --workload B4 --mode rj --steps 5 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_BIGSIM4 -o run --output-format csv -- python3 bench.py --workload BIGSIM4 --mode rj --steps 3 --warmup 1 > $O/trace_BIGSIM4.log 2>&1 || exit 1
echo pkragged done
