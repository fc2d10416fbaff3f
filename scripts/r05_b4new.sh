#!/bin/bash
# Round 5, B3 / B4 on the reference drivers' magnitude ranges (true stars of
# mags 15..20 / 15..20.5) and the RJ driver's record-buffer reuse: the RJ and
# energy tests, the B3 / B4 leapfrog and RJ bench lines, then B3 / B4 PMC
# passes and summaries.  Results under gpurun_out/${R05_OUT:-r05_b4new}/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_b4new}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rj_native.py tests/test_gpu_reference_runs.py \
  tests/test_gpu_energy_device.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
B="python3 bench.py"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 $B "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('rj') or {}; print('$n', '%.4g' % d['value'], d['ms_per_step'], r.get('native_call_s_last'), r.get('accept_rate_within'), r.get('accept_rate_jumps'))"
}
run b4_bench --workload B4 --steps 5 --warmup 2 --no-cpu
run b3_bench --workload B3 --steps 5 --warmup 2 --no-cpu
run rj_b4 --workload B4 --mode rj --steps 5 --warmup 1
run rj_b4_r2 --workload B4 --mode rj --steps 5 --warmup 1
run rj_bigsim4 --workload BIGSIM4 --mode rj --steps 5 --warmup 1
run rj_b4_16k --workload B4 --mode rj --chains 16384 --steps 3 --warmup 1
if [ -n "${PMC_HEAD:-}" ]; then
  for wl in B3 B4; do bash scripts/profile_pmc.sh $wl || exit $?; done
  S=$O/pmc_summaries
  mkdir -p $S
  python3 scripts/pmc_summary.py gpurun_out/pmc_b3 b3 leapfrog 409600 $PMC_HEAD > /dev/null &&
    python3 scripts/pmc_summary.py gpurun_out/pmc_b4 b4 leapfrog 409600 $PMC_HEAD > /dev/null &&
    cp profiles/pmc_b3.json profiles/pmc_b4.json $S/ || exit 1
  run b4_bench_pmc --workload B4 --steps 5 --warmup 2 --no-cpu
fi
echo b4new done
