#!/bin/bash
# GPU suite + C2 A/B (working tree vs HEAD build, corner skip off, one v_rcp_f64 per 8 pixels),
# C5 A/B (multi-star kernel with one v_rcp_f64 per 4 pixels vs HEAD), and one
# default bench line with the end_to_end (host-buffer) measurement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R=3 bash scripts/ab_multi.sh "base noskip rcp8" --no-e2e || exit $?
mkdir -p gpurun_out/ab5
for r in 1 2; do
  for lib in new base; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --workload C5 --steps 3 --warmup 1 > gpurun_out/ab5/$lib.$r.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab5/$lib.$r.json')); print('C5 $lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
timeout -k 10 120 python3 bench.py --no-cpu > gpurun_out/bench_e2e.json || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/bench_e2e.json')); print(d['value'], d['end_to_end'])"
