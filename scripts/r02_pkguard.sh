#!/bin/bash
# GPU suite, then a pixel-major kernel change (new) against the previous build
# (prev): C3 implicit x3 and the explicit modes (used for the guard removal and the row peel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/abg
for r in 1 2 3; do
  for lib in new prev; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --workload C3 --steps 3 --warmup 1 > gpurun_out/abg/$lib.$r.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/abg/$lib.$r.json')); print('C3 $lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
bash scripts/c3_modes.sh prev
