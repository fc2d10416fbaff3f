#!/bin/bash
# GPU suite, then km_steps with two fixed-point iterations per pass (new) vs one
# (spec1) on C3 (pixel-major kernel) and C5 (multi-star window kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/abk
for wl in C3 C5; do
  for r in 1 2; do
    for lib in new spec1; do
      if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
      RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --workload $wl --steps 3 --warmup 1 > gpurun_out/abk/$lib.$wl.$r.json || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/abk/$lib.$wl.$r.json')); print('$wl $lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'], d['fixed_point_iters_per_step'])"
    done
  done
done
