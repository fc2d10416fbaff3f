#!/bin/bash
# GPU suite, then lane-group kernel A/B: PSF factors by recurrence (new) vs one
# exp per factor (nolanerec) at the C4 shard (131,072 chains/GPU, one lane per
# chain) and at 32,768 chains (four lanes per chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/abl
for n in 131072 32768; do
  for r in 1 2; do
    for lib in new nolanerec; do
      if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
      RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --chains $n --steps 5 --warmup 1 > gpurun_out/abl/$lib.$n.$r.json || exit $?
      python3 -c "import json; d=json.load(open('gpurun_out/abl/$lib.$n.$r.json')); print('$n $lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
    done
  done
done
# C2 (register-window kernel, per-chain range check now) against HEAD ebde75f
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for lib in new base; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --steps 20 --warmup 3 > gpurun_out/ab/$lib.$r.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$lib.$r.json')); print('C2 $lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
