#!/bin/bash
# Pixel-major row skip: GPU suite on the in-tree library, then C3 leapfrog /
# MH A/B against build/variants/lib_base.so (HEAD) and lib_noskip.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abskip
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/abskip/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/abskip/pytest.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for lib in new base noskip; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 200 python3 bench.py --workload C3 --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/abskip/$lib.$r.json || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abskip/$lib.$r.json').read().strip().splitlines()[-1]); print('C3 leapfrog $lib $r', '%.4g' % d['value'], '%.3f' % d['roofline']['kernel_ms'])"
  done
done
for lib in new base; do
  if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
  RHMC_LIB=$L timeout -k 10 200 python3 bench.py --workload C3 --mode mh --leap 50 --mh-iter 5 --no-cpu --no-e2e --steps 2 --warmup 1 > gpurun_out/abskip/mh_$lib.json || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/abskip/mh_$lib.json').read().strip().splitlines()[-1]); print('C3 mh 5x50 $lib', '%.4g' % d['value'])"
done
