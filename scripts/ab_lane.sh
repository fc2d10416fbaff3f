#!/bin/bash
# Lane-group kernel (C4) A/B: in-tree library vs build/variants/lib_base.so,
# the C4 shard (131,072 chains) and the whole 2^20 set, after the lane tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ablane
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lane_kernel.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ablane/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/ablane/pytest.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for lib in new base; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    for n in 131072 1048576; do
      RHMC_LIB=$L timeout -k 10 200 python3 bench.py --workload C4 --global-chains $n --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/ablane/$lib.$n.$r.json || exit $?
      python3 -c "import json; d=json.loads(open('gpurun_out/ablane/$lib.$n.$r.json').read().strip().splitlines()[-1]); print('C4 $n $lib $r', '%.4g' % d['value'], '%.3f' % d['roofline']['kernel_ms'])"
    done
  done
done
