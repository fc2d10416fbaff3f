#!/bin/bash
# C3 (pixel-major kernel) A/B: in-tree library vs build/variants/lib_<name>.so,
# leapfrog and the fused MH mode, then the pixel-major GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abpk
V=${1:-old}
for r in 1 2; do
  for lib in new $V; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 200 python3 bench.py --workload C3 --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/abpk/$lib.$r.json || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abpk/$lib.$r.json').read().strip().splitlines()[-1]); print('C3 leapfrog $lib $r', '%.4g' % d['value'], '%.3f' % d['roofline']['kernel_ms'])"
    RHMC_LIB=$L timeout -k 10 200 python3 bench.py --workload C3 --mode mh --leap 50 --mh-iter 5 --no-cpu --no-e2e --steps 2 --warmup 1 > gpurun_out/abpk/mh_$lib.$r.json || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/abpk/mh_$lib.$r.json').read().strip().splitlines()[-1]); print('C3 mh 5x50 $lib $r', '%.4g' % d['value'])"
  done
done
