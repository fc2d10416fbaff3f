#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/mh
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mh_fused_multistar.py tests/test_gpu_sampler.py tests/test_gpu_mh_fused.py -v -rf --timeout 120 --timeout-method thread > gpurun_out/mh/pytest.log 2>&1; rc=$?; tail -25 gpurun_out/mh/pytest.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
for v in "" "--mh-unfused"; do
  timeout -k 10 300 python3 bench.py --workload C3 --mode mh --mh-iter 5 --leap 50 --steps 3 --warmup 1 --no-cpu $v > gpurun_out/mh/b.json || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mh/b.json').read().strip().splitlines()[-1]); print('mh', '$v', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
timeout -k 10 300 python3 bench.py --workload C3 --steps 3 --warmup 1 --no-cpu --no-e2e --leap 250 > gpurun_out/mh/l.json || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/mh/l.json').read().strip().splitlines()[-1]); print('leapfrog 250', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
