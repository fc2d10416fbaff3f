#!/bin/bash
# Fused MH: per-iteration overhead (iterations x leapfrog steps at a fixed 500 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/mh
timeout -k 10 120 python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/mh/leap.json || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/mh/leap.json')); print('leapfrog 500', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
for cfg in "1 500" "10 50" "50 10"; do
  set -- $cfg
  timeout -k 10 120 python3 bench.py --no-cpu --mode mh --mh-iter $1 --leap $2 --steps 5 --warmup 1 \
    > gpurun_out/mh/sweep_$1x$2.json || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/mh/sweep_$1x$2.json')); print('mh $1x$2', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
