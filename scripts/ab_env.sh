#!/bin/bash
# A/B of the default bench between RHMC_KERNEL unset and RHMC_KERNEL=$1, alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
K=$1; shift
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 "$@" > gpurun_out/ab/def.$r.json || exit $?
  RHMC_KERNEL=$K timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 "$@" > gpurun_out/ab/$K.$r.json || exit $?
  for v in def $K; do
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$v.$r.json')); print('$v $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
