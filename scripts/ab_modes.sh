#!/bin/bash
# C3 explicit integrators and HMC_random: pixel-major (default) against
# RHMC_KERNEL=tiledrk (window-major), alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/abm
for m in "integrate --solver leap_frog" "integrate --solver hmc" "hmc_random"; do
  tag=$(echo $m | tr ' -' '__')
  for r in 1 2; do
    timeout -k 10 120 python3 bench.py --no-cpu --workload C3 --steps 5 --warmup 2 --mode $m > gpurun_out/abm/$tag.pk.$r.json || exit $?
    RHMC_KERNEL=tiledrk timeout -k 10 120 python3 bench.py --no-cpu --workload C3 --steps 5 --warmup 2 --mode $m > gpurun_out/abm/$tag.kr.$r.json || exit $?
    for v in pk kr; do
      python3 -c "import json; d=json.load(open('gpurun_out/abm/$tag.$v.$r.json')); print('$tag $v $r', '%.4g' % d['value'], d['unit'], '%.3f ms' % d['ms_per_step'])"
    done
  done
done
