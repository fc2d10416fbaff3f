#!/bin/bash
# C2 / C5 bench lines and the C5 MH loop against bare leapfrog in 50-step
# launches (>= 95 %).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_mh
run() {
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 300 python3 bench.py "$@" > gpurun_out/r04_mh/$name.json 2> gpurun_out/r04_mh/$name.err
  local rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04_mh/$name.json').read().strip().splitlines()[-1]); print('$name', '%.4g' % d['value'], d['unit'], 'kernel_ms', d['roofline']['kernel_ms'])" || tail -5 gpurun_out/r04_mh/$name.err
  [ $rc -eq 0 ] || exit $rc
}
run c2 --no-cpu
run c5_leap50 --workload C5 --no-cpu --no-e2e --leap 50 --steps 10 --warmup 2
run c5_mh_5x50 --workload C5 --no-cpu --mode mh --mh-iter 5 --leap 50 --steps 2 --warmup 1
run c5_mh_5x50_unfused --workload C5 --no-cpu --mode mh --mh-iter 5 --leap 50 --steps 2 --warmup 1 --mh-unfused
run c5 --workload C5 --no-cpu --no-e2e --steps 5 --warmup 1
echo done
