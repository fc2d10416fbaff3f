#!/bin/bash
# Bench lines for the §8(f) "next" rows: on-device MH, explicit integrators,
# device data generation.  One JSON line per run in gpurun_out/next/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/next
run() {
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 300 python3 bench.py --no-cpu "$@" > "gpurun_out/next/$name.json" 2> "gpurun_out/next/$name.err"
  local rc=$?
  tail -c 600 "gpurun_out/next/$name.json"; echo
  if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 "gpurun_out/next/$name.err"; exit $rc; fi
}
run c2_mh_10x50 --mode mh --mh-iter 10 --leap 50 --steps 5 --warmup 1
run c3_mh_5x50 --workload C3 --mode mh --mh-iter 5 --leap 50 --steps 3 --warmup 1
run c2_int_hmc --mode integrate --solver hmc --steps 5 --warmup 1
run c2_int_naive --mode integrate --solver naive --steps 5 --warmup 1
run c2_int_leap_frog --mode integrate --solver leap_frog --steps 5 --warmup 1
for s in hmc naive leap_frog; do run c3_int_$s --workload C3 --mode integrate --solver $s --leap 100 --steps 3 --warmup 1; done
run c2_datagen --mode datagen --n-real 1000 --steps 10 --warmup 2
run c5_datagen --workload C5 --mode datagen --n-real 16 --steps 10 --warmup 2
echo done
