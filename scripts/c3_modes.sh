#!/bin/bash
# C3 bench lines of the explicit integrators and HMC_random (in-tree library
# and build/variants/lib_$1.so when given), one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/modes
for lib in new $1; do
  [ -z "$lib" ] && continue
  if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
  for mode in "integrate --solver leap_frog" "integrate --solver hmc" "hmc_random"; do
    tag=$(echo $mode | tr ' ' '_' | sed 's/--solver_//')
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --workload C3 --steps 3 --warmup 1 --mode $mode \
      > gpurun_out/modes/$lib.$tag.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/modes/$lib.$tag.json')); print('$lib $tag', '%.4g' % d['value'], '%.3f' % d['roofline']['kernel_ms'])"
  done
done
