#!/bin/bash
# A/B of the default bench between the in-tree library ("new") and
# build/variants/lib_<name>.so for each name given, alternating on one box.
#   ab_lib.sh "name1 name2 ..." [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
VS=$1; shift
for r in 1 2 3; do
  for lib in new $VS; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-e2e --steps 20 --warmup 3 "$@" > gpurun_out/ab/$lib.$r.json || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/$lib.$r.json').read().strip().splitlines()[-1]); print('$lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
