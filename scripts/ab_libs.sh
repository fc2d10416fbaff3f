#!/bin/bash
# A/B/C of a bench between the in-tree library and build/variants/lib_<v>.so for each v, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
VS=$1; shift
for r in 1 2; do
  for lib in new $VS; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu "$@" > gpurun_out/ab/$lib.$r.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$lib.$r.json')); print('$lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'], d['fixed_point_iters_per_step']['q_loop_mean'])"
  done
done
