#!/bin/bash
# C5 A/B: in-tree library vs build/variants/lib_<name>.so at 8192 chains (one
# GPU) and at the 1024-chain share of an 8-GPU run, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
V=${1:-old}
for r in 1 2; do
  for lib in new $V; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    for n in 8192 1024; do
      RHMC_LIB=$L timeout -k 10 200 python3 tools/kernel_ab.py C5 auto --chains $n --reps 1 --launches 2 2>/dev/null | sed "s/^/$lib /" || exit $?
    done
  done
done
