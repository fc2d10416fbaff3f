#!/bin/bash
# Kernel A/B for many stars on small images (round 4): the dense kernel
# (rhmc_dense.hpp) against the multi-star register-window kernel and the
# windowed one, on the reference's big-sim geometries and a K sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ab() {
  echo "=== $*"
  timeout -k 10 240 python3 tools/kernel_ab.py "$@" >> gpurun_out/dense_ab.txt 2>&1
  local rc=$?
  tail -n 4 gpurun_out/dense_ab.txt
  [ $rc -eq 0 ] || { echo "kernel_ab rc=$rc"; exit $rc; }
}
: > gpurun_out/dense_ab.txt
ab B4 dense multiwin windowed --chains 2048 --reps 2 --launches 2
ab B3 dense windowed --chains 2048 --reps 2 --launches 2
for wl in S32K12 S32K16 S32K24 S48K12 S48K16 S48K24 S48K40; do
  ab $wl dense multiwin --chains 4096 --reps 2 --launches 2
done
ab S48K10 dense pixmajor --chains 4096 --reps 2 --launches 2
echo done
