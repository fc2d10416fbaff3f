#!/bin/bash
# C2 throughput of the single-star kernel variants at several chain counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c2v
for k in tiled1 tiled2; do
  for n in 4096 8192 16384; do
    RHMC_KERNEL=$k timeout -k 10 120 python3 bench.py --chains $n --steps 5 --warmup 1 --no-cpu > gpurun_out/c2v/${k}_$n.log 2>&1 || exit $?
  done
done
