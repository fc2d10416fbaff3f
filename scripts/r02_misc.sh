#!/bin/bash
# Round 2: C3 PMC passes + summary, C3 bench line + kernel trace, and a
# 2-rank rehearsal of the N>1 bench path on the one GPU (both ranks pinned to
# device 0 via RHMC_BENCH_DEVICE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash scripts/profile_pmc.sh C3 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_c3 c3 leapfrog_pk 8192000 > gpurun_out/pmc_c3_summary.log 2>&1
cp profiles/pmc_c3.json gpurun_out/pmc_c3.json
bash scripts/profile_wl.sh C3 || exit $?
mkdir -p gpurun_out/ranks2
RHMC_BENCH_DEVICE=0 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 \
  > gpurun_out/ranks2/bench.log 2>&1 || exit $?
grep '^{' gpurun_out/ranks2/bench.log
echo misc done
