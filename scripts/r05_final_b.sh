#!/bin/bash
# Round 5 close, part B: every bench line and the kernel-trace summaries at the
# final sources (scripts/r05_head.sh into gpurun_out/r05_final/), plus the RJ
# line at 16,384 chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R05_OUT=r05_final bash scripts/r05_head.sh || exit 1
O=gpurun_out/r05_final
timeout -k 10 400 python3 bench.py --workload B4 --mode rj --chains 16384 --steps 3 --warmup 1 > $O/rj_b4_16k.json 2> $O/rj_b4_16k.err || exit 1
echo final_b done
