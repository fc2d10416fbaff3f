#!/bin/bash
# Round-end evidence at HEAD on one GPU box: smoke + GPU suite + C2 bench /
# 2-rank rehearsal / kernel trace (gpu_check.sh), bench lines + kernel traces
# for C1 C3 C4 C5 (profile_wl.sh), PMC passes + summaries for C2 C3 C5, and two
# dispatch A/Bs (C5 window split at 8192 chains, C4 shard lanes per chain).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
REV=${1:-unknown}
bash scripts/gpu_check.sh all || exit $?
bash scripts/profile_wl.sh C1 C3 C4 C5 || exit $?
for spec in C2:2048000 C3:8192000 C5:4096000; do
  WL=${spec%%:*}; CS=${spec#*:}; TAG=$(echo "$WL" | tr 'A-Z' 'a-z')
  bash scripts/profile_pmc.sh $WL || exit $?
  python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG $TAG leapfrog $CS "$REV" > gpurun_out/pmc_$TAG/summary.log 2>&1 || exit $?
  cp profiles/pmc_$TAG.json gpurun_out/pmc_$TAG.json
done
mkdir -p gpurun_out/kab
timeout -k 10 300 python3 tools/kernel_ab.py C5 auto --window-split 1 2 --reps 2 --launches 3 > gpurun_out/kab/c5_ws.txt 2>&1 || exit $?
timeout -k 10 300 python3 tools/kernel_ab.py C4 auto lane4 --chains 131072 --reps 2 --launches 3 > gpurun_out/kab/c4_lpc.txt 2>&1 || exit $?
cat gpurun_out/kab/*.txt
echo all done
