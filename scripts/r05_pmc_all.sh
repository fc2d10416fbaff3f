#!/bin/bash
# PMC passes for every bench workload at the final kernel sources
# (scripts/profile_pmc.sh each, one counter group per pass), then the
# summaries into gpurun_out/r05_pmc_summaries/ (copied to profiles/ after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for wl in C2 C3 C4 C5 B3 B4; do
  bash scripts/profile_pmc.sh $wl || exit $?
done
PMC_ARGS="--chains 1024" PMC_TAG=c5_1024 bash scripts/profile_pmc.sh C5 || exit $?
S=gpurun_out/r05_pmc_summaries
mkdir -p $S
HEAD=${PMC_HEAD:-unknown}
sum() { python3 scripts/pmc_summary.py gpurun_out/pmc_$1 $1 leapfrog $2 $HEAD > /dev/null && cp profiles/pmc_$1.json $S/; }
sum c2 2048000 && sum c3 8192000 && sum c4 524288000 && sum c5 4096000 && sum b3 409600 && \
  sum b4 409600 && sum c5_1024 512000 || exit 1
echo pmc all done
