#!/bin/bash
# Round 5 close, part A: the whole GPU suite and smoke, then PMC passes of
# every bench workload at the final kernel sources (PMC_HEAD = the commit).
# Results under gpurun_out/r05_final/ and gpurun_out/r05_pmc_summaries/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
R05_OUT=r05_final bash scripts/r05_suite.sh || exit 1
bash scripts/r05_pmc_all.sh || exit 1
echo final_a done
