#!/bin/bash
# Round 2 end: C3 PMC passes + summary (pixel-major kernel after the
# reduce-scatter), C3 and C5 bench lines + kernel-trace summaries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
bash scripts/profile_pmc.sh C3 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_c3 c3 leapfrog_pk 8192000 > gpurun_out/pmc_c3_summary.log 2>&1
cp profiles/pmc_c3.json gpurun_out/pmc_c3.json
bash scripts/profile_wl.sh C3 C5 || exit $?
echo c3c5 done
