#!/bin/bash
# Full GPU session: tests + bench + kernel-trace stats, then the C2 PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_check.sh all || exit $?
bash scripts/profile_pmc.sh C2 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_c2 c2 leapfrog 2048000 "${RHMC_HEAD:-}" > gpurun_out/pmc_summary.log 2>&1
cp profiles/pmc_c2.json gpurun_out/pmc_c2.json
echo all done
