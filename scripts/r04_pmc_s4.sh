#!/bin/bash
# PMC passes for every bench workload with a roofline (C2-C5, B3, B4) at the
# current sources (scripts/profile_pmc.sh each); summarised locally with
# scripts/pmc_summary.py into profiles/pmc_<wl>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for wl in C2 C3 C4 C5 B3 B4; do
  bash scripts/profile_pmc.sh $wl || exit $?
done
echo pmc all done
