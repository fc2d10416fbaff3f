#!/bin/bash
# PMC passes for C2, C3, C4, C5 at the final sources (scripts/profile_pmc.sh each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for wl in C2 C3 C4 C5; do
  bash scripts/profile_pmc.sh $wl || exit $?
done
echo pmc all done
