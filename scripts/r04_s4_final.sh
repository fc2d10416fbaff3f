#!/bin/bash
# Session-4 close: round-end evidence (GPU suite, smoke, bench lines with
# fresh rooflines, kernel traces) and the reversible-jump benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/r04_final.sh && bash scripts/r04_rj_bench.sh && bash scripts/r04_rj_benchline.sh
