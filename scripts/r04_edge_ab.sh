#!/bin/bash
# A/B: wave-uniform skip of the one-star edge-reflection blocks (in-tree "new")
# against the library before it (build/variants/lib_base.so); parity tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "parity or edge or wall or fullsize or delta or coupling or lane or factor or qloop or mh_fused or energy_k1" > gpurun_out/pt_edge.log 2>&1 || { tail -30 gpurun_out/pt_edge.log; exit 1; }
tail -1 gpurun_out/pt_edge.log
bash scripts/ab_lib.sh base || exit 1
bash scripts/ab_lib.sh base --workload C4 --steps 5 --warmup 1 || exit 1
