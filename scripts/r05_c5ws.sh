#!/bin/bash
# Round 5: C5 at its 8-GPU share (1024 chains per GPU): window-split sweep and
# the shard's PMC passes (profiles/pmc_c5_1024.json).  gpurun_out/r05_c5ws/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_c5ws
mkdir -p $O
for ws in 1 2 4 0; do
  timeout -k 10 300 python3 bench.py --workload C5 --chains 1024 --no-cpu --no-e2e --steps 5 --warmup 1 --window-split $ws > $O/ws$ws.json 2> $O/ws$ws.err || { tail -20 $O/ws$ws.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ws$ws.json').read().strip().splitlines()[-1]); print('ws$ws', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
done
PMC_ARGS="--chains 1024" PMC_TAG=c5_1024 bash scripts/profile_pmc.sh C5 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
echo c5ws done
