#!/bin/bash
# RJ bench lines at the final sources, three repeats each on one box (B4 and the
# flagship BIGSIM4 at 4,096 chains), then their kernel traces (r05_rjtrace.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_rjrepeat; mkdir -p $O
for wl in B4 BIGSIM4; do
  for r in 1 2 3; do
    timeout -k 10 300 python3 bench.py --workload $wl --mode rj --steps 3 --warmup 1 > $O/${wl}_$r.json 2> $O/${wl}_$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/${wl}_$r.json').read().strip().splitlines()[-1]); print('$wl r$r', '%.4g' % d['value'])" | tee -a $O/summary.txt
  done
done
R05_OUT=r05_rjrepeat bash scripts/r05_rjtrace.sh
