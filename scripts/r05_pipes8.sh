#!/bin/bash
# RJ pipes 4 / 6 / 8 A/B on one box (B4 4,096 and 16,384 chains, BIGSIM4 4,096), two repeats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r05_pipes8; mkdir -p $O
for r in 1 2; do
 for cfg in "B4 4096" "B4 16384" "BIGSIM4 4096"; do
  set -- $cfg
  for p in 4 6 8; do
    timeout -k 10 300 python3 bench.py --workload $1 --mode rj --chains $2 --rj-pipes $p --no-cpu --steps 3 --warmup 1 > $O/$1_$2_p${p}_r$r.json 2> $O/$1_$2_p${p}_r$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/$1_$2_p${p}_r$r.json').read().strip().splitlines()[-1]); print('$1 $2 pipes $p r$r', '%.4g' % d['value'])" | tee -a $O/summary.txt
  done
 done
done
