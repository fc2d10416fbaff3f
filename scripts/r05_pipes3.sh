#!/bin/bash
# RJ pipes 3 / 4 / 6 / 8 (GPU_MAX_HW_QUEUES 4 on the box: streams share queues).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_pipes3}
mkdir -p $O
for r in 1 2; do
  for p in 3 4 6 8; do
    for wl in BIGSIM4 B4; do
      timeout -k 10 300 python3 bench.py --workload $wl --mode rj --steps 5 --warmup 1 --rj-pipes $p > $O/${wl}_p${p}_r$r.json 2> $O/${wl}_p${p}_r$r.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/${wl}_p${p}_r$r.json').read().strip().splitlines()[-1]); print('$wl p$p r$r', '%.4g' % d['value'], round(d['ms_per_step'],1), round(d['rj']['native_call_s_last']*1e3,1))"
    done
  done
done
echo pipes3 done
