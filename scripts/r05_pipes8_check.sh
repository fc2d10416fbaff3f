#!/bin/bash
# After the 8-pipe default from 16,384 chains: the RJ GPU tests, then the default B4 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/r05_pipes8; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rj_native.py tests/test_gpu_reference_runs.py > $O/pytest_rj.log 2>&1 || { tail -30 $O/pytest_rj.log; exit 1; }
tail -1 $O/pytest_rj.log
for c in 4096 16384; do
  timeout -k 10 300 python3 bench.py --workload B4 --mode rj --chains $c --steps 3 --warmup 1 > $O/default_$c.json 2> $O/default_$c.err || exit 1
  python3 -c "import json; d=json.loads(open('$O/default_$c.json').read().strip().splitlines()[-1]); print('default B4 $c', '%.4g' % d['value'])" | tee -a $O/summary.txt
done
