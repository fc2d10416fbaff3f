#!/bin/bash
# Round 5: window split 8 (512-thread workgroups) on the C5 shard — the
# split tests, then A/B of --window-split 4 / 8 at 1024 and 2048 chains.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_ws8}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_window_split.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --workload C5 --no-cpu --no-e2e --steps 5 --warmup 1 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', '%.4g' % d['value'], r.get('kernel_ms'))"
}
for r in 1 2; do
  run s1024_ws4_r$r --chains 1024 --window-split 4
  run s1024_ws8_r$r --chains 1024 --window-split 8
done
run s2048_ws4 --chains 2048 --window-split 4
run s2048_ws8 --chains 2048 --window-split 8
run s4096_ws4 --chains 4096 --window-split 4
run s4096_ws8 --chains 4096 --window-split 8
echo ws8 done
