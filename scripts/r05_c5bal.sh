#!/bin/bash
# Round 5: balanced window assignment of the window split (leapfrog_kr WS > 1):
# its bit-identity / parity tests, then the C5 window-split sweep at 1024 ..
# 8192 chains, and the native RJ driver's pipe count at B4.
# gpurun_out/r05_c5bal/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_c5bal
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_window_split.py tests/test_gpu_fullsize_multistar.py tests/test_gpu_ragged.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for n in 1024 2048 4096 8192; do
  for ws in 1 2 4; do
    timeout -k 10 300 python3 bench.py --workload C5 --chains $n --no-cpu --no-e2e --steps 3 --warmup 1 --window-split $ws > $O/c5_${n}_ws$ws.json 2> $O/c5_${n}_ws$ws.err || { tail -20 $O/c5_${n}_ws$ws.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c5_${n}_ws$ws.json').read().strip().splitlines()[-1]); print('c5 $n ws$ws', '%.4g' % d['value'], d['roofline']['kernel_ms'])"
  done
done
for pp in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --workload B4 --mode rj --rj-pipes $pp --steps 4 --warmup 1 > $O/rj_b4_p$pp.json 2> $O/rj_b4_p$pp.err || { tail -20 $O/rj_b4_p$pp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rj_b4_p$pp.json').read().strip().splitlines()[-1]); print('rj b4 pipes $pp', '%.4g' % d['value'])"
done
echo c5bal done
