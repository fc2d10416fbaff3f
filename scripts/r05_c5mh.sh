#!/bin/bash
# Round 5: C5 MH with run_RHMC's f_pos=True — acceptance vs trajectory length
# and start floor.  gpurun_out/r05_c5mh/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05_c5mh
mkdir -p $O
for cfg in "10 1.5" "10 3" "20 3" "50 3" "10 10" "50 10"; do
  set -- $cfg
  n=leap$1_floor$2
  timeout -k 10 300 python3 bench.py --workload C5 --mode mh --mh-iter 5 --leap $1 --mh-floor $2 --no-cpu --steps 2 --warmup 1 --f-pos 1 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', '%.4g' % d['value'], d['mh_accept_rate_last_launch'])"
done
echo c5mh done
