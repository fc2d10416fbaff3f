#!/bin/bash
# Bench lines of the K > 256 completeness path (global-table slotted kernels)
# beside K = 256 (LDS tables) on the same image sizes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_hugek_bench}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --no-e2e "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', '%.4g' % d['value'], r.get('kernel_ms'), d['config'].get('workload'))"
}
run s64k256 --workload S64K256 --chains 1024 --leap 10 --steps 2 --warmup 1
run s64k300 --workload S64K300 --chains 1024 --leap 10 --steps 2 --warmup 1
run s128k700 --workload S128K700 --chains 1024 --leap 10 --steps 2 --warmup 1
echo hugek bench done
