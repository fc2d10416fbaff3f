#!/bin/bash
# Bench line + rocprofv3 kernel-trace stats for each workload (full 500-step
# launches), written under gpurun_out/wl_<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for WL in "$@"; do
  TAG=$(echo "$WL" | tr 'A-Z' 'a-z')
  OUT=gpurun_out/wl_$TAG
  mkdir -p "$OUT"
  timeout -k 10 600 python3 bench.py --workload $WL --steps ${STEPS:-3} --warmup 1 --no-cpu > "$OUT/bench.log" 2>&1 || exit $?
  tail -1 "$OUT/bench.log" > "$OUT/bench.json"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --workload $WL --steps ${STEPS:-3} --warmup 1 --no-cpu --no-e2e > "$OUT/rocprof.log" 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], '%.4e' % d['value'], 'kernel_ms %.3f' % d['roofline']['kernel_ms'])" "$OUT/bench.json" $WL
done
