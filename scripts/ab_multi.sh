#!/bin/bash
# GPU suite on the working tree, then the default bench alternating between the
# working tree and each build/variants/lib_<v>.so (R rounds, default 3).
#   ab_multi.sh "v1 v2" [bench args...]     (R=4 ab_multi.sh ... for 4 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
VS=$1; shift
mkdir -p gpurun_out/ab
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
for r in $(seq 1 ${R:-3}); do
  for lib in new $VS; do
    if [ $lib = new ]; then L=hmc-stellar-toy-model_amd/librhmc.so; else L=build/variants/lib_$lib.so; fi
    RHMC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 "$@" > gpurun_out/ab/$lib.$r.json || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$lib.$r.json')); print('$lib $r', '%.4g' % d['value'], '%.4f' % d['roofline']['kernel_ms'])"
  done
done
python3 - $VS <<'PY'
import json, sys, statistics as S
for lib in ["new"] + sys.argv[1:]:
    ms = []
    r = 1
    while True:
        try:
            ms.append(json.load(open("gpurun_out/ab/%s.%d.json" % (lib, r)))["roofline"]["kernel_ms"])
        except OSError:
            break
        r += 1
    print("%-8s kernel ms median %.4f  min %.4f  (%d runs)" % (lib, S.median(ms), min(ms), len(ms)))
PY
