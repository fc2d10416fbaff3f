#!/bin/bash
# Round 5: K > 256 (global-table slotted kernels) — the new tests and the
# many-star / ragged / parity tests around them.  Results under
# gpurun_out/${R05_OUT:-r05_hugek}/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_hugek}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_hugek.py tests/test_gpu_bigk.py tests/test_gpu_ragged.py tests/test_gpu_parity.py \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
grep -E "hugek" $O/pytest.log | head -20
echo hugek done
