#!/bin/bash
# Round 5: K > 256 through the ragged entry points, the kinetic kernel and the
# reversible-jump driver (N_max up to 1024), with the RJ and window-split tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R05_OUT:-r05_bigrj}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ragged.py tests/test_gpu_rj_native.py tests/test_gpu_hugek.py \
  tests/test_gpu_window_split.py tests/test_gpu_reference_runs.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
echo bigrj done
