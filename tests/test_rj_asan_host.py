"""Host AddressSanitizer run of the native reversible-jump driver
(librhmc_rj, include/rhmc_rj.h): `make -C hmc-stellar-toy-model_amd/host asan`
builds tests/native/rj_asan.cpp with the driver's source under
-fsanitize=address; it runs rhmc_rj_run_physics with C stand-in physics over
every move mix, one and two pipes, dead ends, schedules, records on and off,
and every error path — no GPU needed.  ASan aborts on the first heap error, so
exit status 0 and "rj asan ok" mean a clean run."""
import os
import subprocess

import pytest

from conftest import PKG_DIR, ROOT

BIN = os.path.join(ROOT, "build", "asan", "rj_asan")


def test_rj_driver_under_asan():
    if not os.path.exists(os.path.join(PKG_DIR, "librhmc.so")):
        pytest.skip("librhmc.so not built")
    subprocess.run(["make", "-C", os.path.join(PKG_DIR, "host"), "asan"], check=True,
                   capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1")
    r = subprocess.run([BIN], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rj asan ok" in r.stdout
    assert "AddressSanitizer" not in r.stderr


@pytest.mark.gpu
def test_rj_driver_on_the_engine_under_asan(gpu_lib):
    """rhmc_rj_run on a real context (staged groups on concurrent streams,
    one and two pipes, K from 1 to 13) with the driver's host code under ASan;
    leak detection off (the HIP runtime keeps process-lifetime allocations)."""
    if not os.path.exists(BIN):
        pytest.skip("build/asan/rj_asan not built (make -C hmc-stellar-toy-model_amd/host asan)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([BIN, "gpu"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "rj asan gpu ok" in r.stdout
    assert "AddressSanitizer" not in r.stderr
