"""The fixed-point stopping test at the delta boundary.

The reference stops each fixed-point loop at the first iteration whose
max |dq| (or |dp|) is <= delta (sampler_RHMC.py:528-545).  The kernels form
the same iterates in a division-lean affine form (and the one-star kernels'
q-loop by binary powering across lanes), which agree with the reference's to
a few ulp, not bit for bit.  When an iterate's test value sits within those
ulps of delta the loop may stop one iteration earlier or later than the
reference.  These cases put delta exactly on (and one ulp either side of) a
test value the reference computed, and assert the bound: per loop at most
one iteration of difference, and the resulting state within the distance
that extra iteration moves it (<= delta-scale) of the reference's — far
inside the trajectory parity bar."""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _edges(m, q, p, loop):
    tr = {}
    m.step(q, p, 1e-6, 1000, trace=tr)
    vals = tr[loop]
    # test values that were > 1e-6 (a later iteration ran) are edges to sit on
    return [v for v in vals[:-1] if v > 1e-6][:2]


@pytest.mark.parametrize("kernel", ["auto", "regwin32", "lane4", "generic"])
@pytest.mark.parametrize("loop", ["dq", "dp"])
def test_delta_on_a_reference_test_value(gpu_lib, kernel, loop):
    capi = gpu_lib
    wl = workloads.make("C2", n_chains=6)
    par = dict(wl.params, rows=48, cols=48)
    m = R.RefModel(wl.D, par)
    ctx = capi.Context(wl.D, kernel=kernel)
    checked = diffs = 0
    for c in range(wl.n_chains):
        for d in _edges(m, wl.q0[c], wl.p0[c], loop):
            for delta in (np.nextafter(d, 0), d, np.nextafter(d, np.inf)):
                P = capi.make_params(**dict(wl.params, delta=float(delta)))
                qg, pg, it, _ = ctx.leapfrog(P, wl.q0[c], wl.p0[c], 1, return_info=True)
                qo, po, n_p, n_q = m.step(wl.q0[c], wl.p0[c], float(delta), 1000)
                assert abs(int(it[0]) - n_p) <= 1 and abs(int(it[1]) - n_q) <= 1, \
                    (c, delta, it, n_p, n_q)
                diffs += int(it[0] != n_p or it[1] != n_q)
                # one iteration more or less moves the state by about the test
                # value (a contraction); scale by the step's dt-weighted metric
                tol = 1e-11 if (it[0] == n_p and it[1] == n_q) else 50 * d
                assert np.abs(qg - qo).max() / (np.abs(qo).max() + 1) <= tol, (c, delta)
                assert np.abs(pg - po).max() / (np.abs(po).max() + 1) <= max(tol, 1e-10), \
                    (c, delta)
                checked += 1
    ctx.close()
    print("%s %s: %d delta-edge steps, %d with a one-iteration difference"
          % (kernel, loop, checked, diffs))
    assert checked >= 6
