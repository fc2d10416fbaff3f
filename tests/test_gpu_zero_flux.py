"""A star at zero flux: the kernels fold f into the PSF column
factors and divide the flux sum by f again, which at f = 0 exactly would give
0/0.  The reference's -sum psf (D/Lambda - 1) (sampler_RHMC.py:404) is finite
there without the prior, so the kernels fold 2^-600 for |f| < 2^-500
(flux_fold, rhmc_wave.hpp).  Chains starting at f = 0 (and at a subnormal f)
against the CPU oracle: the implicit step on the one-star register-window
kernel and on the pixel-major / window-major multi-star kernels, and the
explicit HMC leapfrog (unit metric, :628-645), exact iteration counts and
the usual 1e-9 / 1e-8 parity bar."""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _case(name, n):
    wl = workloads.make(name, n_chains=n)
    q0, p0 = wl.q0.copy(), wl.p0.copy()
    q0[0, 0] = 0.0                     # star 0 of chain 0 at zero flux
    q0[1, 0] = 5e-324                  # the smallest subnormal
    q0[2, 3 if wl.K > 1 else 0] = -0.0
    return wl, q0, p0


@pytest.mark.parametrize("name,kernel", [("C2", "auto"), ("C2", "lane1"), ("C2", "generic"),
                                         ("C3", "auto"), ("C3", "multiwin")])
def test_zero_flux_implicit_step(gpu_lib, name, kernel):
    capi = gpu_lib
    wl, q0, p0 = _case(name, 6)
    ctx = capi.Context(wl.D, kernel=kernel)
    P = capi.make_params(**wl.params)
    q, p, it, st = ctx.leapfrog(P, q0, p0, 5, return_info=True)
    ctx.close()
    assert not (st & capi.STATUS_NONFINITE).any(), st
    m = R.RefModel(wl.D, dict(wl.params, rows=wl.D.shape[0], cols=wl.D.shape[1]))
    for c in range(3):
        g = m.dphidq(q0[c])
        assert np.isfinite(g).all()
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], 5, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), (c, it[c], NP.sum(), NQ.sum())
        assert_state_close(q[c], qo, 1e-9, "%s %s q chain %d" % (name, kernel, c))
        assert_state_close(p[c], po, 1e-8, "%s %s p chain %d" % (name, kernel, c))


@pytest.mark.parametrize("name", ["C2", "C3"])
def test_zero_flux_gradient_and_hmc(gpu_lib, name):
    capi = gpu_lib
    wl, q0, p0 = _case(name, 4)
    ctx = capi.Context(wl.D)
    P = capi.make_params(**wl.params)
    m = R.RefModel(wl.D, dict(wl.params, rows=wl.D.shape[0], cols=wl.D.shape[1]))
    g = ctx.gradient(P, q0, kind=0)
    for c in range(3):
        want = m.dVdq(q0[c])
        assert np.abs(g[c] - want).max() / (np.abs(want).max() + 1) < 1e-10, c
    q, p = ctx.integrate(P, capi.SOLVER_HMC, q0, p0, 4, f_pos=False)
    ctx.close()
    for c in range(3):
        qo, po = q0[c].copy(), p0[c].copy()
        for _ in range(4):
            qo, po = m.hmc_step(qo, po)
        assert_state_close(q[c], qo, 1e-9, "%s HMC q chain %d" % (name, c))
        assert_state_close(p[c], po, 1e-8, "%s HMC p chain %d" % (name, c))
