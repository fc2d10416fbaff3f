"""PSF factors by recurrence in the register-window kernels (rhmc_tiledr.hpp
factors_rec) against the oracle, through the C-ABI (rhmc_leapfrog):

* a wave whose chains sit far outside their windows (x = 300, y = -250; the
  window clamps to the image corner) takes the direct-exp factors, the other
  waves of the same launch the recurrence; every chain agrees with the oracle;
* clamped windows at the image edges (star within a few px of a border, and
  just outside it) on the recurrence path;
* PSF widths on both sides of the recurrence's range guard: FWHM 1.2 px
  (sigma 0.51, rec_vmax 11.6 < the window offsets: direct factors) and
  FWHM 2.5 px (recurrence), with images drawn at that width.
Tolerances as tests/test_gpu_parity.py: 1e-9 (q) / 1e-8 (p) relative to
|value| + 1 after the trajectory, iteration counts exact.
"""
import numpy as np
import pytest

from helpers import assert_state_close
from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _check(capi, D, par, q0, p0, steps, chains=None):
    ctx = capi.Context(D)
    P = capi.make_params(**par)
    q, p, it, st = ctx.leapfrog(P, q0, p0, steps, return_info=True)
    ctx.close()
    m = R.RefModel(D, dict(par, rows=D.shape[0], cols=D.shape[1]))
    for c in (range(len(q0)) if chains is None else chains):
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], steps, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), (c, it[c], NP.sum(), NQ.sum())
        assert_state_close(q[c], qo, 1e-9, "q chain %d" % c)
        assert_state_close(p[c], po, 1e-8, "p chain %d" % c)
    return q, p, st


def test_far_chain_wave_and_edges(gpu_lib, monkeypatch):
    wl = workloads.make("C2", n_chains=12)
    q0, p0 = wl.q0.copy(), wl.p0.copy()
    q0[2, 1], q0[2, 2] = 300.0, -250.0     # wave 0: far outside (direct factors)
    q0[4, 1], q0[4, 2] = 0.4, 46.8         # wave 1: clamped windows at the edges
    q0[5, 1], q0[5, 2] = 47.3, 1.2
    q0[6, 1], q0[6, 2] = -0.6, 24.0        # just outside the image
    q0[7, 1], q0[7, 2] = 24.0, 47.9
    _check(gpu_lib, wl.D, wl.params, q0, p0, 30)


@pytest.mark.parametrize("fwhm", [1.2, 2.5])
def test_psf_widths_either_side_of_the_range_guard(gpu_lib, monkeypatch, fwhm):
    par, ftc = workloads.base_params(dt=0.1)
    par["fwhm_pix"] = fwhm
    rng = np.random.RandomState(int(fwhm * 10))
    xt, yt = 23.7, 24.2
    D = workloads._image(48, [(19., xt, yt)], ftc, par["B_count"], fwhm, rng)
    n = 8
    f = workloads.mag2flux(19.) * ftc
    q0 = np.stack([f * (1 + 0.1 * rng.randn(n)), xt + 0.5 * rng.randn(n),
                   yt + 0.5 * rng.randn(n)], 1)
    q0[3, 1] = 2.2                          # one clamped window
    p0 = rng.randn(*q0.shape) * np.sqrt(workloads.metric_diag(q0, par))
    _check(gpu_lib, D, par, q0, p0, 30)
