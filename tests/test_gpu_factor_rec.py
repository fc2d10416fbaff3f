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
Both run on the register-window kernel (`auto` at these batch sizes) and on the
lane-group kernel forced to 1 and 4 lanes per chain, whose runs-of-7
recurrences (rhmc_tiledl.hpp) fall back per lane: chains 8-11 sit 20-85 px
outside the image, so some of their window offsets are inside rec_vmax (55.6
px) and some not.
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


KERNELS = ["auto", "lane1", "lane4"]


@pytest.mark.parametrize("kernel", KERNELS)
def test_far_chain_wave_and_edges(gpu_lib, monkeypatch, kernel):
    monkeypatch.setattr(gpu_lib, "DEFAULT_KERNEL", kernel)
    wl = workloads.make("C2", n_chains=12)
    q0, p0 = wl.q0.copy(), wl.p0.copy()
    q0[2, 1], q0[2, 2] = 300.0, -250.0     # wave 0: far outside (direct factors)
    q0[4, 1], q0[4, 2] = 0.4, 46.8         # wave 1: clamped windows at the edges
    q0[5, 1], q0[5, 2] = 47.3, 1.2
    q0[6, 1], q0[6, 2] = -0.6, 24.0        # just outside the image
    q0[7, 1], q0[7, 2] = 24.0, 47.9
    q0[8, 1] = -20.0                       # rows 20.5-47.5 px off: recurrence
    q0[9, 1] = -40.0                       # rows 40.5-67.5 px off: straddles rec_vmax
    q0[10, 2] = 85.0                       # columns 37.5-64.5 px off: straddles it
    q0[11, 1], q0[11, 2] = 70.0, -45.0     # both
    _check(gpu_lib, wl.D, wl.params, q0, p0, 30)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("fwhm", [1.2, 2.5])
def test_psf_widths_either_side_of_the_range_guard(gpu_lib, monkeypatch, fwhm, kernel):
    monkeypatch.setattr(gpu_lib, "DEFAULT_KERNEL", kernel)
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


@pytest.mark.parametrize("kernel", ["pixmajor", "multiwin"])
def test_many_star_far_chain_and_narrow_psf(gpu_lib, kernel):
    """The multi-star kernels' factor tables by recurrence (PixK::tables_rec)
    fall back to direct exps when a run starts outside rec_vmax: a chain whose
    star sits far outside the image (x = 300) and a narrow PSF (FWHM 1.2 px)
    with 2 <= K <= 10, both chains of the wave against the oracle."""
    capi = gpu_lib
    from rhmc_amd.photometry import mag2flux
    for fwhm in (3.4999999999999996, 1.2):
        par, ftc = workloads.base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
        par["fwhm_pix"] = fwhm
        rng = np.random.RandomState(5)
        K = 4
        stars = [(17. + k, 10. + 8 * k, 30. - 5 * k) for k in range(K)]
        D = workloads._image(48, stars, ftc, par["B_count"], fwhm, rng)
        n = 4
        q0 = np.empty((n, 3 * K))
        q0[:, 0::3] = [mag2flux(s[0]) * ftc for s in stars]
        q0[:, 1::3] = [s[1] for s in stars]
        q0[:, 2::3] = [s[2] for s in stars]
        q0 *= 1 + 0.01 * rng.randn(n, 3 * K)
        q0[1, 1] = 300.0                    # chain 1 (wave-mate of chain 0): far out
        q0[2, 5] = -280.0                   # chain 2: far out in y
        p0 = rng.randn(n, 3 * K) * np.sqrt(workloads.metric_diag(q0, par))
        ctx = capi.Context(D, kernel=kernel)
        P = capi.make_params(**par)
        q, p, it, st = ctx.leapfrog(P, q0, p0, 20, return_info=True)
        ctx.close()
        m = R.RefModel(D, dict(par, rows=48, cols=48))
        for c in range(n):
            qo, po, NP, NQ = m.trajectory(q0[c], p0[c], 20, record=False)
            assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), (fwhm, c)
            assert_state_close(q[c], qo, 1e-9, "q fwhm %g chain %d" % (fwhm, c))
            assert_state_close(p[c], po, 1e-8, "p fwhm %g chain %d" % (fwhm, c))
