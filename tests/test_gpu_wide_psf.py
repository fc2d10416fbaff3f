"""Kernel-selection coverage on the pixel-major and window-major multi-star
paths (SURVEY §8(a) a6 and §8(f) next-3 through the C-ABI):

* a PSF wider than the 28-px window bound (FWHM 4.5 px, sigma 1.91 px; the
  window kernels need sigma <= 1.51) on a 48-px image with K = 4: the
  pixel-major kernel is full-image, so the implicit step (rhmc_leapfrog), the
  explicit integrators (rhmc_integrate) and HMC_random (rhmc_hmc_random) all
  take it and agree with the oracle (no window_unsupported error);
* the "multiwin" kernel option forces the window-major kernel (leapfrog_kr with
  kSolverHmcRandom) for HMC_random at K <= 10, where the default is the
  pixel-major kernel: both agree with the oracle and with each other.
Tolerances as tests/test_gpu_parity.py: 1e-9 (q) / 1e-8 (p) relative to
|value| + 1; HMC_random 1e-10 as tests/test_gpu_samplers.py.
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _field(side, K, n_chains, seed, fwhm):
    """A C3-style star field (big-sim4 parameters, power-law fluxes) drawn and
    sampled with PSF FWHM `fwhm` px."""
    img_rng = np.random.RandomState(seed)
    rng = np.random.RandomState(seed + 1)
    par, ftc = workloads.base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    par["fwhm_pix"] = fwhm
    ft, xt, yt = workloads._powlaw_stars(img_rng, K, side, ftc, mag_hi=21.)
    D = workloads._image(side, [(22.5 - 2.5 * np.log10(a / ftc), b, c)
                                for a, b, c in zip(ft, xt, yt)],
                         ftc, par["B_count"], fwhm, img_rng)
    q0 = np.empty((n_chains, 3 * K))
    q0[:, 0::3] = ft * np.exp(0.1 * rng.randn(n_chains, K))
    q0[:, 1::3] = xt + 0.3 * rng.randn(n_chains, K)
    q0[:, 2::3] = yt + 0.3 * rng.randn(n_chains, K)
    p0 = rng.randn(*q0.shape) * np.sqrt(workloads.metric_diag(q0, par))
    return D, q0, p0, par


def _close(got, want, rel, what):
    err = np.abs(got - want) / (np.abs(want) + 1)
    assert err.max() <= rel, (what, err.max())


@pytest.fixture(scope="module")
def wide(gpu_lib):
    D, q0, p0, par = _field(48, 4, 67, 41, 4.5)
    sig = 4.5 / 2.354
    assert (14.0 ** 2) / (2 * sig * sig) < 42.98      # outside the 28-px window bound
    ctx = gpu_lib.Context(D)
    yield gpu_lib, D, q0, p0, par, ctx
    ctx.close()


def test_wide_psf_implicit_vs_oracle(wide, monkeypatch):
    capi, D, q0, p0, par, ctx = wide
    P = capi.make_params(**par)
    n = 40
    q, p, it, st = ctx.leapfrog(P, q0, p0, n, return_info=True)
    assert not (st & capi.STATUS_NONFINITE).any()
    m = R.RefModel(D, dict(par, rows=48, cols=48))
    for c in (0, 33, 66):
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], n, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum(), c
        _close(q[c], qo, 1e-9, "q")
        _close(p[c], po, 1e-8, "p")


@pytest.mark.parametrize("name", ["hmc", "naive", "leap_frog"])
def test_wide_psf_explicit_vs_oracle(wide, name, monkeypatch):
    capi, D, q0, p0, par, ctx = wide
    sid = {"hmc": capi.SOLVER_HMC, "naive": capi.SOLVER_RHMC_NAIVE,
           "leap_frog": capi.SOLVER_RHMC_LEAPFROG}[name]
    P = capi.make_params(**par)
    n = 30
    q, p, st = ctx.integrate(P, sid, q0, p0, n, f_pos=True, return_status=True)
    assert not (st & capi.STATUS_NONFINITE).any()
    m = R.RefModel(D, dict(par, rows=48, cols=48))
    for c in (0, 66):
        qo, po = q0[c].copy(), p0[c].copy()
        for _ in range(n):
            if name == "hmc":
                qo, po = m.hmc_step(qo, po)
            elif name == "naive":
                qo, po = m.rhmc_naive_step(qo, po, True)
            else:
                qo, po = m.rhmc_leapfrog_step(qo, po, True)
        _close(q[c], qo, 1e-9, name + " q")
        _close(p[c], po, 1e-8, name + " p")


def _hmc_random_case(par, q0, seed):
    rs = np.random.RandomState(seed)
    K = q0.shape[1] // 3
    f_lim = 0.9 * np.sort(q0[0, 0::3])[1]             # the faintest stars reach the wall
    hp = dict(par, dt=1., f_lim=f_lim, f_low=1., g_xx=1., g_ff=1., g_ff2=1., g0=1., g1=1.,
              g2=1., use_prior=False)
    p0 = rs.randn(*q0.shape)
    dt = np.tile([1.0, 0.005, 0.005], K)
    steps = rs.randint(1, 20, size=q0.shape[0]).astype(np.int32)
    return hp, f_lim, p0, dt, steps


def test_wide_psf_hmc_random_vs_oracle(wide, monkeypatch):
    capi, D, q0, _, par, ctx = wide
    hp, f_lim, p0, dt, steps = _hmc_random_case(par, q0, 5)
    P = capi.make_params(**hp)
    q, p, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
    m = R.RefModel(D, dict(hp, rows=48, cols=48))
    for k in (0, 1, 40, 66):
        qo, po, flip = m.hmc_random_traj(q0[k], p0[k], dt, int(steps[k]), f_lim)
        assert bool(st[k] & capi.STATUS_REFLECT_F) == flip, k
        _close(q[k], qo, 1e-10, "q")
        _close(p[k], po, 1e-10, "p")


@pytest.mark.parametrize("side,K,n", [(48, 10, 131), (32, 4, 67)])
def test_hmc_random_window_major_forced(gpu_lib, side, K, n, monkeypatch):
    """K <= 10 on a 32/48-px image: pixel-major by default, window-major
    (leapfrog_kr) under the "multiwin" kernel option; both against the oracle."""
    capi = gpu_lib
    D, q0, _, par = _field(side, K, n, 7 + K, 3.4999999999999996)
    hp, f_lim, p0, dt, steps = _hmc_random_case(par, q0, K)
    P = capi.make_params(**hp)
    ctx = capi.Context(D)
    try:
        q, p, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        ctx.set_kernel("multiwin")
        qk, pk, stk = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        idx = np.arange(9)
        qs, ps = ctx.hmc_random(P, dt, q0[idx], p0[idx], steps[idx])
        ctx.set_kernel("auto")
    finally:
        ctx.close()
    np.testing.assert_array_equal(qs, qk[idx])         # window-major: batch invariance
    np.testing.assert_array_equal(ps, pk[idx])
    np.testing.assert_array_equal(st & capi.STATUS_REFLECT_F, stk & capi.STATUS_REFLECT_F)
    _close(qk, q, 1e-10, "window-major vs pixel-major q")
    _close(pk, p, 1e-10, "window-major vs pixel-major p")
    m = R.RefModel(D, dict(hp, rows=side, cols=side))
    for k in (0, n // 2, n - 1):
        qo, po, flip = m.hmc_random_traj(q0[k], p0[k], dt, int(steps[k]), f_lim)
        assert bool(stk[k] & capi.STATUS_REFLECT_F) == flip, k
        _close(qk[k], qo, 1e-10, "q")
        _close(pk[k], po, 1e-10, "p")
