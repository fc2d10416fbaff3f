"""The explicit integrators on the one-star register-
window kernel (integrate_k1_tiledr, rhmc_tiledr.hpp) through the C-ABI
rhmc_integrate, at the bench's C2 geometry:

* oracle sample: chains of the full 4096-chain launch match oracle/rhmc_ref's
  hmc_step / rhmc_naive_step / rhmc_leapfrog_step (sampler_RHMC.py:628-645,
  :690-728) after 100 steps to 1e-9 (q) / 1e-8 (p) relative to |value| + 1,
  flux wall on (f_pos), with and without the flux prior;
* the windowed kernel (kernel option "windowed", the other implementation of the
  same step) agrees on the whole batch to the same tolerance;
* batch invariance: a ragged subset run on its own is bit-identical;
* a 32-px image (C1's) and a 64-px image take the same kernel family.
The 16x16 reference goldens (tests/golden/solvers.npz) go through the windowed
kernel (test_gpu_sampler.py::test_single_gym_alternative_integrators).
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu

N_STEPS = 100
SOLVERS = ("hmc", "naive", "leap_frog")


def _sid(capi, name):
    return {"hmc": capi.SOLVER_HMC, "naive": capi.SOLVER_RHMC_NAIVE,
            "leap_frog": capi.SOLVER_RHMC_LEAPFROG}[name]


def _oracle_run(m, name, q, p, n):
    q, p = q.copy(), p.copy()
    for _ in range(n):
        if name == "hmc":
            q, p = m.hmc_step(q, p)
        elif name == "naive":
            q, p = m.rhmc_naive_step(q, p, True)
        else:
            q, p = m.rhmc_leapfrog_step(q, p, True)
    return q, p


def _case(wl, name, **kw):
    """Parameters and starting momenta: the workload's RHMC ones, except for
    unit-metric HMC, which gets p ~ N(0, 1) (run_single_HMC, :620) and
    dt = 0.05 — at the workload's dt = 0.1 with momenta scaled by sqrt(H) its
    leapfrog is past the stability limit on the position coordinates for some
    chains (a 1e-13 perturbation grows to O(1) in 100 steps, measured on the
    oracle), which no two implementations can agree on."""
    params = dict(wl.params, **kw)
    if name != "hmc":
        return params, wl.p0
    params["dt"] = 0.05
    return params, np.random.RandomState(3).randn(*wl.p0.shape)


def _check_sample(capi, wl, params, p0, name, q, p, chains):
    par = dict(params)
    par["rows"], par["cols"] = wl.D.shape
    m = R.RefModel(wl.D, par)
    for c in chains:
        qo, po = _oracle_run(m, name, wl.q0[c], p0[c], N_STEPS)
        err_q = np.abs(q[c] - qo) / (np.abs(qo) + 1)
        err_p = np.abs(p[c] - po) / (np.abs(po) + 1)
        assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (name, c, err_q, err_p)


@pytest.fixture(scope="module")
def c2(gpu_lib):
    wl = workloads.make("C2")
    ctx = gpu_lib.Context(wl.D)
    yield gpu_lib, wl, ctx
    ctx.close()


@pytest.mark.parametrize("prior", [False, True])
@pytest.mark.parametrize("name", SOLVERS)
def test_c2_explicit_vs_oracle_and_windowed(c2, name, prior, monkeypatch):
    capi, wl, ctx = c2
    params, p0 = _case(wl, name, use_prior=prior, alpha=2.0)
    P = capi.make_params(**params)
    q, p, st = ctx.integrate(P, _sid(capi, name), wl.q0, p0, N_STEPS, f_pos=True,
                             return_status=True)
    assert not (st & capi.STATUS_NONFINITE).any()
    _check_sample(capi, wl, params, p0, name, q, p, (0, 1, 777, 2048, 2913, 4095))
    ctx.set_kernel("windowed")
    try:
        qw, pw = ctx.integrate(P, _sid(capi, name), wl.q0, p0, N_STEPS, f_pos=True)
    finally:
        ctx.set_kernel("auto")
    err_q = np.abs(q - qw) / (np.abs(qw) + 1)
    err_p = np.abs(p - pw) / (np.abs(pw) + 1)
    assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (err_q.max(), err_p.max())


@pytest.mark.parametrize("name", SOLVERS)
def test_c2_explicit_batch_invariance(c2, name):
    capi, wl, ctx = c2
    params, p0 = _case(wl, name)
    P = capi.make_params(**params)
    q, p = ctx.integrate(P, _sid(capi, name), wl.q0, p0, 50, f_pos=True)
    idx = np.r_[3:10, 2000:2006]                    # 13 chains: a ragged last wave
    qs, ps = ctx.integrate(P, _sid(capi, name), wl.q0[idx], p0[idx], 50, f_pos=True)
    np.testing.assert_array_equal(qs, q[idx])
    np.testing.assert_array_equal(ps, p[idx])
    q2, p2 = ctx.integrate(P, _sid(capi, name), wl.q0, p0, 50, f_pos=True)
    np.testing.assert_array_equal(q2, q)            # deterministic
    np.testing.assert_array_equal(p2, p)


@pytest.mark.parametrize("side", [32, 64])
@pytest.mark.parametrize("name", SOLVERS)
def test_explicit_other_image_sides(gpu_lib, side, name):
    capi = gpu_lib
    rng = np.random.RandomState(5 + side)
    c = side / 2.0
    setup = R.default_setup()
    D = R.model_image(side, side, [(R.mag2flux(19.) * setup["flux_to_count"], c + 0.2, c - 0.3)],
                      setup["B_count"], setup["fwhm_pix"])
    D = rng.poisson(D).astype(np.float64)
    wl = workloads.make("C2", n_chains=9)
    q0 = wl.q0.copy()
    q0[:, 1:] += c - 24.0                           # star near this image's centre
    params, p0 = _case(wl, name)
    ctx = capi.Context(D)
    try:
        P = capi.make_params(**params)
        q, p = ctx.integrate(P, _sid(capi, name), q0, p0, 60, f_pos=True)
    finally:
        ctx.close()
    par = dict(params)
    par["rows"], par["cols"] = D.shape
    m = R.RefModel(D, par)
    for k in (0, 4, 8):
        qo, po = _oracle_run(m, name, q0[k], p0[k], 60)
        err_q = np.abs(q[k] - qo) / (np.abs(qo) + 1)
        err_p = np.abs(p[k] - po) / (np.abs(po) + 1)
        assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (side, name, k, err_q, err_p)


# ---- many stars: the multi-star register-window kernel (leapfrog_kr<..., SOLVER>)
def _star_field(side, K, n_chains, seed):
    """A C3-style workload (big-sim4 parameters, power-law fluxes) on a
    side x side image with K stars."""
    img_rng = np.random.RandomState(seed)
    rng = np.random.RandomState(seed + 1)
    par, ftc = workloads.base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    ft, xt, yt = workloads._powlaw_stars(img_rng, K, side, ftc)
    D = workloads._image(side, [(22.5 - 2.5 * np.log10(a / ftc), b, c)
                                for a, b, c in zip(ft, xt, yt)],
                         ftc, par["B_count"], par["fwhm_pix"], img_rng)
    q0 = np.empty((n_chains, 3 * K))
    q0[:, 0::3] = ft * np.exp(0.1 * rng.randn(n_chains, K))
    q0[:, 1::3] = xt + 0.5 * rng.randn(n_chains, K)
    q0[:, 2::3] = yt + 0.5 * rng.randn(n_chains, K)
    p0 = rng.randn(*q0.shape) * np.sqrt(workloads.metric_diag(q0, par))
    return workloads.Workload("field", D, q0, p0, par, 0, K, "")


@pytest.mark.parametrize("name", SOLVERS)
@pytest.mark.parametrize("side,K,n_chains", [(48, 10, 16384),   # C3: LDS factor tables
                                             (32, 4, 301),      # pixel-major, 32-px image
                                             (48, 20, 37),      # exp path, one star slot
                                             (64, 40, 5)])      # two star slots per lane
def test_many_star_explicit_vs_oracle(gpu_lib, name, side, K, n_chains, monkeypatch):
    capi = gpu_lib
    wl = workloads.make("C3") if K == 10 else _star_field(side, K, n_chains, 11 + K)
    params, p0 = _case(wl, name)
    n = 30
    ctx = capi.Context(wl.D)
    try:
        P = capi.make_params(**params)
        q, p, st = ctx.integrate(P, _sid(capi, name), wl.q0, p0, n, f_pos=True,
                                 return_status=True)
        assert not (st & capi.STATUS_NONFINITE).any()
        ctx.set_kernel("windowed")
        qw, pw = ctx.integrate(P, _sid(capi, name), wl.q0, p0, n, f_pos=True)
        ctx.set_kernel("auto")
        idx = np.arange(min(n_chains, 13))
        qs, ps = ctx.integrate(P, _sid(capi, name), wl.q0[idx], p0[idx], n, f_pos=True)
    finally:
        ctx.close()
    np.testing.assert_array_equal(qs, q[idx])      # batch invariance (ragged wave)
    np.testing.assert_array_equal(ps, p[idx])
    err_q = np.abs(q - qw) / (np.abs(qw) + 1)
    err_p = np.abs(p - pw) / (np.abs(pw) + 1)
    assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (err_q.max(), err_p.max())
    par = dict(params)
    par["rows"], par["cols"] = wl.D.shape
    m = R.RefModel(wl.D, par)
    for c in sorted({0, 1, n_chains - 1}):
        qo, po = _oracle_run(m, name, wl.q0[c], p0[c], n)
        err_q = np.abs(q[c] - qo) / (np.abs(qo) + 1)
        err_p = np.abs(p[c] - po) / (np.abs(po) + 1)
        assert err_q.max() <= 1e-9 and err_p.max() <= 1e-8, (name, K, c, err_q.max(),
                                                             err_p.max())
