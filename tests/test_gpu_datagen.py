"""GPU tests of device data generation (rhmc_gen_image).

* gen_model (sampler_RHMC.py:101-116): the device model image against the
  reference's own gen_model outputs (goldens) and the oracle's model_image at
  C5 size.  Tolerance 1e-13 relative: the device exp may differ from NumPy's
  by an ulp per PSF value; the expression order is the reference's.
* gen_mock_data / gen_noise_profile Poisson draws: the device stream is
  Philox, not NumPy's, so parity is distributional — mean, variance and a
  G-test of the empirical pmf against the exact Poisson pmf, on both sides of
  the sampler switch (lam < 10: multiplication method; lam >= 10: PTRS).
* stream layout, determinism, install-into-context and the error paths.
"""
import numpy as np
import pytest
from scipy import stats

from conftest import load_golden
from helpers import capi_params
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu


def _flat_params(capi, B, fwhm=3.5):
    return capi.make_params(dt=0.1, delta=1e-6, counter_max=1, B_count=B, f_lim=0., f_low=0.,
                            fwhm_pix=fwhm, g_xx=1., g_ff=1., g_ff2=1., g0=1., g1=1., g2=1.)


@pytest.mark.parametrize("name", ["k1_48", "k1_32", "k2_16", "k10_48"])
def test_model_image_matches_reference(gpu_lib, name):
    z = load_golden("datagen")
    par = R.params_from_npz(z, name + "/par_")
    ctx = gpu_lib.Context(None)
    P = capi_params(gpu_lib, par)
    got = ctx.gen_image(P, z[name + "/q"], int(par["rows"]), int(par["cols"]))
    np.testing.assert_allclose(got, z[name + "/model"], rtol=1e-13, atol=0)


def test_model_image_c5_size_vs_oracle(gpu_lib):
    from rhmc_amd import workloads
    w = workloads.make("C5", n_chains=1)
    p = w.params
    stars = w.q0[0].reshape(-1, 3)
    want = R.model_image(256, 256, stars, p["B_count"], p["fwhm_pix"])
    ctx = gpu_lib.Context(None)
    got = ctx.gen_image(gpu_lib.make_params(**p), stars, 256, 256)
    np.testing.assert_allclose(got, want, rtol=1e-13, atol=0)
    empty = ctx.gen_image(gpu_lib.make_params(**p), np.zeros((0, 3)), 8, 8)
    np.testing.assert_array_equal(empty, np.full((8, 8), p["B_count"]))


@pytest.mark.parametrize("lam", [0.37, 3.7, 9.99, 10.0, 57.3, 2500.0])
def test_poisson_distribution(gpu_lib, lam):
    ctx = gpu_lib.Context(None)
    n_real, side = 16, 128
    x = ctx.gen_image(_flat_params(gpu_lib, lam), np.zeros((0, 3)), side, side,
                      n_real=n_real, seed=1234).ravel()
    n = x.size
    assert np.all(x == np.floor(x)) and x.min() >= 0
    assert abs(x.mean() - lam) < 5 * np.sqrt(lam / n)
    sd_var = np.sqrt((lam + 2 * lam * lam) / n)
    assert abs(x.var() - lam) < 6 * sd_var
    # G-test over the pmf bins with >= 20 expected counts (+ both tails)
    lo, hi = stats.poisson.ppf(1e-4, lam), stats.poisson.ppf(1 - 1e-4, lam)
    ks = np.arange(lo, hi + 1)
    expct = stats.poisson.pmf(ks, lam) * n
    keep = expct >= 20
    ks, expct = ks[keep], expct[keep]
    obs = np.array([(x == k).sum() for k in ks], float)
    rest_e = n - expct.sum()
    rest_o = n - obs.sum()
    obs = np.append(obs, rest_o)
    expct = np.append(expct, rest_e)
    g, pval = stats.power_divergence(obs, expct, lambda_="log-likelihood")
    assert pval > 1e-6, (lam, g, pval)


def test_poisson_zero_and_huge(gpu_lib):
    ctx = gpu_lib.Context(None)
    z0 = ctx.gen_image(_flat_params(gpu_lib, 0.0), np.zeros((0, 3)), 32, 32, n_real=2, seed=1)
    np.testing.assert_array_equal(z0, 0.0)
    lam = 1e7
    x = ctx.gen_image(_flat_params(gpu_lib, lam), np.zeros((0, 3)), 64, 64, n_real=4,
                      seed=2).ravel()
    assert abs(x.mean() - lam) < 5 * np.sqrt(lam / x.size)
    assert abs(x.std() / np.sqrt(lam) - 1) < 0.05


def test_stream_layout_and_determinism(gpu_lib):
    z = load_golden("datagen")
    par = R.params_from_npz(z, "k10_48/par_")
    P = capi_params(gpu_lib, par)
    q = z["k10_48/q"]
    ctx = gpu_lib.Context(None)
    a = ctx.gen_image(P, q, 48, 48, n_real=3, seed=99)
    b = ctx.gen_image(P, q, 48, 48, n_real=3, seed=99)
    np.testing.assert_array_equal(a, b)
    one = ctx.gen_image(P, q, 48, 48, n_real=1, seed=99)
    np.testing.assert_array_equal(one[0], a[0])   # realisation r uses pixels r*npix + pix
    c = ctx.gen_image(P, q, 48, 48, n_real=3, seed=100)
    assert (c != a).mean() > 0.5
    assert (a[1] != a[0]).mean() > 0.5
    # residuals of independent realisations: uncorrelated between pixels
    m = ctx.gen_image(P, q, 48, 48)
    big = ctx.gen_image(P, q, 48, 48, n_real=400, seed=5) - m
    r = (big / np.sqrt(m)).reshape(400, -1)
    assert abs(np.corrcoef(r[:, :-1].ravel(), r[:, 1:].ravel())[0, 1]) < 0.01
    assert abs(np.corrcoef(r[:-1].ravel(), r[1:].ravel())[0, 1]) < 0.01
    # per-pixel mean over realisations tracks the model
    zscore = (big.mean(0)) / np.sqrt(m / 400)
    assert abs(zscore.mean()) < 5 / 48 and 0.85 < zscore.std() < 1.15


def test_install_into_context(gpu_lib):
    z = load_golden("functions")
    par = R.params_from_npz(z, "k1/par_")
    P = capi_params(gpu_lib, par)
    q = np.array([[par["B_count"] * 30, 24.3, 23.8]])
    ctx = gpu_lib.Context(None)
    with pytest.raises(gpu_lib.RhmcError):
        ctx.gradient(P, q.ravel())                # no image yet
    D = ctx.gen_image(P, q, 48, 48, n_real=1, seed=7, install=True)[0]
    ref = gpu_lib.Context(D)
    qs = z["k1/q"]
    np.testing.assert_array_equal(ctx.gradient(P, qs), ref.gradient(P, qs))
    V1, _ = ctx.energy(P, qs)
    V2, _ = ref.energy(P, qs)
    np.testing.assert_array_equal(V1, V2)
    m = R.RefModel(D, par)
    np.testing.assert_allclose(ctx.gradient(P, qs[0]), m.dVdq(qs[0]), rtol=1e-11, atol=1e-9)


def test_sampler_device_datagen(gpu_lib):
    from rhmc_amd import sampler
    z = load_golden("datagen")
    stars = z["k10_48/stars"]
    g = sampler.multi_gym(g_xx=1., g_ff=1., g_ff2=1.)
    np.testing.assert_allclose(g.gen_model(stars, device=True), z["k10_48/model"], rtol=1e-13)
    g.gen_mock_data(stars, rng="device", seed=3)
    D = g.D.copy()
    again = g.gen_mock_data(stars, return_data=True, rng="device", seed=3)
    np.testing.assert_array_equal(again, D)
    q = g.format_q(stars.copy())
    m = R.RefModel(D, R.params_from_npz(z, "k10_48/par_"))
    np.testing.assert_allclose(g.dVdq(q), m.dVdq(q), rtol=1e-10, atol=1e-8)
    g.gen_noise_profile(stars, N_trial=200, rng="device", seed=4)
    width = g.centers_noise[1] - g.centers_noise[0]
    mass = g.hist_noise.sum() * width
    assert 0.9 < mass <= 1.0 + 1e-12
    mean = (g.hist_noise * g.centers_noise).sum() * width
    assert abs(mean) < 0.1 * np.sqrt(g.B_count)


def test_gen_image_errors(gpu_lib):
    ctx = gpu_lib.Context(None)
    P = _flat_params(gpu_lib, 10.)
    lib = gpu_lib.lib()
    import ctypes
    assert lib.rhmc_gen_image(ctx.handle, ctypes.byref(P), None, 0, 8, 8, 0, 0, None, 0) != 0
    with pytest.raises(gpu_lib.RhmcError):
        ctx.gen_image(P, np.zeros((0, 3)), 8, 9, install=True)
    with pytest.raises(gpu_lib.RhmcError):
        ctx.gen_image(P, np.zeros((0, 3)), 0, 8)
    assert lib.rhmc_gen_image(ctx.handle, ctypes.byref(P), None, 0, 8, 8, -1, 0,
                              (ctypes.c_double * 64)(), 0) != 0
