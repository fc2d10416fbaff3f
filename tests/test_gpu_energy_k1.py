"""The one-star register-window energy kernel (energy_k1_tiledr, rhmc_mhk1.hpp:
V = image background + window correction, 16 lanes per chain) against the
full-image per-wave energy kernels (the "generic" / "windowed" kernel options select them)
and the CPU oracle (RefModel.V / T, sampler_RHMC.py:294-363):

* V and T to 1e-12 relative on a C2-sized batch, with chains inside the
  image, on the flux wall, past the position support (+-1 px around the
  image) and with the prior on;
* the support flags: f_pos (flux wall -> inf) and pos_check=False
  (samplers.lightsource_gym.V has no position check);
* 32- and 64-px images; a ragged batch is bit-identical to the full one's rows.
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu


def _batch(wl, n, side, rng):
    c = side / 2.0
    q = np.empty((n, 3))
    q[:, 0] = wl.q0[:n, 0] * np.exp(0.3 * rng.randn(n))
    q[:, 1] = c + 3.0 * rng.randn(n)
    q[:, 2] = c + 3.0 * rng.randn(n)
    q[0] = (wl.params["f_lim"] * 0.5, c, c)          # below the flux wall
    q[1] = (q[1, 0], -1.5, c)                        # past the support (x < -1)
    q[2] = (q[2, 0], c, side + 0.5)                  # inside (y <= cols + 1)
    q[3] = (q[3, 0], 0.2, side - 1.3)                # window clamped at two edges
    p = rng.randn(n, 3) * 5.0
    return q, p


def _energies(ctx, P, q, p, monkeypatch, new, **kw):
    ctx.set_kernel("auto" if new else "windowed")
    try:
        return ctx.energy(P, q, p, **kw)
    finally:
        ctx.set_kernel("auto")


def _close(a, b, rtol):
    assert np.array_equal(np.isinf(a), np.isinf(b))
    fin = np.isfinite(b)
    np.testing.assert_allclose(a[fin], b[fin], rtol=rtol)


@pytest.mark.parametrize("side", [48, 32, 64])
@pytest.mark.parametrize("prior", [False, True])
def test_energy_k1_vs_full_image_and_oracle(gpu_lib, side, prior, monkeypatch):
    capi = gpu_lib
    rng = np.random.RandomState(side + prior)
    if side == 48:
        wl = workloads.make("C2")
        D = wl.D
    else:
        wl = workloads.make("C2", n_chains=4096)
        setup = R.default_setup()
        c = side / 2.0
        D = R.model_image(side, side, [(R.mag2flux(19.) * setup["flux_to_count"], c + 0.2,
                                        c - 0.3)], setup["B_count"], setup["fwhm_pix"])
        D = rng.poisson(D).astype(np.float64)
    params = dict(wl.params, use_prior=prior, alpha=2.0, V_prior_const=1.25 if prior else 0.0)
    q, p = _batch(wl, 4096, side, rng)
    ctx = capi.Context(D)
    try:
        P = capi.make_params(**params)
        V, T = _energies(ctx, P, q, p, monkeypatch, True, f_pos=True)
        Vo, To = _energies(ctx, P, q, p, monkeypatch, False, f_pos=True)
        Vn, _ = _energies(ctx, P, q, None, monkeypatch, True, f_pos=False, pos_check=False)
        Vno, _ = _energies(ctx, P, q, None, monkeypatch, False, f_pos=False, pos_check=False)
        Vr, Tr = _energies(ctx, P, q[:13], p[:13], monkeypatch, True, f_pos=True)
    finally:
        ctx.close()
    assert np.isinf(V[0]) and np.isinf(V[1]) and np.isfinite(V[2]) and np.isfinite(V[3])
    assert np.isfinite(Vn[0]) and np.isfinite(Vn[1])
    _close(V, Vo, 1e-12)
    _close(Vn, Vno, 1e-12)
    np.testing.assert_allclose(T, To, rtol=1e-12, atol=1e-12)
    np.testing.assert_array_equal(Vr, V[:13])
    np.testing.assert_array_equal(Tr, T[:13])
    par = dict(params, fmin=1.0, fmax=1e5)
    par["rows"], par["cols"] = D.shape
    m = R.RefModel(D, par)
    m.V_prior_const = params["V_prior_const"]
    for c in (0, 1, 2, 3, 77, 4095):
        want = m.V(q[c], f_pos=True)
        if np.isinf(want):
            assert np.isinf(V[c])
        else:
            np.testing.assert_allclose(V[c], want, rtol=1e-12)
        np.testing.assert_allclose(T[c], m.T(p[c], m.H(q[c])), rtol=1e-12)
