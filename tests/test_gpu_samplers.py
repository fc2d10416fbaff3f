"""GPU parity of the older `samplers` API path: lightsource_gym.HMC_random
(samplers.py:460-572) — unit-mass HMC with a per-coordinate dt vector, random
trajectory lengths and the flux wall with the reference's quirks (the flip
mask is never cleared inside a trajectory; when the last step flipped, the
trajectory is scored with the momentum it started from).

Tolerances (fp64): trajectories to 1e-10 relative to |value| + 1 (<= 20
leapfrog steps of the same explicit integrator); energies rtol 1e-11; the
accept/reject sequence and the stale-momentum flags exactly.
"""
import numpy as np
import pytest

from conftest import load_golden
from test_oracle_goldens import hmc_random_model

pytestmark = pytest.mark.gpu


def _gym(z, name):
    from rhmc_amd.samplers import lightsource_gym
    g = lightsource_gym()
    g.num_rows = g.num_cols = z[name + "/D"].shape[0]
    g.D = z[name + "/D"]
    K = z[name + "/q0"].size // 3
    g.Nobjs, g.d, g.dt = K, 3 * K, z[name + "/dt"]
    assert g.B_count == float(z[name + "/B_count"])
    assert g.PSF_FWHM_pix == float(z[name + "/fwhm_pix"])
    return g


@pytest.mark.parametrize("name", ["k1", "k2", "wall", "wall2"])
def test_HMC_random_reproduces_reference_chain(gpu_lib, name):
    z = load_golden("hmc_random")
    g = _gym(z, name)
    np.random.seed(int(z[name + "/seed"]))
    g.HMC_random(q_model_0=z[name + "/q0"].reshape(-1, 3), Niter=int(z[name + "/Niter"]),
                 steps_min=int(z[name + "/steps_min"]), steps_max=int(z[name + "/steps_max"]),
                 f_lim=float(z[name + "/f_lim"]))
    np.testing.assert_array_equal(g.A_chain[0], z[name + "/A_chain"])
    want = z[name + "/q_chain"]
    err = np.abs(g.q_chain[0] - want) / (np.abs(want) + 1)
    assert err.max() <= 1e-10, err.max()
    E, Ew = g.E_chain[0], z[name + "/E_chain"]
    assert np.array_equal(np.isinf(E), np.isinf(Ew))
    fin = np.isfinite(Ew)
    np.testing.assert_allclose(E[fin], Ew[fin], rtol=1e-11)


@pytest.mark.parametrize("name", ["k1", "wall", "wall2"])
def test_hmc_random_trajectories_vs_oracle(gpu_lib, name):
    """rhmc_hmc_random on many chains (random starts, momenta, lengths; the
    wall cases hit the flux wall) against the oracle trajectory, chain by
    chain, including which chains end on a flip (stale momentum)."""
    capi = gpu_lib
    z = load_golden("hmc_random")
    g = _gym(z, name)
    g.f_lim = float(z[name + "/f_lim"])
    m = hmc_random_model(z, name)
    rs = np.random.RandomState(11)
    n = 24
    q0 = np.tile(z[name + "/q0"], (n, 1))
    q0[:, 0::3] *= np.exp(0.15 * rs.randn(n, g.Nobjs))
    q0[:, 1::3] += 0.3 * rs.randn(n, g.Nobjs)
    q0[:, 2::3] += 0.3 * rs.randn(n, g.Nobjs)
    p0 = rs.randn(n, g.d)
    steps = rs.randint(1, 25, size=n).astype(np.int32)
    q, p, st = g._context().hmc_random(g._params(), g.dt, q0, p0, steps, return_status=True)
    stale = 0
    for c in range(n):
        qo, po, flip = m.hmc_random_traj(q0[c], p0[c], g.dt, int(steps[c]), g.f_lim)
        assert bool(st[c] & capi.STATUS_REFLECT_F) == flip, c
        stale += flip
        assert np.abs(q[c] - qo).max() / (np.abs(qo).max() + 1) <= 1e-10, c
        assert np.abs(p[c] - po).max() / (np.abs(po).max() + 1) <= 1e-10, c
    if name.startswith("wall"):
        assert stale > 0


def test_HMC_random_batched(gpu_lib):
    """Many chains at once: one chain reproduces HMC_random's draws exactly;
    several chains equal the oracle run on the batched draw order."""
    z = load_golden("hmc_random")
    name = "wall2"
    g = _gym(z, name)
    kw = dict(Niter=12, steps_min=int(z[name + "/steps_min"]),
              steps_max=int(z[name + "/steps_max"]), f_lim=float(z[name + "/f_lim"]))
    np.random.seed(int(z[name + "/seed"]))
    g.HMC_random_batched(z[name + "/q0"][None], **kw)
    np.testing.assert_array_equal(g.A_chain[0, :12], z[name + "/A_chain"][:12])
    assert np.abs(g.q_chain[0] - z[name + "/q_chain"][:13]).max() <= 1e-10 * 2e3

    n = 3
    q0 = np.tile(z[name + "/q0"], (n, 1))
    q0[:, 1::3] += np.array([[0.], [0.2], [-0.3]])
    np.random.seed(4)
    g.HMC_random_batched(q0, **kw)
    m = hmc_random_model(z, name)
    rs = np.random.RandomState(4)
    d = g.d
    p_init = rs.randn(n, d)
    qt = q0.copy()
    for i in range(1, 13):
        p = rs.randn(n, d)
        steps = rs.randint(kw["steps_min"], kw["steps_max"], size=n)
        lnu = np.log(rs.random_sample(n))
        for c in range(n):
            Ei = m.ls_E(qt[c], p[c], kw["f_lim"])
            qn, pn, _ = m.hmc_random_traj(qt[c], p[c], g.dt, int(steps[c]), kw["f_lim"])
            dE = m.ls_E(qn, pn, kw["f_lim"]) - Ei
            acc = (dE < 0) or (lnu[c] < -dE)
            assert g.A_chain[c, i - 1, 0] == acc, (c, i)
            if acc:
                qt[c] = qn
            assert np.abs(g.q_chain[c, i] - qt[c]).max() / (np.abs(qt[c]).max() + 1) <= 1e-10
    assert p_init.shape == (n, d)


@pytest.mark.parametrize("side,wall", [(48, False), (48, True), (32, True), (64, False)])
def test_hmc_random_register_window_vs_oracle_and_windowed(gpu_lib, side, wall, monkeypatch):
    """One star on a 32/48/64-px image takes the register-window kernel
    (hmc_random_k1_tiledr): trajectories against the oracle and the windowed
    kernel (kernel option "windowed") to 1e-10, identical stale-momentum flags,
    ragged batch (the last wave partly empty, lengths differing inside a wave)."""
    from oracle import rhmc_ref as R
    capi = gpu_lib
    setup = R.default_setup()
    rs = np.random.RandomState(side + wall)
    c = side / 2.0
    f_true = R.mag2flux(19.) * setup["flux_to_count"]
    D = rs.poisson(R.model_image(side, side, [(f_true, c + 0.2, c - 0.3)],
                                 setup["B_count"], setup["fwhm_pix"])).astype(np.float64)
    f_lim = 0.97 * f_true if wall else setup["B_count"]
    par = dict(rows=side, cols=side, B_count=setup["B_count"], fwhm_pix=setup["fwhm_pix"],
               use_prior=0, use_Vc=0, alpha=2., beta=1., Vc_r_pow=1., dt=1., f_lim=f_lim,
               f_low=1., g_xx=1., g_ff=1., g_ff2=1., g0=1., g1=1., g2=1., fmin=-1., fmax=-1.)
    m = R.RefModel(D, par)
    P = capi.make_params(dt=1., delta=1e-6, counter_max=1000, B_count=par["B_count"],
                         f_lim=f_lim, f_low=1., fwhm_pix=par["fwhm_pix"], g_xx=1., g_ff=1.,
                         g_ff2=1., g0=1., g1=1., g2=1., use_prior=False, alpha=2.,
                         use_Vc=False, beta=1., Vc_r_pow=1., V_prior_const=0.)
    n = 203
    q0 = np.stack([f_true * np.exp(0.1 * rs.randn(n)), c + 0.5 * rs.randn(n),
                   c + 0.5 * rs.randn(n)], 1)
    p0 = rs.randn(n, 3)
    dt = np.array([2.0, 0.02, 0.02])
    steps = rs.randint(1, 30, size=n).astype(np.int32)
    ctx = capi.Context(D)
    try:
        q, p, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        ctx.set_kernel("windowed")
        qw, pw, stw = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        ctx.set_kernel("auto")
        qs, ps = ctx.hmc_random(P, dt, q0[5:18], p0[5:18], steps[5:18])
    finally:
        ctx.close()
    np.testing.assert_array_equal(qs, q[5:18])
    np.testing.assert_array_equal(ps, p[5:18])
    np.testing.assert_array_equal(st & capi.STATUS_REFLECT_F, stw & capi.STATUS_REFLECT_F)
    for a, b in ((q, qw), (p, pw)):
        assert (np.abs(a - b) / (np.abs(b) + 1)).max() <= 1e-10
    stale = 0
    for k in range(0, n, 10):
        qo, po, flip = m.hmc_random_traj(q0[k], p0[k], dt, int(steps[k]), f_lim)
        assert bool(st[k] & capi.STATUS_REFLECT_F) == flip, k
        stale += flip
        assert np.abs(q[k] - qo).max() / (np.abs(qo).max() + 1) <= 1e-10, k
        assert np.abs(p[k] - po).max() / (np.abs(po).max() + 1) <= 1e-10, k
    if wall:
        assert (st & capi.STATUS_REFLECT_F).any()


@pytest.mark.parametrize("side,K,n", [(48, 10, 517), (32, 4, 129), (48, 20, 37), (64, 40, 9)])
def test_hmc_random_many_stars_vs_oracle_and_windowed(gpu_lib, side, K, n, monkeypatch):
    """K >= 2 takes the multi-star register-window kernel (leapfrog_kr with
    kSolverHmcRandom): trajectories against the windowed kernel and the oracle
    to 1e-10, the flux wall hit by the faint stars (any star below flips every
    star whose flag is set), identical stale-momentum flags, ragged batches."""
    from oracle import rhmc_ref as R
    from test_gpu_integrators import _star_field
    capi = gpu_lib
    wl = _star_field(side, K, n, 5 + K)
    rs = np.random.RandomState(K)
    fl = np.sort(wl.q0[0, 0::3])
    f_lim = 0.9 * fl[2]                              # the faintest stars reach it
    par = dict(rows=side, cols=side, B_count=wl.params["B_count"],
               fwhm_pix=wl.params["fwhm_pix"], use_prior=0, use_Vc=0, alpha=2., beta=1.,
               Vc_r_pow=1., dt=1., f_lim=f_lim, f_low=1., g_xx=1., g_ff=1., g_ff2=1., g0=1.,
               g1=1., g2=1., fmin=-1., fmax=-1.)
    m = R.RefModel(wl.D, par)
    P = capi.make_params(dt=1., delta=1e-6, counter_max=1000, B_count=par["B_count"],
                         f_lim=f_lim, f_low=1., fwhm_pix=par["fwhm_pix"], g_xx=1., g_ff=1.,
                         g_ff2=1., g0=1., g1=1., g2=1., use_prior=False, alpha=2.,
                         use_Vc=False, beta=1., Vc_r_pow=1., V_prior_const=0.)
    q0 = wl.q0
    p0 = rs.randn(*q0.shape)
    dt = np.tile([1.0, 0.005, 0.005], K)
    steps = rs.randint(1, 20, size=n).astype(np.int32)
    ctx = capi.Context(wl.D)
    try:
        q, p, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        ctx.set_kernel("windowed")
        qw, pw, stw = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
        ctx.set_kernel("auto")
        idx = np.arange(min(n, 7))
        qs, ps = ctx.hmc_random(P, dt, q0[idx], p0[idx], steps[idx])
    finally:
        ctx.close()
    np.testing.assert_array_equal(qs, q[idx])
    np.testing.assert_array_equal(ps, p[idx])
    np.testing.assert_array_equal(st & capi.STATUS_REFLECT_F, stw & capi.STATUS_REFLECT_F)
    for a, b in ((q, qw), (p, pw)):
        assert (np.abs(a - b) / (np.abs(b) + 1)).max() <= 1e-10
    for k in sorted({0, 1, n // 2, n - 1}):
        qo, po, flip = m.hmc_random_traj(q0[k], p0[k], dt, int(steps[k]), f_lim)
        assert bool(st[k] & capi.STATUS_REFLECT_F) == flip, k
        assert np.abs(q[k] - qo).max() / (np.abs(qo).max() + 1) <= 1e-10, k
        assert np.abs(p[k] - po).max() / (np.abs(po).max() + 1) <= 1e-10, k
