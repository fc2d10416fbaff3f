"""The fused multi-star MH iteration (mh_pk_iter, rhmc_mhpk.hpp: one launch
per iteration of run_RHMC's move-0 branch, sampler_RHMC.py:1018-1083, on the
pixel-major kernel, 2 <= K <= 10) against the four-kernel loop
(RHMC_OPT_MH_FUSED = 0: mh_begin / leapfrog / energy / mh_end) and the CPU
oracle, at the bench's C3 geometry (48x48, K = 10, big-sim4 parameters) and
on a 32-px K = 4 image:

* host randoms: identical accept sequences, chains and final states to
  1e-12, E / V / T records to 1e-11 relative (V is the same image sum in
  another order and with log_pos, within 2 ulp of log);
* device Philox randoms: identical accept sequences and final states;
* a ragged chain count equals the full batch's first chains bit for bit;
* oracle: two chains' MH chains from RefModel with the same randoms.
The reference goldens (tests/golden/mh.npz "mh3": 32x32, K = 3) go through
this kernel in test_gpu_sampler.py::test_run_RHMC_batched_one_chain_equals_reference.
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu

N_ITER, N_STEPS = 6, 20


def _run(capi, ctx, P, q0, z, u, fused, seed=0):
    ctx.set_option(capi.OPT_MH_FUSED, int(bool(fused)))
    try:
        return ctx.mh(P, q0, N_ITER, N_STEPS, f_pos=True, z=z, u=u, seed=seed)
    finally:
        ctx.set_option(capi.OPT_MH_FUSED, 1)


def _close(a, b, rel, what):
    err = np.abs(a - b) / (np.abs(b) + 1)
    assert err.max() <= rel, (what, err.max())


@pytest.fixture(scope="module")
def c3(gpu_lib):
    wl = workloads.make("C3", n_chains=1001)
    # C3's power-law fluxes reach below the wall (f_lim): V(q0) = inf there and
    # every proposal would be rejected; start the MH chains above it
    wl.q0[:, 0::3] = np.maximum(wl.q0[:, 0::3], 1.5 * wl.params["f_lim"])
    ctx = gpu_lib.Context(wl.D)
    rng = np.random.RandomState(19)
    z = rng.randn(N_ITER, wl.n_chains, 3 * wl.K)
    u = rng.uniform(size=(N_ITER, wl.n_chains))
    yield gpu_lib, wl, ctx, z, u
    ctx.close()


def test_fused_vs_unfused_host_randoms(c3):
    capi, wl, ctx, z, u = c3
    P = capi.make_params(**wl.params)
    fu = _run(capi, ctx, P, wl.q0, z, u, True)
    un = _run(capi, ctx, P, wl.q0, z, u, False)
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    assert 0.05 < fu["accept"].mean() < 1.0
    _close(fu["q"], un["q"], 1e-12, "q")
    _close(fu["q_chain"], un["q_chain"], 1e-12, "q_chain")
    for k in ("E_chain", "V_chain", "T_chain"):
        np.testing.assert_allclose(fu[k], un[k], rtol=1e-11, err_msg=k)


def test_fused_vs_unfused_device_rng(c3):
    capi, wl, ctx, z, u = c3
    P = capi.make_params(**wl.params)
    fu = _run(capi, ctx, P, wl.q0, None, None, True, seed=5)
    un = _run(capi, ctx, P, wl.q0, None, None, False, seed=5)
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    _close(fu["q"], un["q"], 1e-12, "q")


def test_fused_ragged_batch(c3):
    capi, wl, ctx, z, u = c3
    P = capi.make_params(**wl.params)
    full = _run(capi, ctx, P, wl.q0, z, u, True)
    part = _run(capi, ctx, P, wl.q0[:7], z[:, :7], u[:, :7], True)
    np.testing.assert_array_equal(part["accept"], full["accept"][:, :7])
    np.testing.assert_array_equal(part["q"], full["q"][:7])
    np.testing.assert_array_equal(part["E_chain"], full["E_chain"][:, :7])


def _oracle_mh(m, q0, z, u, n_steps):
    """run_RHMC's move-0 iteration (sampler_RHMC.py:1018-1083) with given randoms."""
    q = q0.copy()
    acc = []
    V0 = m.V(q, f_pos=True)
    for it in range(z.shape[0]):
        H = m.H(q)
        p = z[it] * np.sqrt(H)
        E0 = V0 + m.T(p, H)
        qn, pn, _, _ = m.trajectory(q, p, n_steps, record=False)
        V1 = m.V(qn, f_pos=True)
        dE = V1 + m.T(pn, m.H(qn)) - E0
        a = bool(dE < 0 or np.log(u[it]) < -dE)
        acc.append(a)
        if a:
            q, V0 = qn, V1
    return q, np.array(acc)


def test_fused_vs_oracle(c3):
    capi, wl, ctx, z, u = c3
    P = capi.make_params(**wl.params)
    fu = _run(capi, ctx, P, wl.q0, z, u, True)
    par = dict(wl.params, fmin=1.0, fmax=1e7)   # the reference's V needs them (:320-321)
    par["rows"], par["cols"] = wl.D.shape
    m = R.RefModel(wl.D, par)
    for c in (0, 500):
        qo, ao = _oracle_mh(m, wl.q0[c], z[:, c], u[:, c], N_STEPS)
        np.testing.assert_array_equal(fu["accept"][:, c].astype(bool), ao)
        _close(fu["q"][c], qo, 1e-9, "q chain %d" % c)


def test_fused_32px_four_stars_with_prior(gpu_lib):
    capi = gpu_lib
    from rhmc_amd.photometry import mag2flux
    par, ftc = workloads.base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4., use_prior=True)
    a_, fmin, fmax = 2.0, mag2flux(23.3) * ftc, mag2flux(15.) * ftc
    par["V_prior_const"] = np.log(32 * 32) - np.log((1 - a_) / (fmax ** (1 - a_) - fmin ** (1 - a_)))
    rng = np.random.RandomState(11)
    stars = [(17.5, 8.2, 20.1), (18.3, 22.7, 9.4), (19.0, 15.0, 15.5), (20.2, 25.1, 26.3)]
    D = workloads._image(32, stars, ftc, par["B_count"], par["fwhm_pix"], rng)
    n, K = 77, 4
    q0 = np.empty((n, 3 * K))
    q0[:, 0::3] = [mag2flux(s[0]) * ftc for s in stars]
    q0[:, 1::3] = [s[1] for s in stars]
    q0[:, 2::3] = [s[2] for s in stars]
    q0 *= 1 + 0.01 * rng.randn(n, 3 * K)
    z = rng.randn(N_ITER, n, 3 * K)
    u = rng.uniform(size=(N_ITER, n))
    ctx = capi.Context(D)
    try:
        P = capi.make_params(**par)
        fu = _run(capi, ctx, P, q0, z, u, True)
        un = _run(capi, ctx, P, q0, z, u, False)
    finally:
        ctx.close()
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    _close(fu["q"], un["q"], 1e-12, "q")
    for k in ("E_chain", "V_chain", "T_chain"):
        np.testing.assert_allclose(fu[k], un[k], rtol=1e-11, err_msg=k)
