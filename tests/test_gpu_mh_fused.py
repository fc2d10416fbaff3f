"""The fused one-star MH loop (mh_k1_tiledr, rhmc_mhk1.hpp: every iteration of
run_RHMC's move-0 branch, sampler_RHMC.py:1018-1083, in one launch) against
the four-kernel loop (RHMC_OPT_MH_FUSED = 0: mh_begin / leapfrog / energy / mh_end)
and the CPU oracle, at the bench's C2 geometry and on a 32-px image:

* host randoms (the exact-parity mode): identical accept sequences, chains to
  1e-12, E / V / T records to 1e-11 relative (V is the same sum in another
  order: image background + window correction);
* device Philox randoms: identical accept sequences and final states;
* a ragged chain count (13: the last wave half full) equals the full batch's
  first chains;
* oracle: the first chains' MH chains from RefModel (V, T, trajectory) with
  the same randoms.
The reference goldens (tests/golden/mh.npz, 32x32, K = 1) go through this
kernel in test_gpu_sampler.py::test_run_RHMC_batched_one_chain_equals_reference.
"""
import numpy as np
import pytest

from oracle import rhmc_ref as R
from rhmc_amd import workloads

pytestmark = pytest.mark.gpu

N_ITER, N_STEPS = 8, 25


def _run(ctx, P, q0, z, u, monkeypatch, fused, seed=0):
    ctx.set_option(ctx_opt(), int(bool(fused)))
    try:
        return ctx.mh(P, q0, N_ITER, N_STEPS, f_pos=True, z=z, u=u, seed=seed)
    finally:
        ctx.set_option(ctx_opt(), 1)


def ctx_opt():
    from rhmc_amd import capi
    return capi.OPT_MH_FUSED


@pytest.fixture(scope="module")
def c2(gpu_lib):
    wl = workloads.make("C2")
    ctx = gpu_lib.Context(wl.D)
    rng = np.random.RandomState(17)
    z = rng.randn(N_ITER, wl.q0.shape[0], 3)
    u = rng.uniform(size=(N_ITER, wl.q0.shape[0]))
    yield gpu_lib, wl, ctx, z, u
    ctx.close()


def _close(a, b, rel, what):
    err = np.abs(a - b) / (np.abs(b) + 1)
    assert err.max() <= rel, (what, err.max())


def test_fused_vs_unfused_host_randoms(c2, monkeypatch):
    capi, wl, ctx, z, u = c2
    P = capi.make_params(**wl.params)
    fu = _run(ctx, P, wl.q0, z, u, monkeypatch, True)
    un = _run(ctx, P, wl.q0, z, u, monkeypatch, False)
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    assert 0.2 < fu["accept"].mean() < 1.0
    _close(fu["q"], un["q"], 1e-12, "q")
    _close(fu["q_chain"], un["q_chain"], 1e-12, "q_chain")
    for k in ("E_chain", "V_chain", "T_chain"):
        np.testing.assert_allclose(fu[k], un[k], rtol=1e-11, err_msg=k)


def test_fused_vs_unfused_device_rng(c2, monkeypatch):
    capi, wl, ctx, z, u = c2
    P = capi.make_params(**wl.params)
    fu = _run(ctx, P, wl.q0, None, None, monkeypatch, True, seed=99)
    un = _run(ctx, P, wl.q0, None, None, monkeypatch, False, seed=99)
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    _close(fu["q"], un["q"], 1e-12, "q")


def test_fused_ragged_batch(c2, monkeypatch):
    capi, wl, ctx, z, u = c2
    P = capi.make_params(**wl.params)
    full = _run(ctx, P, wl.q0, z, u, monkeypatch, True)
    part = _run(ctx, P, wl.q0[:13], z[:, :13], u[:, :13], monkeypatch, True)
    np.testing.assert_array_equal(part["accept"], full["accept"][:, :13])
    np.testing.assert_array_equal(part["q"], full["q"][:13])
    np.testing.assert_array_equal(part["E_chain"], full["E_chain"][:, :13])


def _oracle_mh(m, q0, z, u, n_steps, f_lim):
    """run_RHMC's move-0 iteration (sampler_RHMC.py:1018-1083) with given randoms."""
    q = q0.copy()
    acc, E = [], []
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
        E.append(E0)
        if a:
            q, V0 = qn, V1
    return q, np.array(acc), np.array(E)


def test_fused_vs_oracle(c2, monkeypatch):
    capi, wl, ctx, z, u = c2
    P = capi.make_params(**wl.params)
    fu = _run(ctx, P, wl.q0, z, u, monkeypatch, True)
    par = dict(wl.params, fmin=1.0, fmax=1e5)   # the reference's V needs them (:320-321);
    par["rows"], par["cols"] = wl.D.shape       # C2 adds no prior
    m = R.RefModel(wl.D, par)
    for c in (0, 2049):
        qo, ao, Eo = _oracle_mh(m, wl.q0[c], z[:, c], u[:, c], N_STEPS, par["f_lim"])
        np.testing.assert_array_equal(fu["accept"][:, c].astype(bool), ao)
        _close(fu["q"][c], qo, 1e-9, "q chain %d" % c)
        np.testing.assert_allclose(fu["E_chain"][:, c], Eo, rtol=1e-11)


def test_fused_32px_image(gpu_lib, monkeypatch):
    capi = gpu_lib
    wl = workloads.make("C1", n_chains=64)
    rng = np.random.RandomState(3)
    q0 = wl.q0 + np.c_[np.zeros(64), 0.4 * rng.randn(64, 2)]
    z = rng.randn(N_ITER, 64, 3)
    u = rng.uniform(size=(N_ITER, 64))
    ctx = capi.Context(wl.D)
    try:
        P = capi.make_params(**wl.params)
        fu = _run(ctx, P, q0, z, u, monkeypatch, True)
        un = _run(ctx, P, q0, z, u, monkeypatch, False)
    finally:
        ctx.close()
    np.testing.assert_array_equal(fu["accept"], un["accept"])
    _close(fu["q"], un["q"], 1e-12, "q")
    np.testing.assert_allclose(fu["V_chain"], un["V_chain"], rtol=1e-11)
