"""K > 64 stars per chain through the C-ABI: the reference's own many-star
drivers run K = 100 (RHMC-big-sim3.py:18-19) and grow K by births up to
N_max = 120 (RHMC-big-sim4.py:77); its dVdq / V / RHMC_single_step take any
3 * Nobjs (sampler_RHMC.py:365-425, :294-351, :522-566).  The engine takes
1 <= K <= 1024 (past 256: tests/test_gpu_hugek.py).  Every test runs on the automatic choice (32/48-px images: the
dense many-star kernel, rhmc_dense.hpp; 256 px: the windowed kernel) and
with each family forced.

Pinned by reference fixtures (tests/golden/make_goldens.py case_bigk):
bigk.npz (dVdq, dphidq, V, T at K = 100 on 32x32 with prior and with
repulsion, K = 120 on 48x48, K = 128 on 256x256), traj_bigk.npz (32x32,
K = 100, big-sim4 parameters, 2 chains x 50 steps) and traj_bigk256.npz
(256x256, K = 128, 1 chain x 4 steps).  Every step is checked from the
reference's own state (1e-11 / 1e-10, exact fixed-point iteration counts);
free-running, the dense K = 100 trajectory is chaotic — the reference itself,
started 1e-15 away, leaves 1e-9 agreement after ~35 steps (measured with the
oracle) — so the fused comparison stops at 25 steps.  The integrators,
HMC_random, MH and K = 256 go against the oracle.
"""
import numpy as np
import pytest

from conftest import load_golden
from helpers import assert_state_close, capi_params
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu

BIGK_KERNELS = ["auto", "windowed", "multiwin", "dense"]


@pytest.fixture(params=BIGK_KERNELS)
def bigk_kernel(request, monkeypatch):
    from rhmc_amd import capi
    monkeypatch.setattr(capi, "DEFAULT_KERNEL", request.param)
    return request.param


@pytest.mark.parametrize("name", ["b100", "b100vc", "b120", "b128"])
def test_bigk_gradient_energy(gpu_lib, bigk_kernel, name):
    capi = gpu_lib
    z = load_golden("bigk")
    par = R.params_from_npz(z, name + "/par_")
    ctx = capi.Context(z[name + "/D"])
    P = capi_params(capi, par)
    q, p = z[name + "/q"], z[name + "/p"]
    assert q.shape[1] // 3 > 64
    for kind, key in ((0, "dVdq"), (1, "dphidq")):
        g = ctx.gradient(P, q, kind=kind)
        want = z[name + "/" + key]
        scale = np.abs(want).max(axis=1, keepdims=True) + 1.0
        np.testing.assert_array_less(np.abs(g - want) / scale, 1e-10)
    V, T = ctx.energy(P, q, p, f_pos=False)
    np.testing.assert_allclose(V, z[name + "/V"], rtol=1e-12)
    np.testing.assert_allclose(T, z[name + "/T"], rtol=1e-12, atol=1e-12)
    Vp, _ = ctx.energy(P, q, None, f_pos=True)
    want = z[name + "/Vpos"]
    assert np.array_equal(np.isinf(Vp), np.isinf(want))
    fin = np.isfinite(want)
    np.testing.assert_allclose(Vp[fin], want[fin], rtol=1e-12)
    ctx.close()


@pytest.mark.parametrize("name", ["traj_bigk", "traj_bigk256"])
def test_bigk_trajectory_stepwise(gpu_lib, bigk_kernel, name):
    capi = gpu_lib
    z = load_golden(name)
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par, float(z["delta"]), int(z["counter_max"]))
    Q, Pm = z["Q"], z["P"]
    for s in range(Q.shape[1] - 1):
        q, p, it, st = ctx.leapfrog(P, Q[:, s], Pm[:, s], 1, return_info=True)
        np.testing.assert_array_equal(it[:, 0], z["n_p"][:, s], err_msg="p-iters step %d" % s)
        np.testing.assert_array_equal(it[:, 1], z["n_q"][:, s], err_msg="q-iters step %d" % s)
        assert_state_close(q, Q[:, s + 1], 1e-11, "%s q step %d" % (name, s))
        assert_state_close(p, Pm[:, s + 1], 1e-10, "%s p step %d" % (name, s))
    ctx.close()


@pytest.mark.parametrize("name,horizon", [("traj_bigk", 25), ("traj_bigk256", 4)])
def test_bigk_trajectory_fused(gpu_lib, bigk_kernel, name, horizon):
    capi = gpu_lib
    z = load_golden(name)
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par, float(z["delta"]), int(z["counter_max"]))
    Q, Pm = z["Q"], z["P"]
    q, p, it, st = ctx.leapfrog(P, Q[:, 0], Pm[:, 0], horizon, return_info=True)
    np.testing.assert_array_equal(it[:, 0], z["n_p"][:, :horizon].sum(1))
    np.testing.assert_array_equal(it[:, 1], z["n_q"][:, :horizon].sum(1))
    assert_state_close(q, Q[:, horizon], 1e-9, name + " q")
    assert_state_close(p, Pm[:, horizon], 1e-8, name + " p")
    assert not (st & capi.STATUS_NONFINITE).any()
    if name == "traj_bigk":       # the flux wall fires within the horizon
        assert (st & capi.STATUS_REFLECT_F).all()
    ctx.close()


def _bigk_batch(z, n, seed):
    """n chains around the traj_bigk start states (fluxes and positions jittered)."""
    rs = np.random.RandomState(seed)
    Q0, P0 = z["Q"][:, 0], z["P"][:, 0]
    idx = np.arange(n) % Q0.shape[0]
    q = Q0[idx].copy()
    q[:, 0::3] *= np.exp(0.05 * rs.randn(n, q.shape[1] // 3))
    q[:, 1::3] += 0.2 * rs.randn(n, q.shape[1] // 3)
    q[:, 2::3] += 0.2 * rs.randn(n, q.shape[1] // 3)
    return q, P0[idx].copy()


def test_bigk_batch_invariance_and_oracle(gpu_lib, bigk_kernel):
    """A ragged batch of K = 100 chains: every chain equals its single-chain
    launch bit for bit; a sample agrees with the oracle over 10 steps."""
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    q0, p0 = _bigk_batch(z, 13, 4)
    qb, pb, itb, stb = ctx.leapfrog(P, q0, p0, 10, return_info=True)
    m = R.RefModel(z["D"], par)
    for c in (0, 5, 12):
        qs, ps, its, sts = ctx.leapfrog(P, q0[c], p0[c], 10, return_info=True)
        assert np.array_equal(qs, qb[c]) and np.array_equal(ps, pb[c])
        assert np.array_equal(its, itb[c]) and sts == stb[c]
    for c in (0, 7):
        qo, po, NP, NQ = m.trajectory(q0[c], p0[c], 10, record=False)
        assert itb[c, 0] == NP.sum() and itb[c, 1] == NQ.sum()
        assert_state_close(qb[c], qo, 1e-9, "q chain %d" % c)
        assert_state_close(pb[c], po, 1e-8, "p chain %d" % c)
    ctx.close()


@pytest.mark.parametrize("solver", ["hmc", "naive", "leap_frog"])
def test_bigk_integrators_vs_oracle(gpu_lib, bigk_kernel, solver):
    """run_single_HMC / run_single_RHMC naive / leap_frog steps at K = 100
    (sampler_RHMC.py:628-645, :690-728) against the oracle, flux wall on."""
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    m = R.RefModel(z["D"], par)
    q0, p0 = _bigk_batch(z, 3, 6)
    sol = {"hmc": capi.SOLVER_HMC, "naive": capi.SOLVER_RHMC_NAIVE,
           "leap_frog": capi.SOLVER_RHMC_LEAPFROG}[solver]
    if solver == "hmc":       # unit metric: momenta of order one
        p0 = np.random.RandomState(2).randn(*q0.shape)
    qg, pg = ctx.integrate(P, sol, q0, p0, 8, f_pos=True)
    for c in range(3):
        q, p = q0[c].copy(), p0[c].copy()
        for _ in range(8):
            if solver == "hmc":
                q, p = m.hmc_step(q, p)
            elif solver == "naive":
                q, p = m.rhmc_naive_step(q, p, True)
            else:
                q, p = m.rhmc_leapfrog_step(q, p, True)
        assert_state_close(qg[c], q, 1e-9, "%s q chain %d" % (solver, c))
        assert_state_close(pg[c], p, 1e-8, "%s p chain %d" % (solver, c))
    ctx.close()


def test_bigk_hmc_random_vs_oracle(gpu_lib, bigk_kernel):
    """samplers.HMC_random trajectories (samplers.py:519-552) at K = 100,
    sticky flip and stale-momentum quirks included, against the oracle."""
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    m = R.RefModel(z["D"], par)
    q0, _ = _bigk_batch(z, 3, 8)
    K = q0.shape[1] // 3
    p0 = np.random.RandomState(3).randn(*q0.shape)
    dt = np.tile([2.0, 0.01, 0.01], K)
    steps = np.array([3, 5, 7], np.int32)
    qg, pg, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
    for c in range(3):
        qo, po, flip = m.hmc_random_traj(q0[c], p0[c], dt, int(steps[c]), par["f_lim"])
        assert bool(st[c] & capi.STATUS_REFLECT_F) == flip
        assert_state_close(qg[c], qo, 1e-9, "q chain %d" % c)
        assert_state_close(pg[c], po, 1e-8, "p chain %d" % c)
    ctx.close()


def _oracle_mh(m, q, z, u, n_iter, n_steps, f_pos=True):
    """run_RHMC's move-0 iteration (sampler_RHMC.py:1018-1083) on the oracle
    with given draws: returns the accept sequence and the final q."""
    acc = []
    for it in range(n_iter):
        Hd = m.H(q)
        p = z[it] * np.sqrt(Hd)
        E0 = m.V(q, f_pos) + m.T(p, Hd)
        q1, p1, _, _ = m.trajectory(q, p, n_steps, record=False)
        E1 = m.V(q1, f_pos) + m.T(p1, m.H(q1))
        dE = E1 - E0
        a = bool((dE < 0) or (np.log(u[it]) < -dE))
        acc.append(a)
        if a:
            q = q1
    return np.array(acc), q


def _bigk_mh_case(par, K=100, n=32, seed=31):
    """A 32x32 image of K true stars (RHMC-big-sim4.py's power law, mags
    15-20: every flux above the wall) and two chains at the truth, jittered
    (flux x lognormal 2 %, 0.05 px): with f_pos=True V is finite, so the MH
    test below really accepts and rejects."""
    rs = np.random.RandomState(seed)
    ftc = par["flux_to_count"]
    fmin, fmax = R.mag2flux(20.) * ftc, R.mag2flux(15.) * ftc
    u = rs.random_sample(K)                       # gen_pow_law_sample, alpha 2 (utils.py:460-471)
    f = np.exp(np.log(fmin ** -1. + u * (fmax ** -1. - fmin ** -1.)) / -1.)
    x = rs.random_sample(K) * (n - 2.) + 1.
    y = rs.random_sample(K) * (n - 2.) + 1.
    D = rs.poisson(R.model_image(n, n, np.stack([f, x, y], 1), par["B_count"],
                                 par["fwhm_pix"])).astype(float)
    q = np.empty((2, 3 * K))
    q[:, 0::3] = f * np.exp(0.02 * rs.randn(2, K))
    q[:, 1::3] = x + 0.05 * rs.randn(2, K)
    q[:, 2::3] = y + 0.05 * rs.randn(2, K)
    assert (q[:, 0::3] > 1.5 * par["f_lim"]).all()
    return D, q


def test_bigk_mh_vs_oracle(gpu_lib, bigk_kernel):
    """rhmc_mh (the four-kernel MH loop) at K = 100 with host draws: the
    accept sequence and chains of the oracle's run_RHMC move-0 iterations.
    The chains start above the flux wall (V finite), and the draws make both
    chains accept and reject (checked: a reject-everything or
    accept-everything MH fails)."""
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = dict(R.params_from_npz(z), dt=0.1)
    D, q0 = _bigk_mh_case(par)
    ctx = capi.Context(D)
    P = capi_params(capi, par)           # V_prior_const for V's prior (:320-321)
    m = R.RefModel(D, par)
    n_iter, n_steps = 6, 4
    rs = np.random.RandomState(12)
    zz = rs.randn(n_iter, 2, q0.shape[1])
    uu = rs.rand(n_iter, 2)
    out = ctx.mh(P, q0, n_iter, n_steps, f_pos=True, z=zz, u=uu, record=True)
    acc_all = out["accept"].astype(bool)
    for c in range(2):
        acc, qo = _oracle_mh(m, q0[c], zz[:, c], uu[:, c], n_iter, n_steps)
        assert 0 < acc.mean() < 1, acc
        np.testing.assert_array_equal(acc_all[:, c], acc)
        assert_state_close(out["q"][c], qo, 1e-9, "mh q chain %d" % c)
    assert np.isfinite(out["E_chain"]).all()
    ctx.close()


def test_k256_limit(gpu_lib, bigk_kernel):
    """K = 256 (four star slots per lane, the last LDS-table count) runs and
    matches the oracle; K = 1025 is rejected with RHMC_ERR_ARG."""
    capi = gpu_lib
    z = load_golden("traj_bigk")
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par)
    m = R.RefModel(z["D"], par)
    rs = np.random.RandomState(12)
    K = 256
    q = np.empty((2, 3 * K))
    q[:, 0::3] = par["f_lim"] * np.exp(1.5 * rs.rand(2, K) + 0.05)
    q[:, 1::3] = 1 + 30 * rs.rand(2, K)
    q[:, 2::3] = 1 + 30 * rs.rand(2, K)
    p = rs.randn(2, 3 * K) * np.sqrt(np.array([m.H(x) for x in q]))
    g = ctx.gradient(P, q, kind=1)
    for c in range(2):
        want = m.dphidq(q[c])
        assert np.abs(g[c] - want).max() / (np.abs(want).max() + 1) < 1e-10
    q1, p1, it, st = ctx.leapfrog(P, q, p, 2, return_info=True)
    for c in range(2):
        qo, po, NP, NQ = m.trajectory(q[c], p[c], 2, record=False)
        assert it[c, 0] == NP.sum() and it[c, 1] == NQ.sum()
        assert_state_close(q1[c], qo, 1e-10, "K=256 q")
        assert_state_close(p1[c], po, 1e-9, "K=256 p")
    with pytest.raises(capi.RhmcError):
        ctx.leapfrog(P, np.ones((1, 3 * 1025)), np.zeros((1, 3 * 1025)), 1)
    ctx.close()


def test_births_past_64_then_steps(gpu_lib):
    """Births from 64 stars (birth_death_move, sampler_RHMC.py:1200-1240; the
    engine's one-wave-per-chain kernels change register slot count at 64)
    followed by RHMC steps, V and T at the new dimension agree with the
    oracle, every flux above the wall so that V(f_pos=True) is finite (a
    32x32 image of 100 true stars, the chain at 64 of them).  The
    reference's own run_RHMC across K = 64 (rj_big.npz) is
    test_gpu_reference_runs.py::test_rj_big_run_RHMC_births_past_64."""
    from rhmc_amd.sampler import multi_gym
    zb = load_golden("traj_bigk")
    par = R.params_from_npz(zb)
    g = multi_gym(dt=0., Nsteps=0, g_xx=0.05, g_ff=4., g_ff2=4.)
    g.num_rows = g.num_cols = 32
    g.dt = 0.05
    g.use_prior, g.alpha = True, 2.
    g.fmin, g.fmax = g.mag2flux_converter(20.), g.mag2flux_converter(15.)
    g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
    D, qq = _bigk_mh_case(par)      # 100 true stars above the wall, chains near the truth
    g.D = D
    q = qq[0, :3 * 64].copy()       # 64 of them
    p = np.random.RandomState(4).randn(3 * 64) * np.sqrt(g.H(q))
    g.Nobjs, g.d = 64, 192
    g.V(q, f_pos=True)        # caches V_prior_const (:320-321), as run_RHMC's first V does
    np.random.seed(5)
    for _ in range(3):                                    # 64 -> 67 stars
        q, p, _ = g.birth_death_move(q, p, True)
    assert g.Nobjs == 67 and q.size == 201
    m = R.RefModel(D, dict(par, fmin=g.fmin, fmax=g.fmax))
    q1, p1 = g.RHMC_steps(q, p, 2)
    qo, po, _, _ = m.trajectory(q, p, 2, record=False)
    assert_state_close(q1, qo, 1e-9, "q after births")
    assert_state_close(p1, po, 1e-8, "p after births")
    Vg, Vo = g.V(q1, f_pos=True), m.V(q1, f_pos=True)
    assert np.isfinite(Vo)
    np.testing.assert_allclose(Vg, Vo, rtol=1e-12)
