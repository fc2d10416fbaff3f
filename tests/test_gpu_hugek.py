"""K > 256 stars per chain through the C-ABI: the slotted one-wave-per-chain
kernels at 8 and 16 register slots (up to 512 / 1024 stars) with their
windowed factor tables in global memory (rhmc_windowed.hpp WinGG; allocated
in a per-stream buffer of the context).  The reference's dVdq / V /
RHMC_single_step take any 3 * Nobjs (sampler_RHMC.py:365-425, :294-351,
:522-566); its own drivers stop at 120 stars, so this is the completeness
path, not a tuned one.

Pinned by reference fixtures (tests/golden/make_goldens.py case_hugek):
hugek.npz (dVdq, dphidq, V, T at K = 300 on 64x64 and K = 700 on 128x128,
big-sim4 parameters + prior), traj_hugek.npz (64x64, K = 300, 3 steps) and
traj_hugek700.npz (128x128, K = 700, 2 steps): every step from the
reference's own state with exact fixed-point iteration counts.  The
integrators, HMC_random, MH and the ragged entry points go against the
oracle or the fixed-K calls.
"""
import numpy as np
import pytest

from conftest import load_golden
from helpers import assert_state_close, capi_params
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["h300", "h700"])
def test_hugek_gradient_energy(gpu_lib, name):
    capi = gpu_lib
    z = load_golden("hugek")
    par = R.params_from_npz(z, name + "/par_")
    ctx = capi.Context(z[name + "/D"])
    P = capi_params(capi, par)
    q, p = z[name + "/q"], z[name + "/p"]
    assert q.shape[1] // 3 > 256
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


@pytest.mark.parametrize("name", ["traj_hugek", "traj_hugek700"])
def test_hugek_trajectory_stepwise_and_fused(gpu_lib, name):
    capi = gpu_lib
    z = load_golden(name)
    par = R.params_from_npz(z)
    ctx = capi.Context(z["D"])
    P = capi_params(capi, par, float(z["delta"]), int(z["counter_max"]))
    Q, Pm = z["Q"], z["P"]
    assert Q.shape[2] // 3 > 256
    n = Q.shape[1] - 1
    for s in range(n):
        q, p, it, st = ctx.leapfrog(P, Q[:, s], Pm[:, s], 1, return_info=True)
        np.testing.assert_array_equal(it[:, 0], z["n_p"][:, s], err_msg="p-iters step %d" % s)
        np.testing.assert_array_equal(it[:, 1], z["n_q"][:, s], err_msg="q-iters step %d" % s)
        assert_state_close(q, Q[:, s + 1], 1e-11, "%s q step %d" % (name, s))
        assert_state_close(p, Pm[:, s + 1], 1e-10, "%s p step %d" % (name, s))
    q, p, it, st = ctx.leapfrog(P, Q[:, 0], Pm[:, 0], n, return_info=True)
    np.testing.assert_array_equal(it[:, 0], z["n_p"][:, :n].sum(1))
    np.testing.assert_array_equal(it[:, 1], z["n_q"][:, :n].sum(1))
    assert_state_close(q, Q[:, n], 1e-10, name + " q fused")
    assert_state_close(p, Pm[:, n], 1e-9, name + " p fused")
    assert not (st & capi.STATUS_NONFINITE).any()
    ctx.close()


def _case(K, n_img, n_chains, seed, flux_floor=1.5):
    """A power-law image of K true stars (mags 15-20, every flux above the
    wall) and n_chains chains at the truth, jittered."""
    z = load_golden("traj_hugek")
    par = dict(R.params_from_npz(z), rows=n_img, cols=n_img)
    rs = np.random.RandomState(seed)
    ftc = par["flux_to_count"]
    fmin, fmax = R.mag2flux(20.) * ftc, R.mag2flux(15.) * ftc
    u = rs.random_sample(K)
    f = np.exp(np.log(fmin ** -1. + u * (fmax ** -1. - fmin ** -1.)) / -1.)
    x = rs.random_sample(K) * (n_img - 2.) + 1.
    y = rs.random_sample(K) * (n_img - 2.) + 1.
    D = rs.poisson(R.model_image(n_img, n_img, np.stack([f, x, y], 1), par["B_count"],
                                 par["fwhm_pix"])).astype(float)
    q = np.empty((n_chains, 3 * K))
    q[:, 0::3] = f * np.exp(0.02 * rs.randn(n_chains, K))
    q[:, 1::3] = x + 0.05 * rs.randn(n_chains, K)
    q[:, 2::3] = y + 0.05 * rs.randn(n_chains, K)
    assert (q[:, 0::3] > flux_floor * par["f_lim"]).all()
    return D, q, par


def test_hugek_batch_invariance_and_limit(gpu_lib):
    """Five K = 300 chains: each equals its single-chain launch bit for bit
    (the table region follows the launch's wave index), one agrees with the
    oracle; K = 1025 is rejected with RHMC_ERR_ARG."""
    capi = gpu_lib
    D, q0, par = _case(300, 64, 5, 3)
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    m = R.RefModel(D, par)
    p0 = np.random.RandomState(5).randn(*q0.shape) * np.sqrt(np.array([m.H(x) for x in q0]))
    qb, pb, itb, stb = ctx.leapfrog(P, q0, p0, 3, return_info=True)
    for c in (0, 2, 4):
        qs, ps, its, sts = ctx.leapfrog(P, q0[c], p0[c], 3, return_info=True)
        assert np.array_equal(qs, qb[c]) and np.array_equal(ps, pb[c])
        assert np.array_equal(its, itb[c]) and sts == stb[c]
    qo, po, NP, NQ = m.trajectory(q0[1], p0[1], 3, record=False)
    assert itb[1, 0] == NP.sum() and itb[1, 1] == NQ.sum()
    assert_state_close(qb[1], qo, 1e-10, "q chain 1")
    assert_state_close(pb[1], po, 1e-9, "p chain 1")
    with pytest.raises(capi.RhmcError) as e:
        ctx.leapfrog(P, np.ones((1, 3 * 1025)), np.zeros((1, 3 * 1025)), 1)
    assert e.value.code == capi.RHMC_ERR_ARG
    ctx.close()


@pytest.mark.parametrize("solver", ["hmc", "naive", "leap_frog"])
def test_hugek_integrators_vs_oracle(gpu_lib, solver):
    """run_single_HMC / run_single_RHMC naive / leap_frog at K = 300
    (sampler_RHMC.py:628-645, :690-728) against the oracle, flux wall on."""
    capi = gpu_lib
    D, q0, par = _case(300, 64, 2, 6)
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    m = R.RefModel(D, par)
    sol = {"hmc": capi.SOLVER_HMC, "naive": capi.SOLVER_RHMC_NAIVE,
           "leap_frog": capi.SOLVER_RHMC_LEAPFROG}[solver]
    rs = np.random.RandomState(2)
    if solver == "hmc":       # unit metric: momenta of order one
        p0 = rs.randn(*q0.shape)
    else:
        p0 = rs.randn(*q0.shape) * np.sqrt(np.array([m.H(x) for x in q0]))
    qg, pg = ctx.integrate(P, sol, q0, p0, 3, f_pos=True)
    for c in range(2):
        q, p = q0[c].copy(), p0[c].copy()
        for _ in range(3):
            if solver == "hmc":
                q, p = m.hmc_step(q, p)
            elif solver == "naive":
                q, p = m.rhmc_naive_step(q, p, True)
            else:
                q, p = m.rhmc_leapfrog_step(q, p, True)
        assert_state_close(qg[c], q, 1e-9, "%s q chain %d" % (solver, c))
        assert_state_close(pg[c], p, 1e-8, "%s p chain %d" % (solver, c))
    ctx.close()


def test_hugek_hmc_random_vs_oracle(gpu_lib):
    """samplers.HMC_random trajectories (samplers.py:519-552) at K = 600
    (16 register slots) against the oracle."""
    capi = gpu_lib
    D, q0, par = _case(600, 96, 2, 8)
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    m = R.RefModel(D, par)
    K = q0.shape[1] // 3
    p0 = np.random.RandomState(3).randn(*q0.shape)
    dt = np.tile([2.0, 0.01, 0.01], K)
    steps = np.array([2, 3], np.int32)
    qg, pg, st = ctx.hmc_random(P, dt, q0, p0, steps, return_status=True)
    for c in range(2):
        qo, po, flip = m.hmc_random_traj(q0[c], p0[c], dt, int(steps[c]), par["f_lim"])
        assert bool(st[c] & capi.STATUS_REFLECT_F) == flip
        assert_state_close(qg[c], qo, 1e-9, "q chain %d" % c)
        assert_state_close(pg[c], po, 1e-8, "p chain %d" % c)
    ctx.close()


def test_hugek_mh_vs_oracle(gpu_lib):
    """rhmc_mh at K = 300 with host draws against the oracle's run_RHMC
    move-0 iterations (sampler_RHMC.py:1018-1083), f_pos on, chains above the
    wall; both chains accept and reject."""
    from test_gpu_bigk import _oracle_mh
    capi = gpu_lib
    D, q0, par = _case(300, 64, 2, 21)
    par = dict(par, dt=0.3)                # the oracle: 2 / 5 and 4 / 5 accepted
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    m = R.RefModel(D, par)
    n_iter, n_steps = 5, 3
    rs = np.random.RandomState(14)
    zz = rs.randn(n_iter, 2, q0.shape[1])
    uu = rs.rand(n_iter, 2)
    out = ctx.mh(P, q0, n_iter, n_steps, f_pos=True, z=zz, u=uu, record=True)
    acc_all = out["accept"].astype(bool)
    for c in range(2):
        acc, qo = _oracle_mh(m, q0[c], zz[:, c], uu[:, c], n_iter, n_steps)
        assert 0 < acc.mean() < 1, acc
        np.testing.assert_array_equal(acc_all[:, c], acc)
        assert_state_close(out["q"][c], qo, 1e-9, "mh q chain %d" % c)
    ctx.close()


def test_hugek_ragged_equals_fixed_K(gpu_lib):
    """The ragged entry points past 256 stars: chains of 257..512 stars (8
    slots) in one launch equal fixed-K calls bit for bit; a set that spans
    8 and 16 slots is rejected (RHMC_ERR_ARG)."""
    import torch
    capi = gpu_lib
    D, qa, par = _case(512, 96, 1, 11)
    ctx = capi.Context(D)
    P = capi_params(capi, par)
    m = R.RefModel(D, par)
    Ks = [300, 512, 257, 400]
    ld = 3 * 512
    q = np.zeros((len(Ks), ld))
    p = np.zeros((len(Ks), ld))
    rs = np.random.RandomState(2)
    for c, K in enumerate(Ks):
        q[c, :3 * K] = qa[0, :3 * K]
        q[c, 1:3 * K:3] += 0.05 * rs.randn(K)
        p[c, :3 * K] = rs.randn(3 * K) * np.sqrt(m.H(q[c, :3 * K]))
    for K in Ks:
        assert ctx.ragged_ok(P, K)
    dev = torch.device("cuda:0")
    qd = torch.from_numpy(q.copy()).to(dev)
    pd = torch.from_numpy(p.copy()).to(dev)
    Kd = torch.tensor(Ks, dtype=torch.int32, device=dev)
    Vd = torch.zeros(len(Ks), dtype=torch.float64, device=dev)
    ctx.energy_ragged_device(P, qd.data_ptr(), ld, 0, Kd.data_ptr(), len(Ks), 257, 512,
                             capi.V_FLUX_WALL, Vd.data_ptr())
    ctx.leapfrog_ragged_device(P, qd.data_ptr(), pd.data_ptr(), ld, 0, Kd.data_ptr(), len(Ks),
                               257, 512, 2)
    torch.cuda.synchronize()
    qg, pg, Vg = qd.cpu().numpy(), pd.cpu().numpy(), Vd.cpu().numpy()
    for c, K in enumerate(Ks):
        V, _ = ctx.energy(P, q[c, :3 * K][None], None, f_pos=True)
        assert Vg[c] == V[0], (c, K)
        q1, p1 = ctx.leapfrog(P, q[c, :3 * K][None], p[c, :3 * K][None], 2)
        assert np.array_equal(qg[c, :3 * K], q1[0]) and np.array_equal(pg[c, :3 * K], p1[0]), c
        assert not qg[c, 3 * K:].any() and not pg[c, 3 * K:].any()
    with pytest.raises(capi.RhmcError) as e:
        ctx.leapfrog_ragged_device(P, qd.data_ptr(), pd.data_ptr(), ld, 0, Kd.data_ptr(),
                                   len(Ks), 256, 512, 1)
    assert e.value.code == capi.RHMC_ERR_ARG
    ctx.close()
