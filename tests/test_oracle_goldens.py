"""Pin the CPU oracle (oracle/rhmc_ref.py) to the reference's own outputs.

The golden vectors were produced by running the reference itself
(tests/golden/make_goldens.py).  The oracle restates the same NumPy
expressions in the same order, so agreement is expected to the last ulp or
so; trajectories must reproduce the per-step fixed-point iteration counts
exactly.
"""
import numpy as np
import pytest

from conftest import load_golden
from oracle import rhmc_ref as R


def test_constants_match_reference():
    z = load_golden("functions")
    par = R.params_from_npz(z, "k1/par_")
    d = R.default_setup()
    for k in ("B_count", "f_lim", "f_low", "flux_to_count"):
        assert d[k] == par[k], k
    assert d["fwhm_pix"] == par["fwhm_pix"]
    g = R.factors(48, 48, 24., 24., d["fwhm_pix"])
    assert g == (par["g0"], par["g1"], par["g2"])     # bit-exact


def test_gauss_psf_and_factors():
    z = load_golden("functions")
    for i in range(4):
        r, c, x, y, fw = z["psf%d_args" % i]
        np.testing.assert_array_equal(R.gauss_psf(int(r), int(c), x, y, fw), z["psf%d" % i])
    for args, want in zip(z["factors_args"], z["factors"]):
        got = R.factors(int(args[0]), int(args[1]), args[2], args[3], 1.4 / 0.4)
        np.testing.assert_array_equal(np.array(got), want)


@pytest.mark.parametrize("name", ["k1", "k1gff2", "k10", "vc5"])
def test_functions(name):
    z = load_golden("functions")
    par = R.params_from_npz(z, name + "/par_")
    m = R.RefModel(z[name + "/D"], par)
    qs, ps = z[name + "/q"], z[name + "/p"]
    tol = dict(rtol=1e-13, atol=1e-13)
    for i, (q, p) in enumerate(zip(qs, ps)):
        np.testing.assert_allclose(m.dVdq(q), z[name + "/dVdq"][i], **tol)
        np.testing.assert_allclose(m.H(q), z[name + "/H"][i], rtol=1e-15)
        hv, hg = m.H(q, grad=True)
        np.testing.assert_allclose(hv, z[name + "/Hv"][i], rtol=1e-15)
        np.testing.assert_allclose(hg, z[name + "/Hg"][i], rtol=1e-15)
        np.testing.assert_allclose(m.dphidq(q), z[name + "/dphidq"][i], **tol)
        np.testing.assert_allclose(m.dtaudq(q, p), z[name + "/dtaudq"][i], rtol=1e-15)
        np.testing.assert_allclose(m.dtaudp(q, p), z[name + "/dtaudp"][i], rtol=1e-15)
        np.testing.assert_allclose(m.V(q), z[name + "/V"][i], rtol=1e-14)
        np.testing.assert_allclose(m.V(q, f_pos=True), z[name + "/Vpos"][i], rtol=1e-14)
        np.testing.assert_allclose(m.T(p, m.H(q)), z[name + "/T"][i], rtol=1e-14)


def test_single_steps_exact():
    z = load_golden("steps")
    m = R.RefModel(z["D"], R.params_from_npz(z))
    for i in range(len(z["q0"])):
        q1, p1, a, b = m.step(z["q0"][i], z["p0"][i])
        assert (a, b) == (z["n_p"][i], z["n_q"][i])
        np.testing.assert_allclose(q1, z["q1"][i], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(p1, z["p1"][i], rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("name,steps", [("traj_c1", 100), ("traj_c2", 60), ("traj_gff2", 200),
                                        ("traj_c3", 40), ("traj_prior", 80), ("traj_vc", 50),
                                        ("traj_edge", 200), ("traj_cmax", 100)])
def test_trajectories(name, steps):
    z = load_golden(name)
    m = R.RefModel(z["D"], R.params_from_npz(z))
    delta, cmax = float(z["delta"]), int(z["counter_max"])
    for c in range(z["Q"].shape[0]):
        Q, P, NP, NQ = m.trajectory(z["Q"][c, 0], z["P"][c, 0], steps, delta, cmax)
        np.testing.assert_array_equal(NP, z["n_p"][c, :steps])
        np.testing.assert_array_equal(NQ, z["n_q"][c, :steps])
        np.testing.assert_allclose(Q, z["Q"][c, :steps + 1], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(P, z["P"][c, :steps + 1], rtol=1e-8, atol=1e-8)


@pytest.mark.parametrize("name,kind", [("hmc", "hmc"), ("naive", "naive"),
                                       ("leap_frog", "lf"), ("leap_frog_k2", "lf"),
                                       ("naive_wall", "naive")])
def test_alternative_integrators(name, kind):
    z = load_golden("solvers")
    m = R.RefModel(z[name + "/D"], R.params_from_npz(z, name + "/par_"))
    Q, P = z[name + "/q_chain"], z[name + "/p_chain"]
    q, p = Q[0].copy(), P[0].copy()
    for s in range(Q.shape[0] - 1):
        if kind == "hmc":
            q, p = m.hmc_step(q, p)
        elif kind == "naive":
            q, p = m.rhmc_naive_step(q, p, True)
        else:
            q, p = m.rhmc_leapfrog_step(q, p, True)
        np.testing.assert_allclose(q, Q[s + 1], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(p, P[s + 1], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("name", ["k1_48", "k1_32", "k2_16", "k10_48"])
def test_model_image(name):
    """oracle model_image == the reference's gen_model (sampler_RHMC.py:101-116)."""
    z = load_golden("datagen")
    par = R.params_from_npz(z, name + "/par_")
    got = R.model_image(int(par["rows"]), int(par["cols"]), z[name + "/q"], par["B_count"],
                        par["fwhm_pix"])
    np.testing.assert_array_equal(got, z[name + "/model"])


def hmc_random_model(z, name):
    """Oracle model for a hmc_random golden case (lightsource_gym: no prior,
    unit metric; only B and the PSF width matter)."""
    D = z[name + "/D"]
    n = D.shape[0]
    par = dict(rows=n, cols=n, B_count=float(z[name + "/B_count"]),
               fwhm_pix=float(z[name + "/fwhm_pix"]), use_prior=0, use_Vc=0, alpha=2.,
               beta=1., Vc_r_pow=1., dt=1., f_lim=float(z[name + "/f_lim"]), f_low=1.,
               g_xx=1., g_ff=1., g_ff2=1., g0=1., g1=1., g2=1., fmin=-1., fmax=-1.)
    return R.RefModel(D, par)


@pytest.mark.parametrize("name", ["k1", "k2", "wall", "wall2"])
def test_hmc_random_exact(name):
    """samplers.lightsource_gym.HMC_random (per-coordinate dt, random
    trajectory lengths, sticky-flip / stale-p flux-wall quirks) replayed from
    the reference's seed: bit-identical chains, energies and decisions."""
    z = load_golden("hmc_random")
    m = hmc_random_model(z, name)
    rs = np.random.RandomState(int(z[name + "/seed"]))
    qc, Ec, dEc, Ac = m.hmc_random(z[name + "/q0"], z[name + "/dt"], int(z[name + "/Niter"]),
                                   int(z[name + "/steps_min"]), int(z[name + "/steps_max"]),
                                   float(z[name + "/f_lim"]), rng=rs)
    np.testing.assert_array_equal(qc, z[name + "/q_chain"])
    np.testing.assert_array_equal(Ec, z[name + "/E_chain"])
    np.testing.assert_array_equal(dEc, z[name + "/dE_chain"])
    np.testing.assert_array_equal(Ac, z[name + "/A_chain"])


@pytest.mark.parametrize("name", ["b100", "b100vc", "b120", "b128"])
def test_functions_bigk(name):
    """K > 64 (RHMC-big-sim3/4 geometry): dVdq, dphidq, V, T of the reference."""
    z = load_golden("bigk")
    par = R.params_from_npz(z, name + "/par_")
    m = R.RefModel(z[name + "/D"], par)
    qs, ps = z[name + "/q"], z[name + "/p"]
    assert qs.shape[1] // 3 > 64
    for i, (q, p) in enumerate(zip(qs, ps)):
        np.testing.assert_allclose(m.dVdq(q), z[name + "/dVdq"][i], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(m.dphidq(q), z[name + "/dphidq"][i], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(m.H(q), z[name + "/H"][i], rtol=1e-15)
        np.testing.assert_allclose(m.V(q), z[name + "/V"][i], rtol=1e-14)
        vp = m.V(q, f_pos=True)
        assert np.isinf(vp) == np.isinf(z[name + "/Vpos"][i])
        np.testing.assert_allclose(m.T(p, m.H(q)), z[name + "/T"][i], rtol=1e-14)


@pytest.mark.parametrize("name,chains,steps", [("traj_bigk", 2, 50), ("traj_bigk256", 1, 4),
                                               ("traj_c5", 1, 8)])
def test_trajectories_many_stars(name, chains, steps):
    """K = 100 (32x32), K = 128 (256x256) and C5 (K = 64, 256x256): the oracle
    reproduces the reference's steps and fixed-point iteration counts."""
    z = load_golden(name)
    m = R.RefModel(z["D"], R.params_from_npz(z))
    for c in range(chains):
        Q, P, NP, NQ = m.trajectory(z["Q"][c, 0], z["P"][c, 0], steps)
        np.testing.assert_array_equal(NP, z["n_p"][c, :steps])
        np.testing.assert_array_equal(NQ, z["n_q"][c, :steps])
        np.testing.assert_allclose(Q, z["Q"][c, :steps + 1], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(P, z["P"][c, :steps + 1], rtol=1e-8, atol=1e-8)


def test_c5_golden_reflects():
    """traj_c5: 4 chains x 50 reference steps, every chain through the flux wall."""
    z = load_golden("traj_c5")
    assert z["Q"].shape[:2] == (4, 51)
    assert (z["Q"][:, 1:, 0::3] < float(z["par_f_lim"])).any(axis=(1, 2)).all()


def _mh_start(z, prefix):
    par = R.params_from_npz(z, prefix + "par_")
    q0 = z[prefix + "q_model"].copy()
    q0[:, 0] = R.mag2flux(q0[:, 0]) * par["flux_to_count"]      # format_q (:209-217)
    return par, q0.reshape(-1)


@pytest.mark.parametrize("golden,name", [("mh", "mh1"), ("mh", "mh3"), ("mh_bigk", "d51"),
                                         ("mh_bigk", "w64")])
def test_run_RHMC_move0_replay(golden, name):
    """multi_gym.run_RHMC with P_move = [1, 0, 0] restated (RefModel.run_mh)
    on the reference's seeded stream reproduces the reference runs: the
    accept sequence exactly, states and energies to a few ulp.  mh_bigk: many
    stars with every start above the flux wall (d51: RHMC-big-sim4.py's
    32x32 / 51-star geometry; w64: the C5 geometry, 256x256 / 64 stars), where
    proposals are really accepted and rejected."""
    z = load_golden(golden)
    p = name + "/"
    par, q0 = _mh_start(z, p)
    m = R.RefModel(z[p + "D"], par)
    n_it = int(z[p + "niter"]) + 1
    o = m.run_mh(q0, np.random.RandomState(int(z[p + "seed"])), n_it, int(z[p + "nsteps"]))
    A = z[p + "A_chain"].astype(bool)
    np.testing.assert_array_equal(o["A_chain"], A)
    if golden == "mh_bigk":
        assert 0 < A.mean() < 1 and np.isfinite(z[p + "E_chain"]).all()
    K3 = q0.size
    np.testing.assert_allclose(o["q_chain"], z[p + "q_chain"][:, :K3], rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(o["p_chain"], z[p + "p_chain"][:, :K3], rtol=1e-12, atol=1e-12)
    for k in ("E_chain", "V_chain"):
        np.testing.assert_allclose(o[k], z[p + k], rtol=1e-13)


def test_rj_goldens_start_above_the_wall_and_jump():
    """rj_big (64 model stars, births / splits past 64, RHMC-big-sim4.py's move
    parameters) and flagship (RHMC-big-sim4.py as written, Niter 40): finite
    energies, every move type proposed, jumps accepted, the chain past 64
    stars in rj_big."""
    z = load_golden("rj_big")
    assert np.isfinite(z["b64/E_chain"]).all()
    assert z["b64/N_chain"].max() > 65 and z["b64/N_chain"][0] == 64
    assert 0 < z["b64/A_chain"].mean() < 1
    assert (z["b64/beta_a"], z["b64/beta_b"], z["b64/K_split"]) == (4., 4., 1.)
    f = load_golden("flagship")
    assert np.isfinite(f["E_chain"]).all()
    assert set(np.unique(f["move_chain"])) == {0, 1, 2, 3, 4}
    acc = f["A_chain"].astype(bool)
    assert set(np.unique(f["move_chain"][acc])) == {0, 1, 2, 3, 4}
    assert f["N_chain"][0] == 5 and f["q_true"].shape == (51, 3)
    assert list(f["P_move"]) == [0.6, 0.2, 0.2] and int(f["N_max"]) == 120
