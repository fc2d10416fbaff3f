"""GPU tests of the sampler_RHMC mirror against the reference's own outputs:
full MH runs (multi_gym.run_RHMC) with the same global-RNG stream, the
single_gym implicit-solver energy trace, and the per-call methods."""
import numpy as np
import pytest

from conftest import load_golden
from helpers import assert_state_close
from oracle import rhmc_ref as R

pytestmark = pytest.mark.gpu


def _gym(par, cls="multi"):
    from rhmc_amd import sampler
    if cls == "multi":
        g = sampler.multi_gym(dt=0., Nsteps=0, g_xx=par["g_xx"], g_ff=par["g_ff"],
                              g_ff2=par["g_ff2"])
    else:
        g = sampler.single_gym(dt=0., Nsteps=0, g_xx=par["g_xx"], g_ff=par["g_ff"])
    g.num_rows, g.num_cols = int(par["rows"]), int(par["cols"])
    g.dt = par["dt"]
    g.use_prior = bool(par["use_prior"])
    g.alpha = par["alpha"]
    g.fmin, g.fmax = par["fmin"], par["fmax"]
    return g


@pytest.mark.parametrize("name", ["mh1", "mh3"])
def test_run_RHMC_reproduces_reference_chain(gpu_lib, name):
    z = load_golden("mh")
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    np.random.seed(int(z[name + "/seed"]))
    g.run_RHMC(z[name + "/q_model"].copy(), f_pos=True, delta=1e-6,
               Niter=int(z[name + "/niter"]), Nsteps=int(z[name + "/nsteps"]),
               dt=float(z[name + "/dt"]), N_max=z[name + "/q_model"].shape[0])
    np.testing.assert_array_equal(g.A_chain.astype(np.int32), z[name + "/A_chain"])
    assert_state_close(g.q_chain, z[name + "/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain, z[name + "/p_chain"], 1e-9, "p_chain")
    np.testing.assert_allclose(g.E_chain, z[name + "/E_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.V_chain, z[name + "/V_chain"], rtol=1e-11)


def test_single_gym_implicit_energy_trace(gpu_lib):
    z = load_golden("mh")
    par = R.params_from_npz(z, "single/par_")
    from rhmc_amd import sampler
    g = sampler.single_gym(dt=0., Nsteps=0, g_xx=1., g_ff=1.)
    g.num_rows = g.num_cols = 16
    g.fmin, g.fmax = par["fmin"], par["fmax"]
    g.D = z["single/D"]
    g.Nsteps, g.dt = 100, 0.1
    np.random.seed(5)
    g.run_single_RHMC(q_model_0=np.array([[19., 9., 8.]]), f_pos=True, solver="implicit",
                      delta=1e-6)
    assert_state_close(g.q_chain, z["single/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain, z["single/p_chain"], 1e-8, "p_chain")
    np.testing.assert_allclose(g.E_chain, z["single/E_chain"], atol=1e-8)


def test_methods_match_functions_golden(gpu_lib):
    z = load_golden("functions")
    for name in ("k1", "k10"):
        par = R.params_from_npz(z, name + "/par_")
        g = _gym(par)
        g.D = z[name + "/D"]
        for i, q in enumerate(z[name + "/q"]):
            want = z[name + "/dVdq"][i]
            scale = np.abs(want).max() + 1
            assert np.abs(g.dVdq(q) - want).max() / scale < 1e-10
            want = z[name + "/dphidq"][i]
            assert np.abs(g.dphidq(q) - want).max() / (np.abs(want).max() + 1) < 1e-10
            np.testing.assert_allclose(g.V(q), z[name + "/V"][i], rtol=1e-12)


def test_RHMC_single_step_matches_reference(gpu_lib):
    z = load_golden("steps")
    par = R.params_from_npz(z)
    g = _gym(par)
    g.D = z["D"]
    for i in range(0, len(z["q0"]), 5):
        q1, p1 = g.RHMC_single_step(z["q0"][i], z["p0"][i])
        assert_state_close(q1, z["q1"][i], 1e-11, "q")
        assert_state_close(p1, z["p1"][i], 1e-10, "p")


@pytest.mark.parametrize("name", ["mh1", "mh3"])
def test_run_RHMC_batched_one_chain_equals_reference(gpu_lib, name):
    """The fully on-device MH loop (rhmc_mh) fed the reference's own NumPy
    draws reproduces the reference chain (accept sequence exactly)."""
    z = load_golden("mh")
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    np.random.seed(int(z[name + "/seed"]))
    niter = int(z[name + "/niter"])
    g.run_RHMC_batched(z[name + "/q_model"].copy(), f_pos=True, Niter=niter,
                       Nsteps=int(z[name + "/nsteps"]), dt=float(z[name + "/dt"]))
    np.testing.assert_array_equal(g.A_chain[:, 0].astype(np.int32), z[name + "/A_chain"])
    K3 = g.q_chain.shape[2]
    assert_state_close(g.q_chain[:, 0], z[name + "/q_chain"][:, :K3], 1e-9, "q_chain")
    np.testing.assert_allclose(g.E_chain[:, 0], z[name + "/E_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.V_chain[:, 0], z[name + "/V_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.T_chain[:, 0], z[name + "/T_chain"], rtol=1e-10, atol=1e-10)


def test_run_RHMC_batched_many_chains_equal_single_runs(gpu_lib):
    """Chains with their own RandomState seeds equal one run_RHMC per seed."""
    z = load_golden("mh")
    par = R.params_from_npz(z, "mh3/par_")
    seeds = [123, 7, 99]
    g = _gym(par)
    g.D = z["mh3/D"]
    qm = z["mh3/q_model"]
    g.run_RHMC_batched(np.stack([qm] * 3), f_pos=True, Niter=10, Nsteps=10, dt=0.05,
                       seeds=seeds)
    Ab, qb = g.A_chain.copy(), g.q_chain.copy()
    for c, s in enumerate(seeds):
        h = _gym(par)
        h.D = z["mh3/D"]
        np.random.seed(s)
        h.run_RHMC(qm.copy(), f_pos=True, Niter=10, Nsteps=10, dt=0.05, N_max=3)
        np.testing.assert_array_equal(Ab[:, c], h.A_chain)
        assert_state_close(qb[:, c], h.q_chain, 1e-12, "chain %d" % c)


def test_mh_device_rng_deterministic_and_sane(gpu_lib):
    z = load_golden("mh")
    par = R.params_from_npz(z, "mh1/par_")
    g = _gym(par)
    g.D = z["mh1/D"]
    qm = np.stack([z["mh1/q_model"]] * 64)
    q1 = g.run_RHMC_batched(qm, Niter=30, Nsteps=10, dt=0.1, rng="device", seed=42)
    A1, E1 = g.A_chain.copy(), g.E_chain.copy()
    q2 = g.run_RHMC_batched(qm, Niter=30, Nsteps=10, dt=0.1, rng="device", seed=42)
    assert np.array_equal(q1, q2) and np.array_equal(A1, g.A_chain)
    q3 = g.run_RHMC_batched(qm, Niter=30, Nsteps=10, dt=0.1, rng="device", seed=43)
    assert not np.array_equal(q1, q3)
    assert np.isfinite(E1).all() and np.isfinite(q1).all()
    rate = A1.mean()
    assert 0.3 < rate <= 1.0, rate          # small-dt RHMC: high acceptance
    # chains decorrelate: not all identical after 30 iterations
    assert np.unique(q1[:, 1]).size > 32


@pytest.mark.parametrize("name,solver", [("hmc", None), ("naive", "naive"),
                                         ("leap_frog", "leap_frog"),
                                         ("leap_frog_k2", "leap_frog"),
                                         ("naive_wall", "naive")])
def test_single_gym_alternative_integrators(gpu_lib, name, solver):
    """run_single_HMC / run_single_RHMC(naive, leap_frog) on the GPU vs the reference."""
    from rhmc_amd import sampler
    z = load_golden("solvers")
    par = R.params_from_npz(z, name + "/par_")
    g = sampler.single_gym(dt=0., Nsteps=0, g_xx=1., g_ff=1.)
    g.num_rows = g.num_cols = 16
    g.fmin, g.fmax = par["fmin"], par["fmax"]
    g.D = z[name + "/D"]
    g.Nsteps, g.dt = int(z[name + "/nsteps"]), par["dt"]
    q0 = z[name + "/q_chain"][0].reshape(-1, 3).copy()
    q0[:, 0] = g.flux2mag_converter(q0[:, 0])
    np.random.seed(5)
    if solver is None:
        g.run_single_HMC(q_model_0=q0, f_pos=False)
    else:
        g.run_single_RHMC(q_model_0=q0, f_pos=True, solver=solver)
    assert_state_close(g.q_chain, z[name + "/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain, z[name + "/p_chain"], 1e-8, "p_chain")
    E, Ew = g.E_chain, z[name + "/E_chain"]
    assert np.array_equal(np.isinf(E), np.isinf(Ew))
    fin = np.isfinite(Ew)
    np.testing.assert_allclose(E[fin], Ew[fin], rtol=1e-9, atol=1e-7)


@pytest.mark.parametrize("name", ["rj_bd", "rj_sm", "rj_all"])
def test_run_RHMC_reversible_jump_moves(gpu_lib, name):
    """run_RHMC with birth/death and split/merge proposals (sampler_RHMC.py
    :1089-1187, :1200-1445): the same global-RNG stream (incl. scipy's Beta
    draws) gives the reference's move types, accept decisions, star counts
    and chains; the trajectories on both sides of a jump run on the GPU at
    the changed dimension."""
    z = load_golden("rj")
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    np.random.seed(int(z[name + "/seed"]))
    g.run_RHMC(z[name + "/q_model"].copy(), f_pos=True, delta=1e-6,
               Niter=int(z[name + "/niter"]), Nsteps=int(z[name + "/nsteps"]),
               dt=float(z[name + "/dt"]), N_max=int(z[name + "/N_max"]),
               P_move=list(z[name + "/P_move"]))
    np.testing.assert_array_equal(g.move_chain, z[name + "/move_chain"])
    np.testing.assert_array_equal(g.N_chain, z[name + "/N_chain"])
    np.testing.assert_array_equal(g.A_chain.astype(np.int32), z[name + "/A_chain"])
    assert (g.move_chain[g.A_chain] > 0).any()       # some dimension change accepted
    assert_state_close(g.q_chain, z[name + "/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain, z[name + "/p_chain"], 1e-9, "p_chain")
    np.testing.assert_allclose(g.E_chain, z[name + "/E_chain"], rtol=1e-11)


@pytest.mark.parametrize("engine", ["native", "python"])
def test_run_RHMC_rj_batched_equals_single_runs(gpu_lib, engine):
    """run_RHMC_rj_batched: chains at different, changing star counts, each on
    its own seeded stream, with every GPU phase batched over the chains
    (grouped by K) — through librhmc_rj.so (native) and the NumPy loop.  Chain 0 is the reference's rj_all run (its seed and
    start) and reproduces the golden; the others equal one run_RHMC per seed
    (which test_run_RHMC_reversible_jump_moves pins to the reference)."""
    z = load_golden("rj")
    name = "rj_all"
    par = R.params_from_npz(z, name + "/par_")
    kw = dict(f_pos=True, delta=1e-6, Niter=int(z[name + "/niter"]),
              Nsteps=int(z[name + "/nsteps"]), dt=float(z[name + "/dt"]),
              N_max=int(z[name + "/N_max"]), P_move=list(z[name + "/P_move"]))
    qm = z[name + "/q_model"]
    seed0 = int(z[name + "/seed"])
    # further chains: 2- and 3-star starts on seeds whose single runs complete
    # (the reference dead-ends on some: no star left, nothing mergeable)
    chains, singles = [(qm, seed0)], []
    for s in range(400, 440):
        if len(chains) == 4:
            break
        start = qm[:2] if len(chains) % 2 else qm
        h = _gym(par)
        h.D = z[name + "/D"]
        np.random.seed(s)
        try:
            with np.errstate(all="ignore"):
                h.run_RHMC(start.copy(), **kw)
        except Exception:
            continue
        chains.append((start, s))
        singles.append(h)
    assert len(chains) == 4
    g = _gym(par)
    g.D = z[name + "/D"]
    np.random.seed(1)
    before = np.random.get_state()[1].copy()
    q_end = g.run_RHMC_rj_batched([c[0].copy() for c in chains], [c[1] for c in chains],
                                  engine=engine, **kw)
    assert np.array_equal(np.random.get_state()[1], before)   # the global stream is untouched
    assert len(q_end) == 4
    # chain 0: the reference's own run
    np.testing.assert_array_equal(g.move_chain[:, 0], z[name + "/move_chain"])
    np.testing.assert_array_equal(g.N_chain[:, 0], z[name + "/N_chain"])
    np.testing.assert_array_equal(g.A_chain[:, 0].astype(np.int32), z[name + "/A_chain"])
    assert_state_close(g.q_chain[:, 0], z[name + "/q_chain"], 1e-9, "q_chain")
    assert_state_close(g.p_chain[:, 0], z[name + "/p_chain"], 1e-9, "p_chain")
    np.testing.assert_allclose(g.E_chain[:, 0], z[name + "/E_chain"], rtol=1e-11)
    # the others: one run_RHMC per seed
    for c, h in enumerate(singles, start=1):
        np.testing.assert_array_equal(g.move_chain[:, c], h.move_chain)
        np.testing.assert_array_equal(g.N_chain[:, c], h.N_chain)
        np.testing.assert_array_equal(g.A_chain[:, c], h.A_chain)
        assert_state_close(g.q_chain[:, c], h.q_chain, 1e-11, "chain %d" % c)
        np.testing.assert_allclose(g.E_chain[:, c], h.E_chain, rtol=1e-12)
    # the batch really mixed star counts, and some jump was accepted
    assert len(set(g.N_chain[-1])) > 1 or len(set(g.N_chain[:, 0])) > 1
    assert (g.move_chain[g.A_chain] > 0).any()


def _sched_gym(z, name):
    par = R.params_from_npz(z, name + "/par_")
    g = _gym(par)
    g.D = z[name + "/D"]
    if par["use_Vc"]:
        g.use_Vc, g.Vc_r_pow = True, par["Vc_r_pow"]
        g.f_expnt = np.zeros(z[name + "/q_model"].shape[0])
    sg = z[name + "/schedule_g_ff2"]
    sb = z[name + "/schedule_beta"]
    return g, sg, (sb if sb.size else None)


@pytest.mark.parametrize("name", ["g1", "g3", "g3vc"])
def test_run_RHMC_schedules_reproduce_reference(gpu_lib, name):
    """run_RHMC with schedule_g_ff2 (and schedule_beta with repulsion),
    sampler_RHMC.py:1010-1016 — the schedules are shorter than the run, so the
    hold-the-last-value rule is exercised."""
    z = load_golden("mh_sched")
    g, sg, sb = _sched_gym(z, name)
    np.random.seed(int(z[name + "/seed"]))
    g.run_RHMC(z[name + "/q_model"].copy(), f_pos=True, delta=1e-6,
               Niter=int(z[name + "/niter"]), Nsteps=int(z[name + "/nsteps"]),
               dt=float(z[name + "/dt"]), N_max=z[name + "/q_model"].shape[0],
               schedule_g_ff2=sg, schedule_beta=sb)
    np.testing.assert_array_equal(g.A_chain.astype(np.int32), z[name + "/A_chain"])
    assert_state_close(g.q_chain, z[name + "/q_chain"], 1e-9, "q_chain")
    np.testing.assert_allclose(g.E_chain, z[name + "/E_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.V_chain, z[name + "/V_chain"], rtol=1e-11)
    assert g.g_ff2 == z[name + "/g_ff2_final"] and g.beta == z[name + "/beta_final"]


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("name", ["g1", "g3", "g3vc"])
def test_run_RHMC_batched_schedules_reproduce_reference(gpu_lib, monkeypatch, name, fused):
    """The on-device MH loop (rhmc_mh_scheduled) with the reference's NumPy
    draws and its schedules reproduces the reference chain — on the fused
    one-star kernel (one launch per iteration under a schedule), the fused
    multi-star kernel and the four-kernel loop (fused=False, and g3vc: the
    repulsion re-evaluates V(q) per iteration under a beta schedule)."""
    from rhmc_amd import capi
    monkeypatch.setattr(capi, "DEFAULT_MH_FUSED", fused)
    z = load_golden("mh_sched")
    g, sg, sb = _sched_gym(z, name)
    np.random.seed(int(z[name + "/seed"]))
    g.run_RHMC_batched(z[name + "/q_model"].copy(), f_pos=True, Niter=int(z[name + "/niter"]),
                       Nsteps=int(z[name + "/nsteps"]), dt=float(z[name + "/dt"]),
                       schedule_g_ff2=sg, schedule_beta=sb)
    np.testing.assert_array_equal(g.A_chain[:, 0].astype(np.int32), z[name + "/A_chain"])
    K3 = g.q_chain.shape[2]
    assert_state_close(g.q_chain[:, 0], z[name + "/q_chain"][:, :K3], 1e-9, "q_chain")
    np.testing.assert_allclose(g.E_chain[:, 0], z[name + "/E_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.V_chain[:, 0], z[name + "/V_chain"], rtol=1e-11)
    np.testing.assert_allclose(g.T_chain[:, 0], z[name + "/T_chain"], rtol=1e-10, atol=1e-10)
    assert g.g_ff2 == z[name + "/g_ff2_final"] and g.beta == z[name + "/beta_final"]


@pytest.mark.parametrize("name", ["g1", "g3"])
def test_mh_constant_schedule_equals_unscheduled_run(gpu_lib, name):
    """A one-entry schedule (held for every iteration) equals the unscheduled
    run at that g_ff2, bit for bit, with device randoms: the scheduled path
    (one launch per iteration, Philox keyed by the run's iteration index,
    V(q) re-evaluated per launch) changes nothing but the constants."""
    z = load_golden("mh_sched")
    g, sg, _ = _sched_gym(z, name)
    g.dt = 0.02
    qm = np.stack([z[name + "/q_model"]] * 6).reshape(6, -1).copy()
    qm[:, 0::3] = g.mag2flux_converter(qm[:, 0::3])
    g.g_ff2 = sg[0]
    a = g._context().mh(g._params(for_energy=True), qm, 5, 6, seed=4, record=True)
    g.g_ff2 = 123.0            # overridden by the schedule in every iteration
    b = g._context().mh(g._params(for_energy=True), qm, 5, 6, seed=4, record=True,
                        schedule_g_ff2=np.array([sg[0]]))
    for k in ("q", "accept", "E_chain", "V_chain", "T_chain", "q_chain"):
        assert np.array_equal(a[k], b[k]), k
