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
