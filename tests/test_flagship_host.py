"""The reference's flagship run, RHMC-big-sim4.py, on the host (no GPU):
rhmc_amd.big_sim4.setup() performs the script's calls in its order, so the
data image, the true and model stars, the noise histogram and NumPy's global
stream state before run_RHMC equal the reference's own run
(tests/golden/flagship.npz, make_goldens.py case_flagship) bit for bit; and
the native driver's Beta(beta_a, beta_b) density — the split / merge moves'
scipy.stats.beta.pdf / logpdf (sampler_RHMC.py:1342, :1363, :1438) —
against scipy at the flagship's (4, 4), the class default (2, 2) and
non-integer shapes."""
import numpy as np
import pytest

from conftest import load_golden


def test_big_sim4_setup_is_the_reference_script():
    from rhmc_amd import big_sim4
    f = load_golden("flagship")
    saved = np.random.get_state()
    try:
        g, q_true, q_model = big_sim4.setup()
        st = np.random.get_state()
    finally:
        np.random.set_state(saved)
    np.testing.assert_array_equal(q_true, f["q_true"])
    np.testing.assert_array_equal(q_model, f["q_model"])
    np.testing.assert_array_equal(g.D, f["D"])
    np.testing.assert_array_equal(g.hist_noise, f["hist_noise"])
    np.testing.assert_array_equal(g.centers_noise, f["centers_noise"])
    assert np.array_equal(st[1], f["rng_key"]) and st[2] == int(f["rng_pos"])
    assert (st[3], st[4]) == tuple(f["rng_gauss"])
    assert (g.K_split, g.beta_a, g.beta_b) == (1., 4., 4.)
    assert g.use_prior and g.alpha == 2.
    assert (g.fmin, g.fmax) == (f["par_fmin"], f["par_fmax"])
    assert (g.g_xx, g.g_ff, g.g_ff2) == (0.05, 4., 4.)
    assert (g.num_rows, g.num_cols) == (32, 32)
    kw = big_sim4.RUN_KW
    assert kw["P_move"] == list(f["P_move"]) and kw["N_max"] == int(f["N_max"])
    assert kw["Nsteps"] == int(f["nsteps"]) and kw["dt"] == float(f["dt"])


@pytest.mark.parametrize("a,b", [(4., 4.), (2., 2.), (1., 1.), (1.5, 3.25), (0.7, 2.), (9., 1.)])
def test_native_beta_density_matches_scipy(a, b):
    from scipy.stats import beta as BETA
    from rhmc_amd import rj_native
    rs = np.random.RandomState(3)
    x = np.concatenate([rs.rand(2000), rs.beta(a, b, 2000), [1e-12, 0.5, 1 - 1e-12, 0.25]])
    pdf, logpdf = rj_native.beta_eval(a, b, x)
    np.testing.assert_allclose(pdf, BETA.pdf(x, a, b), rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(logpdf, BETA.logpdf(x, a, b), rtol=1e-13, atol=1e-13)
    # the merge evaluates the pdf on every pair's F = f_j / (f_i + f_j), 0 outside [0, 1]
    out, _ = rj_native.beta_eval(a, b, np.array([-0.5, 1.5]))
    assert (out == 0).all()
