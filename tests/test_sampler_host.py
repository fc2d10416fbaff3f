"""CPU tests of the sampler mirror's host-side pieces (no GPU needed): the
constructor state, the O(K) metric helpers and the data generation match the
reference goldens; device-backed methods refuse to run without a GPU instead
of falling back to the CPU."""
import numpy as np
import pytest

from conftest import load_golden
from oracle import rhmc_ref as R


def _gym_from(par, cls="multi"):
    from rhmc_amd import sampler
    g = (sampler.multi_gym if cls == "multi" else sampler.single_gym)(
        dt=par["dt"], g_xx=par["g_xx"], g_ff=par["g_ff"], g_ff2=par["g_ff2"])
    g.num_rows, g.num_cols = int(par["rows"]), int(par["cols"])
    g.use_prior = bool(par["use_prior"])
    g.alpha = par["alpha"]
    g.use_Vc = bool(par["use_Vc"])
    g.beta, g.Vc_r_pow = par["beta"], par["Vc_r_pow"]
    g.fmin, g.fmax = par["fmin"], par["fmax"]
    return g


def test_constructor_constants_match_reference():
    from rhmc_amd import sampler
    z = load_golden("functions")
    par = R.params_from_npz(z, "k1/par_")
    g = sampler.multi_gym(g_xx=1., g_ff=1., g_ff2=1.)
    for k, a in (("B_count", "B_count"), ("f_lim", "f_lim"), ("g0", "g0"), ("g1", "g1"),
                 ("g2", "g2"), ("fwhm_pix", "PSF_FWHM_pix"), ("flux_to_count", "flux_to_count")):
        assert getattr(g, a) == par[k], k
    assert g.num_rows == g.num_cols == 48 and g.mB == 23
    s = sampler.single_gym(g_ff2=7.)
    assert s.g_ff2 == 1.                         # single_gym ignores g_ff2 (:578)


@pytest.mark.parametrize("name", ["k1", "k1gff2", "k10", "vc5"])
def test_host_metric_helpers(name):
    z = load_golden("functions")
    par = R.params_from_npz(z, name + "/par_")
    g = _gym_from(par)
    for i, (q, p) in enumerate(zip(z[name + "/q"], z[name + "/p"])):
        np.testing.assert_array_equal(g.H(q), z[name + "/H"][i])
        hv, hg = g.H(q, grad=True)
        np.testing.assert_array_equal(hv, z[name + "/Hv"][i])
        np.testing.assert_array_equal(hg, z[name + "/Hg"][i])
        np.testing.assert_array_equal(g.dtaudq(q, p), z[name + "/dtaudq"][i])
        np.testing.assert_array_equal(g.dtaudp(q, p), z[name + "/dtaudp"][i])
        np.testing.assert_allclose(g.T(p, g.H(q)), z[name + "/T"][i], rtol=1e-15)


def test_gen_mock_data_matches_reference_rng_stream():
    """gen_mock_data draws the same Poisson stream as the reference."""
    from rhmc_amd import sampler
    z = load_golden("functions")
    g = sampler.multi_gym(g_xx=1., g_ff=1., g_ff2=1.)
    np.random.seed(77)
    g.gen_mock_data(np.array([[19., 24.3, 23.8]]))
    np.testing.assert_array_equal(g.D, z["k1/D"])


def test_format_q_roundtrip():
    from rhmc_amd import sampler
    g = sampler.multi_gym()
    stars = np.array([[19., 24.3, 23.8], [21., 3., 4.]])
    q = g.format_q(stars.copy())
    np.testing.assert_allclose(g.reverse_format_q(q), stars, rtol=1e-13)


def test_quirk_errors_like_reference():
    from rhmc_amd import sampler
    g = sampler.multi_gym()
    g.use_Vc = True                               # f_expnt is None -> TypeError (:388)
    with pytest.raises(TypeError):
        g._params()
    g2 = sampler.multi_gym()
    with pytest.raises(TypeError):                # fmin/fmax None -> TypeError (:321)
        g2._params(for_energy=True)
    g3 = sampler.multi_gym()
    g3.fmin = g3.fmax = None
    with pytest.raises(AssertionError):            # birth needs the prior range (:1205-1207)
        g3.birth_death_move(np.zeros(3), np.zeros(3), birth_death=True)


@pytest.mark.parametrize("name,cls", [("k1_48", "multi"), ("k1_32", "single"),
                                      ("k2_16", "single"), ("k10_48", "multi")])
def test_datagen_numpy_path_matches_reference(name, cls):
    """gen_model / gen_mock_data / gen_noise_profile with the NumPy stream are the
    reference's outputs bit for bit (goldens: make_goldens.py case_datagen)."""
    z = load_golden("datagen")
    par = R.params_from_npz(z, name + "/par_")
    g = _gym_from(par, cls)
    stars = z[name + "/stars"]
    np.testing.assert_array_equal(g.gen_model(stars), z[name + "/model"])
    np.random.seed(31)
    np.testing.assert_array_equal(g.gen_mock_data(stars, return_data=True), z[name + "/D"])
    np.random.seed(32)
    g.gen_noise_profile(stars, N_trial=8, sig_fac=10)
    np.testing.assert_array_equal(g.hist_noise, z[name + "/hist"])
    np.testing.assert_array_equal(g.centers_noise, z[name + "/centers"])
    with pytest.raises(ValueError):
        g.gen_mock_data(stars, rng="bogus")


def test_run_RHMC_verbose_report_after_move0(capsys):
    """The verbose progress block (sampler_RHMC.py:1183-1186) runs after every
    move type, including the fixed-dimension move 0: N_objs and the running
    acceptance report are printed at l % 50 == 0.  The device-backed step and
    energy are stubbed (host control flow only)."""
    from rhmc_amd import sampler
    g = sampler.multi_gym(g_xx=1., g_ff=1., g_ff2=1.)
    g.fmin, g.fmax = 1.0, 1e4
    g.RHMC_steps = lambda q, p, n, delta=1e-6, counter_max=1000: (q, p)
    g.V = lambda q, f_pos=True: 0.0
    np.random.seed(0)
    g.run_RHMC(np.array([[19., 24.3, 23.8]]), Niter=50, Nsteps=3, verbose=True)
    out = capsys.readouterr().out
    assert "Completed iteration 0" in out and "Completed iteration 50" in out
    assert out.count("N_objs: 1") == 2
    assert g.A_chain.all()                        # dE = T1 - T0 = 0 with the stubs


def test_vectorised_H_is_bit_identical():
    """run_RHMC_rj_batched's per-chain host work uses _H_vec: it must equal the
    reference-order per-star H bit for bit (fluxes on both sides of the f_low
    clamp, several metric settings)."""
    from rhmc_amd import sampler
    rs = np.random.RandomState(3)
    for g_xx, g_ff, g_ff2 in ((1., 1., 1.), (0.05, 4., 4.), (10., 10., 2.)):
        g = sampler.multi_gym(g_xx=g_xx, g_ff=g_ff, g_ff2=g_ff2)
        f_low = g.mag2flux_converter(g.mB + 2)
        K = 60
        q = np.empty(3 * K)
        q[0::3] = np.concatenate([f_low * rs.uniform(0.01, 0.999, K // 3),
                                  f_low * rs.uniform(1.001, 1e4, K - K // 3 - 1), [f_low]])
        q[1::3] = rs.uniform(0, 32, K)
        q[2::3] = rs.uniform(0, 32, K)
        assert np.array_equal(g._H_vec(q), g.H(q, grad=False))


def test_format_q_fast_is_bit_identical():
    """The batched native RJ driver converts magnitudes with _format_q_fast:
    bit for bit format_q (sampler_RHMC.py:209-217)."""
    from rhmc_amd import sampler
    g = sampler.multi_gym()
    rs = np.random.RandomState(5)
    for K in (1, 3, 51, 120):
        m = np.column_stack([rs.uniform(14, 24, K), rs.uniform(0, 48, K), rs.uniform(0, 48, K)])
        assert np.array_equal(g._format_q_fast(m), g.format_q(m.copy()))


def test_native_start_packing_is_format_q():
    """The native RJ driver's starts (rj_native.pack_starts: one pass in C++
    with libm pow) equal format_q of every chain (sampler_RHMC.py:209-217)
    bit for bit, zero-padded to 3 N_max; flat flux-count starts pass
    unchanged."""
    from rhmc_amd import rj_native, sampler
    g = sampler.multi_gym(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    rs = np.random.RandomState(12)
    starts = [np.column_stack([15 + 8.3 * rs.rand(k), 32 * rs.rand(k), 32 * rs.rand(k)])
              for k in (1, 5, 51, 3, 120)]
    q, K = rj_native.pack_starts(starts, 120, g.flux_to_count)
    assert list(K) == [1, 5, 51, 3, 120]
    for c, m in enumerate(starts):
        want = g.format_q(m.copy())
        assert np.array_equal(q[c, :want.size], want)
        assert not q[c, want.size:].any()
    q2, K2 = rj_native.pack_starts([q[c, :3 * K[c]] for c in range(5)], 120)
    assert np.array_equal(q2, q) and np.array_equal(K2, K)
    with pytest.raises(ValueError):
        rj_native.pack_starts([np.ones((2, 3))], 1)


def test_native_start_packing_array_form():
    """One [n, K, 3] start array packs as the list of its rows does (the
    multi-threaded native pass over 4,096 chains included)."""
    from rhmc_amd import rj_native, sampler
    g = sampler.multi_gym(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.)
    rs = np.random.RandomState(13)
    arr = np.stack([15 + 8.3 * rs.rand(4096, 51), 32 * rs.rand(4096, 51),
                    32 * rs.rand(4096, 51)], 2)
    q, K = rj_native.pack_starts(arr, 122, g.flux_to_count)
    q2, K2 = rj_native.pack_starts(list(arr), 122, g.flux_to_count)
    assert np.array_equal(q, q2) and np.array_equal(K, K2) and (K == 51).all()
    assert np.array_equal(q[7, :153], g.format_q(arr[7].copy()))
    with pytest.raises(ValueError):
        rj_native.pack_starts(arr, 50, g.flux_to_count)
    with pytest.raises(ValueError):
        rj_native.pack_starts(np.ones((2, 3, 2)), 10)
