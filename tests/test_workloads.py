"""Host-side workload generation (CPU)."""
import numpy as np

from conftest import load_golden
from oracle import rhmc_ref as R


def test_base_params_match_reference_constants():
    from rhmc_amd import workloads
    par, ftc = workloads.base_params(dt=0.1)
    z = load_golden("functions")
    ref = R.params_from_npz(z, "k1/par_")
    for k in ("B_count", "f_lim", "f_low", "fwhm_pix", "g0", "g1", "g2"):
        assert par[k] == ref[k], k
    assert ftc == ref["flux_to_count"]


def test_c1_c2_shapes_and_momenta():
    from rhmc_amd import workloads
    from rhmc_amd.photometry import metric_diag
    w = workloads.make("C2", n_chains=64)
    assert w.D.shape == (48, 48) and w.q0.shape == (64, 3) and w.K == 1
    assert np.all(w.D == np.round(w.D)) and w.D.min() >= 0
    H = metric_diag(w.q0, w.params)
    m = R.RefModel(w.D, dict(w.params, rows=48, cols=48))
    for c in range(5):
        np.testing.assert_allclose(H[c], m.H(w.q0[c]), rtol=1e-15)
    w1 = workloads.make("C1")
    assert w1.q0.shape == (1, 3) and w1.D.shape == (32, 32) and w1.n_steps == 100


def test_c3_c5_shapes():
    from rhmc_amd import workloads
    w = workloads.make("C3", n_chains=8)
    assert w.q0.shape == (8, 30) and w.D.shape == (48, 48)
    w = workloads.make("C5", n_chains=2)
    assert w.q0.shape == (2, 192) and w.D.shape == (256, 256) and w.params["use_prior"]
