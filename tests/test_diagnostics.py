"""Post-processing (R-hat, n_eff, acceptance) against the reference's outputs."""
import numpy as np
import pytest

from conftest import load_golden


@pytest.mark.parametrize("name", ["iid", "ar", "ar_hi"])
def test_convergence_stats_match_reference(name):
    from rhmc_amd import diagnostics as Dg
    z = load_golden("solvers")
    k = "conv_" + name + "/"
    x = z[k + "x"]
    R, neff = Dg.convergence_stats(x, thin_rate=2, warm_up_num=10)
    np.testing.assert_allclose(R, z[k + "R"], rtol=1e-13)
    np.testing.assert_allclose(neff, z[k + "neff"], rtol=1e-13)
    R1, neff1 = Dg.convergence_stats(x, thin_rate=1, warm_up_num=0)
    np.testing.assert_allclose(R1, z[k + "R1"], rtol=1e-13)
    np.testing.assert_allclose(neff1, z[k + "neff1"], rtol=1e-13)
    chains = [x[0, :100], x[1, :100]]
    np.testing.assert_allclose([Dg.variogram(chains, 1, t) for t in (1, 2, 5)], z[k + "vg"],
                               rtol=1e-14)
    np.testing.assert_allclose(Dg.acceptance_rate(z[k + "dec"]), z[k + "acc"])
    np.testing.assert_allclose(Dg.acceptance_rate(z[k + "dec"], start=10, end=50), z[k + "acc2"])
