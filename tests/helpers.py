"""Test helpers: golden parameter dicts -> C-ABI params, comparison utilities."""
import numpy as np


def vprior_const(par):
    """V_prior_const exactly as the reference caches it (sampler_RHMC.py:320-321)."""
    a = par["alpha"]
    if par.get("fmax", -1.0) <= 0:
        return 0.0
    return np.log(par["rows"] * par["cols"]) - np.log(
        (1 - a) / (par["fmax"] ** (1 - a) - par["fmin"] ** (1 - a)))


def capi_params(capi, par, delta=1e-6, counter_max=1000):
    return capi.make_params(
        dt=par["dt"], delta=delta, counter_max=counter_max, B_count=par["B_count"],
        f_lim=par["f_lim"], f_low=par["f_low"], fwhm_pix=par["fwhm_pix"], g_xx=par["g_xx"],
        g_ff=par["g_ff"], g_ff2=par["g_ff2"], g0=par["g0"], g1=par["g1"], g2=par["g2"],
        use_prior=par["use_prior"], alpha=par["alpha"], use_Vc=par["use_Vc"],
        beta=par["beta"], Vc_r_pow=par["Vc_r_pow"], V_prior_const=vprior_const(par))


def assert_state_close(got, want, rel, what=""):
    """|got - want| <= rel * (|want| + 1), elementwise."""
    got = np.asarray(got)
    want = np.asarray(want)
    err = np.abs(got - want) / (np.abs(want) + 1.0)
    bad = ~(err <= rel)
    if bad.any():
        idx = np.argwhere(bad)[:5]
        raise AssertionError("%s: %d elements off (max rel err %.3e > %.1e); first %s: got %s want %s"
                             % (what, bad.sum(), np.nanmax(err), rel, idx.tolist(),
                                got[tuple(idx[0])], want[tuple(idx[0])]))
