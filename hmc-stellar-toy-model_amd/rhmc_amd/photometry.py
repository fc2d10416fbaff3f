"""Host-side photometry helpers (input generation and constants).

These build the inputs of the hot path — the data image, the metric factors
g0/g1/g2 and the default experimental constants — the way the reference does
(utils.py / sampler_RHMC.py).  None of them is on the per-step path; the
step itself only runs in librhmc.so.
"""
import numpy as np


def mag2flux(mag):
    """utils.py:24-25"""
    return 10 ** (0.4 * (22.5 - mag))


def flux2mag(flux):
    """utils.py:27-28"""
    return 22.5 - 2.5 * np.log10(flux)


def gauss_PSF(num_rows, num_cols, x, y, FWHM):
    """utils.py:475-486 (returns (num_cols, num_rows); square images only)."""
    sigma = FWHM / 2.354
    xv = np.arange(0.5, num_rows)
    yv = np.arange(0.5, num_cols)
    yv, xv = np.meshgrid(xv, yv)
    return np.exp(-(np.square(xv - x) + np.square(yv - y)) / (2 * sigma ** 2)) \
        / (np.pi * 2 * sigma ** 2)


def poisson_realization(D0, rng=np.random):
    """utils.py:488-496.  The reference draws pixel by pixel in row-major
    order; the vectorized draw consumes the legacy stream identically
    (measured)."""
    return rng.poisson(D0).astype(np.float64)


def gen_pow_law_sample(alpha, fmin, fmax, Nsample=1, rng=np.random):
    """utils.py:460-471 — inverse-CDF draw from f**-alpha on [fmin, fmax]."""
    assert alpha > 1
    alpha = float(alpha)
    u = rng.random_sample(size=Nsample)
    lmbda = fmin ** (1 - alpha) + u * (fmax ** (1 - alpha) - fmin ** (1 - alpha))
    return np.exp(np.log(lmbda) / (1 - alpha))


def factors(num_rows, num_cols, x, y, PSF_FWHM_pix):
    """utils.py:623-644 -> (g0, g1, g2), the metric's PSF moments."""
    lv = np.arange(0, num_rows)
    mv = np.arange(0, num_cols)
    mv, lv = np.meshgrid(lv, mv)
    var = (PSF_FWHM_pix / 2.354) ** 2
    PSF = gauss_PSF(num_rows, num_cols, x, y, FWHM=PSF_FWHM_pix)
    PSF_sq = np.square(PSF)
    factor0 = np.sum(PSF_sq)
    factor1 = np.sum(PSF * (x - lv - 0.5) ** 2) / float(var ** 2)
    factor2 = np.sum(PSF_sq * (x - lv - 0.5) ** 2) / float(var ** 2)
    return factor0, factor1, factor2


def default_exp_setup():
    """sampler_RHMC.py:169-201: (num_rows, num_cols, flux_to_count,
    PSF_FWHM_pix, B_count, arcsec_to_pix, mB, f_lim)."""
    arcsec_to_pix = 0.4
    PSF_FWHM_pix = 1.4 / arcsec_to_pix
    gain = 4.62
    ADU_to_flux = 0.00546689
    flux_to_count = 1. / (ADU_to_flux * gain)
    mB = 23
    B_count = mag2flux(mB) * flux_to_count
    f_lim = mag2flux(mB) * flux_to_count
    return 48, 48, flux_to_count, PSF_FWHM_pix, B_count, arcsec_to_pix, mB, f_lim


def metric_diag(q, c):
    """Vectorized H(q) (sampler_RHMC.py:229-258, grad=False) for momentum
    draws on the host: q [..., 3K] -> H [..., 3K].  `c` holds g_xx, g_ff,
    g_ff2, g0, g1, g2, B_count, f_low."""
    q = np.asarray(q, dtype=np.float64)
    f = q[..., 0::3]
    Hff = 1. / (f / c["g_ff2"] + (c["B_count"] / c["g0"]) / c["g_ff"])
    fl = np.where(f < c["f_low"], c["f_low"], f)
    Hxx = c["g_xx"] * (1. / (c["g1"] * fl) + c["B_count"] / (c["g2"] * fl ** 2)) ** -1
    H = np.empty_like(q)
    H[..., 0::3] = Hff
    H[..., 1::3] = Hxx
    H[..., 2::3] = Hxx
    return H
