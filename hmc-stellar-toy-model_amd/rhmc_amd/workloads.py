"""Synthetic workloads of BASELINE.json's configs.

Every config is a data image plus a batch of chain states (q0, p0):
  C1  32x32,  K=1,  1 chain,        100 steps (reference CPU plumbing case)
  C2  48x48,  K=1,  4096 chains,    500 steps (headline, one MI355X)
  C3  48x48,  K=10, 16384 chains    (multi-source gradient)
  C4  48x48,  K=1,  2^20 chains     sharded over 8 GPUs
  C5  256x256, K=64, 8192 chains    (flux-wall RHMC, prior on)
Beyond BASELINE's configs, the reference's own many-star drivers (dense
32x32 images, big-sim4 parameters, prior on):
  B4  32x32, K=51,  4096 chains, 100 steps (RHMC-big-sim4.py: 32**2 * 0.05 true
      stars of magnitudes 15 .. 20, :20, :30-31)
  B3  32x32, K=100, 4096 chains, 100 steps (RHMC-big-sim3.py: Nobjs = 100 of
      magnitudes 15 .. 20.5, :18, :28-29)
  C5R C5's geometry (256x256, K=64, 8192 chains, prior) with the true stars
      drawn over the reference drivers' magnitude range 15 .. 20
      (RHMC-big-sim4.py:30-31), all above the flux wall: the MH line with
      run_RHMC's f_pos=True (with C5's own stars, down to mag 23.3, the
      posterior sits on the wall and almost every proposal has V = inf)
  S<n>K<k>  n x n, K=k, 4096 chains, 100 steps, the same parameters (kernel
            sweeps, e.g. S48K32)

Randomness: numpy legacy RandomState; the image uses seed 77
(RHMC-big-sim4.py:18), chain initial states seed 1000 (+ shard offset).

MH starts (`mh_start`): C3 and C5 draw magnitudes down to 23.3, below the flux wall at mag 23 (f_lim, sampler_RHMC.py:194-196), so with
run_RHMC's f_pos=True every such start has V = inf (sampler_RHMC.py:303-309)
and every proposal is rejected before any pixel work.  For MH the chains
start near the truth (flux x lognormal 2 %, positions +- 0.1 px; seed 2000 +
shard offset) with every flux raised to at least `floor` f_lim (1.5: mag
22.56).  The leapfrog benches keep the plain starts (truth x lognormal 10 %,
0.5 px: the flux-wall reflections are part of C3/C5).
"""
import re

import numpy as np

from .photometry import (default_exp_setup, factors, gauss_PSF, gen_pow_law_sample,
                         mag2flux, metric_diag, poisson_realization)


class Workload:
    def __init__(self, name, D, q0, p0, params, n_steps, K, note, truth=None):
        self.name = name
        self.D = D
        self.q0 = q0
        self.p0 = p0
        self.params = params        # dict for capi.make_params
        self.n_steps = n_steps
        self.K = K
        self.note = note
        self.truth = truth          # multi-star: the image's (f, x, y) per star, counts

    @property
    def n_chains(self):
        return self.q0.shape[0]


def base_params(dt, g_xx=1., g_ff=1., g_ff2=1., use_prior=False, alpha=2.):
    """Instance constants of multi_gym(g_xx, g_ff, g_ff2) with the factors
    computed once on the default 48x48 grid (sampler_RHMC.py:50, :165)."""
    rows, cols, ftc, fwhm, B, _, mB, f_lim = default_exp_setup()
    g0, g1, g2 = factors(rows, cols, rows / 2., cols / 2., fwhm)
    return dict(dt=dt, delta=1e-6, counter_max=1000, B_count=B, f_lim=f_lim,
                f_low=mag2flux(mB + 2) * ftc, fwhm_pix=fwhm, g_xx=g_xx, g_ff=g_ff,
                g_ff2=g_ff2, g0=g0, g1=g1, g2=g2, use_prior=use_prior, alpha=alpha,
                use_Vc=False, beta=1., Vc_r_pow=1., V_prior_const=0.), ftc


def _image(n, stars, ftc, B, fwhm, rng):
    D0 = np.ones((n, n)) * B
    for mag, x, y in stars:
        D0 += mag2flux(mag) * ftc * gauss_PSF(n, n, x, y, FWHM=fwhm)
    return poisson_realization(D0, rng)


def _powlaw_stars(rng, K, n, ftc, mag_lo=15., mag_hi=23.3, alpha=2.):
    fmin = mag2flux(mag_hi) * ftc
    fmax = mag2flux(mag_lo) * ftc
    f = gen_pow_law_sample(alpha, fmin, fmax, K, rng)
    x = rng.random_sample(K) * (n - 2.) + 1.
    y = rng.random_sample(K) * (n - 2.) + 1.
    return f, x, y


def mh_start(wl, floor=1.5, seed_offset=0):
    """The workload's chain starts for run_RHMC's MH loop with f_pos=True:
    multi-star workloads near the truth (flux x lognormal 2 %, 0.1 px), every
    flux raised to >= floor * f_lim; one-star workloads keep q0 (mag 19, far
    above the wall) with the same floor."""
    if wl.truth is None:
        q = wl.q0.copy()
    else:
        ft, xt, yt = wl.truth
        rng = np.random.RandomState(2000 + seed_offset)
        n = wl.n_chains
        q = np.empty_like(wl.q0)
        q[:, 0::3] = ft * np.exp(0.02 * rng.randn(n, wl.K))
        q[:, 1::3] = xt + 0.1 * rng.randn(n, wl.K)
        q[:, 2::3] = yt + 0.1 * rng.randn(n, wl.K)
    q[:, 0::3] = np.maximum(q[:, 0::3], floor * wl.params["f_lim"])
    return q


def make(name, n_chains=None, seed_offset=0):
    name = name.upper()
    img_rng = np.random.RandomState(77)
    rng = np.random.RandomState(1000 + seed_offset)
    truth = None
    if name in ("C1", "C2", "C4"):
        n = 32 if name == "C1" else 48
        par, ftc = base_params(dt=0.1)
        f = mag2flux(19.) * ftc
        if name == "C1":
            xt, yt = 16.2, 15.7
        else:
            xt, yt = 24. + img_rng.uniform(-.5, .5), 24. + img_rng.uniform(-.5, .5)
        D = _image(n, [(19., xt, yt)], ftc, par["B_count"], par["fwhm_pix"], img_rng)
        nc = {"C1": 1, "C2": 4096, "C4": 1 << 20}[name] if n_chains is None else n_chains
        if name == "C1":
            q0 = np.array([[f, xt + 0.3, yt]]).repeat(nc, 0)
        else:
            q0 = np.stack([f * (1 + 0.1 * rng.randn(nc)), xt + 0.5 * rng.randn(nc),
                           yt + 0.5 * rng.randn(nc)], 1)
        K = 1
        steps = 100 if name == "C1" else 500
    elif name in ("C3", "C5", "C5R", "B3", "B4") or re.fullmatch(r"S\d+K\d+", name):
        if name[0] == "S":
            n, K = (int(v) for v in re.fullmatch(r"S(\d+)K(\d+)", name).groups())
        else:
            n, K = {"C3": (48, 10), "C5": (256, 64), "C5R": (256, 64), "B3": (32, 100),
                    "B4": (32, 51)}[name]
        par, ftc = base_params(dt=0.05, g_xx=0.05, g_ff=4., g_ff2=4.,
                               use_prior=(name != "C3"), alpha=2.)
        if par["use_prior"]:
            # V's prior constant for the power-law flux range (sampler_RHMC.py:321)
            a = par["alpha"]
            fmin, fmax = mag2flux(23.3) * ftc, mag2flux(15.) * ftc
            par["V_prior_const"] = np.log(n * n) - np.log(
                (1 - a) / (fmax ** (1 - a) - fmin ** (1 - a)))
        # true magnitudes: down to 23.3 for BASELINE's C3 / C5 (below the flux
        # wall at 23); the reference drivers' ranges for B4 / B3
        mag_hi = {"B4": 20., "B3": 20.5, "C5R": 20.}.get(name, 23.3)
        ft, xt, yt = _powlaw_stars(img_rng, K, n, ftc, mag_hi=mag_hi)
        D = _image(n, [(22.5 - 2.5 * np.log10(a / ftc), b, c) for a, b, c in zip(ft, xt, yt)],
                   ftc, par["B_count"], par["fwhm_pix"], img_rng)
        nc = ({"C3": 16384, "C5": 8192, "C5R": 8192}.get(name, 4096)) if n_chains is None else n_chains
        # chains start at the truth, perturbed (flux x lognormal 10%, 0.5 px)
        q0 = np.empty((nc, 3 * K))
        q0[:, 0::3] = ft * np.exp(0.1 * rng.randn(nc, K))
        q0[:, 1::3] = xt + 0.5 * rng.randn(nc, K)
        q0[:, 2::3] = yt + 0.5 * rng.randn(nc, K)
        steps = 500 if name[0] == "C" else 100
        truth = (ft, xt, yt)
    else:
        raise ValueError("unknown workload " + name)
    H = metric_diag(q0, par)
    p0 = rng.randn(*q0.shape) * np.sqrt(H)
    note = "%s: %dx%d image, K=%d, %d chains, %d steps" % (name, n, n, K, nc, steps)
    return Workload(name, D, q0, p0, par, steps, K, note,
                    truth=truth if K > 1 or name[0] != "C" else None)
