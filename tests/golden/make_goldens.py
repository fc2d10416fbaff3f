#!/usr/bin/env python3
"""Generate golden fixtures from the REFERENCE implementation (build container only).

This script is test infrastructure.  It never runs on the GPU box and it never
vendors reference source: at run time it converts the reference's Python-2
modules (`sampler_RHMC.py`, `utils.py`, `samplers.py` under /root/reference)
with the standard-library `lib2to3` into a temporary directory OUTSIDE the
repository, applies the two NumPy-2 shims the reference needs (`np.infty`,
`np.product`, see SURVEY.md §4 bit-rot items 3), imports it, runs the cases
below and writes small `.npz` fixtures next to this file.  Only inputs and
outputs (data) are committed.

Fixed-point iteration counts are not returned by the reference; they are
recovered by counting calls to the instance's `dtaudq` / `dtaudp` inside one
`RHMC_single_step` (sampler_RHMC.py:522-566): the p-loop calls `dtaudq` once
per iteration and once more after the q-loop (:532, :548); the q-loop calls
`dtaudp` twice per iteration (:542).

Usage:  python tests/golden/make_goldens.py [--ref /root/reference]
"""
import argparse
import contextlib
import io
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load_reference(ref_dir):
    tmp = tempfile.mkdtemp(prefix="rhmc_ref_py3_")
    for name in ("sampler_RHMC.py", "utils.py", "samplers.py"):
        shutil.copy(os.path.join(ref_dir, name), tmp)
    subprocess.run([sys.executable, "-m", "lib2to3", "-n", "-w",
                    "sampler_RHMC.py", "utils.py", "samplers.py"],
                   cwd=tmp, check=True, stdout=subprocess.DEVNULL,
                   stderr=subprocess.DEVNULL)
    # lib2to3 has no division fixer: restore Python 2's integer `/` at the one
    # place it matters for the code exercised here (utils.py:111,
    # convergence_stats `n = L_chain/2`, an int/int division in Python 2).
    up = os.path.join(tmp, "utils.py")
    src = open(up).read()
    assert src.count("n = L_chain/2") == 1
    open(up, "w").write(src.replace("n = L_chain/2", "n = L_chain//2"))
    np.infty = np.inf          # removed in NumPy 2 (sampler_RHMC.py:312,317,529)
    np.product = np.prod       # removed in NumPy 2 (samplers.py:911)
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, tmp)
    import sampler_RHMC  # noqa: E402
    import utils         # noqa: E402
    import samplers      # noqa: E402
    return sampler_RHMC, utils, samplers, tmp


class Counter:
    """Wrap a gym's dtaudq/dtaudp to count calls (fixed-point iterations)."""

    def __init__(self, gym):
        self.gym = gym
        self.n_tq = 0
        self.n_tp = 0
        orig_q, orig_p = gym.dtaudq, gym.dtaudp

        def dtaudq(q, p):
            self.n_tq += 1
            return orig_q(q, p)

        def dtaudp(q, p):
            self.n_tp += 1
            return orig_p(q, p)

        gym.dtaudq = dtaudq
        gym.dtaudp = dtaudp

    def step(self, q, p, delta, cmax):
        self.n_tq = self.n_tp = 0
        q1, p1 = self.gym.RHMC_single_step(q, p, delta=delta, counter_max=cmax)
        return q1, p1, self.n_tq - 1, self.n_tp // 2


def gym_params(g):
    """Every instance attribute the hot path reads."""
    f_low = g.mag2flux_converter(g.mB + 2)
    return dict(
        rows=g.num_rows, cols=g.num_cols, dt=g.dt, B_count=g.B_count,
        f_lim=g.f_lim, f_low=f_low, fwhm_pix=g.PSF_FWHM_pix, g_xx=g.g_xx,
        g_ff=g.g_ff, g_ff2=g.g_ff2, g0=g.g0, g1=g.g1, g2=g.g2,
        use_prior=int(bool(g.use_prior)), alpha=g.alpha,
        use_Vc=int(bool(g.use_Vc)), beta=g.beta, Vc_r_pow=g.Vc_r_pow,
        fmin=-1.0 if getattr(g, "fmin", None) is None else g.fmin,
        fmax=-1.0 if getattr(g, "fmax", None) is None else g.fmax,
        flux_to_count=g.flux_to_count, mB=g.mB)


def pack(prefix, d):
    return {prefix + k: np.asarray(v) for k, v in d.items()}


def make_gym(S, cls="multi", n=48, g_xx=1., g_ff=1., g_ff2=1., dt=0.1,
             prior=False, alpha=2., fminmax=(20., 15.)):
    g = (S.multi_gym if cls == "multi" else S.single_gym)(
        dt=0., Nsteps=0, g_xx=g_xx, g_ff=g_ff, g_ff2=g_ff2)
    g.num_rows = g.num_cols = n          # factors g0..g2 stay at 48x48 (quirk)
    g.dt = dt
    g.fmin = g.mag2flux_converter(fminmax[0])
    g.fmax = g.mag2flux_converter(fminmax[1])
    if prior:
        g.use_prior = True
        g.alpha = alpha
    return g


def stars_to_q(g, stars):
    """(K,3) mag,x,y -> flat f,x,y in counts (format_q, sampler_RHMC.py:209)."""
    q = np.array(stars, dtype=float).copy()
    return g.format_q(q)


def trajectory(g, q, p, nsteps, delta=1e-6, cmax=1000):
    c = Counter(g)
    Q = [q.copy()]
    P = [p.copy()]
    NP, NQ = [], []
    for _ in range(nsteps):
        q, p, a, b = c.step(q, p, delta, cmax)
        Q.append(q.copy())
        P.append(p.copy())
        NP.append(a)
        NQ.append(b)
    return np.array(Q), np.array(P), np.array(NP, np.int32), np.array(NQ, np.int32)


# ----------------------------------------------------------------------------
# Case 1: per-function vectors (gauss_PSF, dVdq, H, dphidq, dtaudq, dtaudp, V, T)
# ----------------------------------------------------------------------------
def case_functions(S, U):
    out = {}
    rs = np.random.RandomState(5)
    # gauss_PSF (utils.py:475-486): square and rectangular (shape quirk)
    psf_args = [(48, 48, 24.3, 23.8), (32, 32, 0.2, 31.7), (16, 16, 8.0, 8.0),
                (4, 6, 1.3, 2.2)]
    for i, (r, c, x, y) in enumerate(psf_args):
        out["psf%d_args" % i] = np.array([r, c, x, y, 1.4 / 0.4])
        out["psf%d" % i] = U.gauss_PSF(r, c, x, y, FWHM=1.4 / 0.4)

    # factors (utils.py:623-644) at a few grids
    out["factors_args"] = np.array([[48, 48, 24., 24.], [32, 32, 16., 16.],
                                    [64, 64, 32.3, 31.6]])
    out["factors"] = np.array([U.factors(int(a), int(b), x, y, 1.4 / 0.4)
                               for a, b, x, y in out["factors_args"]])

    sets = [
        # name, n, stars(true), gym kwargs, K_model
        ("k1", 48, [[19., 24.3, 23.8]], dict(), 1),
        ("k1gff2", 48, [[20., 24.3, 23.8]], dict(g_ff2=2.), 1),
        ("k10", 48, None, dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05,
                                prior=True), 10),
        ("vc5", 32, None, dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05), 5),
    ]
    for name, n, stars, kw, K in sets:
        np.random.seed(77)
        g = make_gym(S, n=n, **kw)
        if stars is None:
            fmin = g.mag2flux_converter(23.)
            fmax = g.mag2flux_converter(15.)
            mags = g.flux2mag_converter(U.gen_pow_law_sample(2., fmin, fmax, K))
            xs = np.random.random(K) * (n - 2.) + 1.
            ys = np.random.random(K) * (n - 2.) + 1.
            stars = np.stack([mags, xs, ys], 1)
        if name == "vc5":
            g.use_Vc = True
            g.beta = 1e-2
            g.f_expnt = np.zeros(K)
            g.Vc_r_pow = 2.
        g.gen_mock_data(np.array(stars))
        g.Nobjs = K
        g.d = 3 * K
        q_true = stars_to_q(g, stars)
        qs, ps = [], []
        for t in range(6):
            q = q_true.copy()
            q[0::3] *= np.exp(0.2 * rs.randn(K))
            q[1::3] += 0.7 * rs.randn(K)
            q[2::3] += 0.7 * rs.randn(K)
            if t == 5:      # one flux below f_low (H_xx clamp branch, :269-276)
                q[0] = 0.5 * g.mag2flux_converter(g.mB + 2)
            qs.append(q)
            ps.append(rs.randn(3 * K) * np.sqrt(np.abs(g.H(q))))
        qs, ps = np.array(qs), np.array(ps)
        res = dict(D=g.D, q=qs, p=ps)
        res["dVdq"] = np.array([g.dVdq(q) for q in qs])
        res["H"] = np.array([g.H(q) for q in qs])
        hg = [g.H(q, grad=True) for q in qs]
        res["Hv"] = np.array([h[0] for h in hg])
        res["Hg"] = np.array([h[1] for h in hg])
        res["dphidq"] = np.array([g.dphidq(q) for q in qs])
        res["dtaudq"] = np.array([g.dtaudq(q, p) for q, p in zip(qs, ps)])
        res["dtaudp"] = np.array([g.dtaudp(q, p) for q, p in zip(qs, ps)])
        res["V"] = np.array([g.V(q, f_pos=False) for q in qs])
        res["Vpos"] = np.array([g.V(q, f_pos=True) for q in qs])
        res["T"] = np.array([g.T(p, g.H(q)) for q, p in zip(qs, ps)])
        params = gym_params(g)
        if g.use_Vc:
            params["f_expnt_present"] = 1
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", params))
    return out


# ----------------------------------------------------------------------------
# Case 2: single steps incl. flux-wall and edge reflections
# ----------------------------------------------------------------------------
def case_steps(S, U):
    np.random.seed(77)
    g = make_gym(S, n=48)
    g.gen_mock_data(np.array([[19., 24.3, 23.8]]))
    g.Nobjs, g.d = 1, 3
    c = Counter(g)
    rs = np.random.RandomState(11)
    f19 = g.mag2flux_converter(19.)
    Q0, P0, Q1, P1, NP, NQ = [], [], [], [], [], []
    for t in range(48):
        q = np.array([f19 * np.exp(0.3 * rs.randn()), 24.3 + rs.randn(),
                      23.8 + rs.randn()])
        if t % 8 == 1:      # flux just above the wall, moving down
            q[0] = g.f_lim * (1 + 1e-3 * rs.rand())
        if t % 8 == 2:      # near the x edge
            q[1] = 0.02 * rs.rand()
        if t % 8 == 3:      # near the far y edge
            q[2] = g.num_cols - 1 - 0.02 * rs.rand()
        if t % 8 == 4:      # flux under f_low: H_xx clamp (:269)
            q[0] = 3.0
        p = rs.randn(3) * np.sqrt(g.H(q))
        if t % 8 == 1:
            p[0] = -abs(p[0]) * 50
        if t % 8 == 2:
            p[1] = -abs(p[1]) * 5
        if t % 8 == 3:
            p[2] = abs(p[2]) * 5
        q1, p1, a, b = c.step(q, p, 1e-6, 1000)
        Q0.append(q); P0.append(p); Q1.append(q1); P1.append(p1)
        NP.append(a); NQ.append(b)
    res = dict(D=g.D, q0=np.array(Q0), p0=np.array(P0), q1=np.array(Q1),
               p1=np.array(P1), n_p=np.array(NP, np.int32),
               n_q=np.array(NQ, np.int32))
    out = pack("", res)
    out.update(pack("par_", gym_params(g)))
    return out


# ----------------------------------------------------------------------------
# Case 3: trajectories (configs C1, C2-geometry, C3-geometry, C5-geometry, ...)
# ----------------------------------------------------------------------------
def traj_case(S, U, n, stars_true, model_fn, kw, nchains, nsteps, seed=77,
              vc=None, cmax=1000, delta=1e-6, p_mod=None):
    np.random.seed(seed)
    g = make_gym(S, n=n, **kw)
    if callable(stars_true):
        stars_true = stars_true(g)
    if vc is not None:
        g.use_Vc = True
        g.beta, g.Vc_r_pow = vc
    g.gen_mock_data(np.array(stars_true, dtype=float))
    Qs, Ps, NPs, NQs = [], [], [], []
    for c in range(nchains):
        stars = model_fn(g, c)
        K = len(stars)
        g.Nobjs, g.d = K, 3 * K
        if vc is not None:
            g.f_expnt = np.zeros(K)
        q0 = stars_to_q(g, stars)
        p0 = np.random.randn(3 * K) * np.sqrt(g.H(q0))
        if p_mod is not None:
            p0 = p_mod(g, c, p0)
        Q, P, NP, NQ = trajectory(g, q0, p0, nsteps, delta, cmax)
        Qs.append(Q); Ps.append(P); NPs.append(NP); NQs.append(NQ)
    res = dict(D=g.D, Q=np.array(Qs), P=np.array(Ps), n_p=np.array(NPs),
               n_q=np.array(NQs), delta=delta, counter_max=cmax)
    out = pack("", res)
    out.update(pack("par_", gym_params(g)))
    return out


def powlaw_stars(U, g, K, n, mag_lo=15., mag_hi=23.3, alpha=2.):
    fmin = g.mag2flux_converter(mag_hi)
    fmax = g.mag2flux_converter(mag_lo)
    mags = g.flux2mag_converter(U.gen_pow_law_sample(alpha, fmin, fmax, K))
    xs = np.random.random(K) * (n - 2.) + 1.
    ys = np.random.random(K) * (n - 2.) + 1.
    return np.stack([mags, xs, ys], 1)


def case_trajs(S, U):
    cases = {}
    # C1: 32x32, K=1, mag 19 at (16.2, 15.7), init x+0.3, 100 steps, 1 chain
    cases["traj_c1"] = traj_case(
        S, U, 32, [[19., 16.2, 15.7]], lambda g, c: [[19., 16.5, 15.7]],
        dict(), 1, 100)
    # C2 geometry: 48x48 K=1 mag 19, 8 chains x 500 steps
    rs = np.random.RandomState(1000)
    jit = rs.randn(8, 3)
    cases["traj_c2"] = traj_case(
        S, U, 48, [[19., 24.21, 23.86]],
        lambda g, c: [[19. - 2.5 * np.log10(1 + 0.1 * jit[c, 0]),
                       24.21 + 0.5 * jit[c, 1], 23.86 + 0.5 * jit[c, 2]]],
        dict(), 8, 500)
    # g_ff2 != 1 (H_ff grad quirk, :292), base_class default g_ff2=2
    cases["traj_gff2"] = traj_case(
        S, U, 48, [[20., 24.21, 23.86]],
        lambda g, c: [[20.2, 24.0 + 0.3 * c, 23.9]], dict(g_ff2=2.), 2, 200)
    # C3 geometry: 48x48 K=10 big-sim4 parameters + flux wall reflections
    cases["traj_c3"] = traj_case(
        S, U, 48, lambda g: powlaw_stars(U, g, 10, 48),
        lambda g, c: powlaw_stars(U, g, 10, 48),
        dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05), 2, 300)
    # prior on (use_prior, :408-409)
    cases["traj_prior"] = traj_case(
        S, U, 32, lambda g: powlaw_stars(U, g, 3, 32),
        lambda g, c: powlaw_stars(U, g, 3, 32),
        dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True), 2, 200)
    # repulsion on (use_Vc, :411-418)
    cases["traj_vc"] = traj_case(
        S, U, 32, lambda g: powlaw_stars(U, g, 5, 32),
        lambda g, c: powlaw_stars(U, g, 5, 32),
        dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05), 2, 100, vc=(1e-2, 2.))
    # edge: star drifting through the x=0 boundary
    cases["traj_edge"] = traj_case(
        S, U, 32, [[17., 0.6, 16.]], lambda g, c: [[17.2, 0.3 + 0.2 * c, 16.1]],
        dict(dt=0.2), 2, 200,
        p_mod=lambda g, c, p: p * np.array([1., 0., 1.]) + np.array(
            [0., -(40. + 20. * c), 0.]) * np.sqrt(g.H(p * 0 + np.array(
                [g.mag2flux_converter(17.2), 0., 0.]))))
    # small counter_max (loop cut off) and looser delta
    cases["traj_cmax"] = traj_case(
        S, U, 48, [[16., 24.2, 23.9]], lambda g, c: [[16.5, 24.6, 23.3]],
        dict(dt=0.3), 2, 100, cmax=2, delta=1e-9)
    cases.update(case_c5(S, U))
    return cases


def case_c5(S, U):
    """C5 geometry (256x256, K = 64, prior, big-sim4 parameters,
    RHMC-big-sim4.py:11-47): 4 chains x 50 reference steps.  Power-law
    magnitudes reach 23.3, below the flux wall (f_lim = mag 23), so every
    chain's flux-wall reflection (sampler_RHMC.py:554-559) fires within these
    steps; the generator checks that it does."""
    out = traj_case(
        S, U, 256, lambda g: powlaw_stars(U, g, 64, 256),
        lambda g, c: powlaw_stars(U, g, 64, 256),
        dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True), 4, 50)
    f_lim = out["par_f_lim"]
    refl = (out["Q"][:, 1:, 0::3] < f_lim).any(axis=(1, 2))
    assert refl.all(), "a C5 chain never reflected at the flux wall: %s" % refl
    return {"traj_c5": out}


def case_bigk(S, U):
    """K > 64 stars per chain, the reference's own many-star drivers:
    RHMC-big-sim3.py (32x32, K = 100, prior, repulsion) and RHMC-big-sim4.py
    (32x32, big-sim4 parameters, births up to N_max = 120, :77).  The
    reference's dVdq / V / RHMC_single_step are vectorised over any K
    (sampler_RHMC.py:365-425, :294-351, :522-566).

    bigk.npz: per-function vectors (dVdq, dphidq, V, T, H) at K = 100 (32 px,
    big-sim4 parameters + prior; and + repulsion Vc_r_pow = 4 as in big-sim3),
    K = 120 (48 px) and K = 128 (256 px, prior).
    traj_bigk.npz: 2 chains x 50 steps at 32x32, K = 100 (big-sim4
    parameters, prior).  traj_bigk256.npz: 1 chain x 4 steps at 256x256,
    K = 128, prior."""
    out = {}
    rs = np.random.RandomState(8)
    sets = [("b100", 32, 100, None), ("b100vc", 32, 100, (1e-3, 4.)), ("b120", 48, 120, None),
            ("b128", 256, 128, None)]
    for name, n, K, vc in sets:
        np.random.seed(77)
        g = make_gym(S, n=n, g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True)
        stars = powlaw_stars(U, g, K, n)
        if vc is not None:
            g.use_Vc = True
            g.beta, g.Vc_r_pow = vc
            g.f_expnt = np.zeros(K)
        g.gen_mock_data(np.array(stars))
        g.Nobjs, g.d = K, 3 * K
        q_true = stars_to_q(g, stars)
        qs, ps = [], []
        for t in range(4):
            q = q_true.copy()
            q[0::3] *= np.exp(0.2 * rs.randn(K))
            q[1::3] += 0.5 * rs.randn(K)
            q[2::3] += 0.5 * rs.randn(K)
            qs.append(q)
            ps.append(rs.randn(3 * K) * np.sqrt(np.abs(g.H(q))))
        qs, ps = np.array(qs), np.array(ps)
        res = dict(D=g.D, q=qs, p=ps)
        res["dVdq"] = np.array([g.dVdq(q) for q in qs])
        res["H"] = np.array([g.H(q) for q in qs])
        res["dphidq"] = np.array([g.dphidq(q) for q in qs])
        res["V"] = np.array([g.V(q, f_pos=False) for q in qs])
        res["Vpos"] = np.array([g.V(q, f_pos=True) for q in qs])
        res["T"] = np.array([g.T(p, g.H(q)) for q, p in zip(qs, ps)])
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))
        print("bigk", name, "done")
    cases = {"bigk": out}
    big = dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True)
    cases["traj_bigk"] = traj_case(
        S, U, 32, lambda g: powlaw_stars(U, g, 100, 32),
        lambda g, c: powlaw_stars(U, g, 100, 32), big, 2, 50)
    cases["traj_bigk256"] = traj_case(
        S, U, 256, lambda g: powlaw_stars(U, g, 128, 256),
        lambda g, c: powlaw_stars(U, g, 128, 256), big, 1, 4)
    return cases


# ----------------------------------------------------------------------------
# Case 4: full MH loop (multi_gym.run_RHMC move-0 branch) and single_gym trace
# ----------------------------------------------------------------------------
def case_mh(S, U):
    out = {}
    for name, n, stars_t, stars_m, kw, niter, nsteps, dt in [
        ("mh1", 32, [[19., 16.2, 15.7]], [[19.5, 16.6, 15.2]], dict(), 30, 10,
         0.1),
        ("mh3", 32, [[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4], [19.6, 15.3, 24.6]],
         dict(g_xx=0.05, g_ff=4., g_ff2=4., prior=True), 20, 10, 0.05),
    ]:
        np.random.seed(77)
        g = make_gym(S, n=n, **kw)
        g.gen_mock_data(np.array(stars_t))
        np.random.seed(123)
        with contextlib.redirect_stdout(io.StringIO()):
            g.run_RHMC(np.array(stars_m), f_pos=True, delta=1e-6, Niter=niter,
                       Nsteps=nsteps, dt=dt, N_max=len(stars_m))
        res = dict(D=g.D, q_model=np.array(stars_m), q_chain=g.q_chain,
                   p_chain=g.p_chain, E_chain=g.E_chain, V_chain=g.V_chain,
                   T_chain=g.T_chain, A_chain=g.A_chain.astype(np.int32),
                   niter=niter, nsteps=nsteps, seed=123, dt=dt)
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))

    # single_gym.run_single_RHMC(solver="implicit") energy trace (:649-783)
    np.random.seed(77)
    g = S.single_gym(dt=0., Nsteps=0, g_xx=1., g_ff=1.)
    g.num_rows = g.num_cols = 16
    g.fmin = g.mag2flux_converter(20.)   # V needs fmin/fmax (:320-321)
    g.fmax = g.mag2flux_converter(15.)
    g.gen_mock_data(np.array([[19., 8., 8.]]))
    g.Nsteps, g.dt = 100, 0.1
    np.random.seed(5)
    g.run_single_RHMC(q_model_0=np.array([[19., 9., 8.]]), f_pos=True,
                      solver="implicit", delta=1e-6)
    res = dict(D=g.D, q_chain=g.q_chain, p_chain=g.p_chain, E_chain=g.E_chain,
               V_chain=g.V_chain, T_chain=g.T_chain)
    out.update(pack("single/", res))
    out.update(pack("single/par_", gym_params(g)))
    return out


def case_mh_sched(S, U):
    """multi_gym.run_RHMC with parameter schedules (sampler_RHMC.py:1010-1016):
    iteration l sets g_ff2 = schedule_g_ff2[l] / beta = schedule_beta[l]
    while l < the schedule's size, then keeps the last value — as in
    RHMC-big-sim3.py (gff2_list = scheduler(1/5.**2, 4., 1000), beta_list =
    scheduler(1e-5, 1e-7, 1000), utils.py:649-660).  The schedules here are
    shorter than Niter + 1 so that the hold-the-last-value rule is exercised."""
    out = {}
    for name, stars_t, stars_m, kw, niter, nsteps, dt, vc in [
        ("g1", [[19., 16.2, 15.7]], [[19.5, 16.6, 15.2]], dict(), 20, 10, 0.05, False),
        ("g3", [[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4], [19.6, 15.3, 24.6]],
         dict(g_xx=0.05, g_ff=4., g_ff2=4., prior=True), 20, 10, 0.01, False),
        ("g3vc", [[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4], [19.6, 15.3, 24.6]],
         dict(g_xx=0.05, g_ff=4., g_ff2=4., prior=True), 20, 10, 0.01, True),
    ]:
        np.random.seed(77)
        g = make_gym(S, n=32, **kw)
        g.gen_mock_data(np.array(stars_t))
        sg = U.scheduler(1 / 5. ** 2, 4., 15)
        sb = None
        if vc:
            g.use_Vc = True
            g.beta = 1.
            g.Vc_r_pow = 4.
            g.f_expnt = np.zeros(len(stars_m))
            sb = U.scheduler(1e-1, 1e-3, 12)
        np.random.seed(321)
        with contextlib.redirect_stdout(io.StringIO()):
            g.run_RHMC(np.array(stars_m), f_pos=True, delta=1e-6, Niter=niter,
                       Nsteps=nsteps, dt=dt, N_max=len(stars_m), schedule_g_ff2=sg,
                       schedule_beta=sb)
        res = dict(D=g.D, q_model=np.array(stars_m), q_chain=g.q_chain,
                   p_chain=g.p_chain, E_chain=g.E_chain, V_chain=g.V_chain,
                   T_chain=g.T_chain, A_chain=g.A_chain.astype(np.int32),
                   niter=niter, nsteps=nsteps, seed=321, dt=dt, schedule_g_ff2=sg,
                   schedule_beta=np.zeros(0) if sb is None else sb,
                   g_ff2_final=g.g_ff2, beta_final=g.beta)
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))
        print(name, "accepted", g.A_chain.sum(), "of", niter + 1)
    return out


# ----------------------------------------------------------------------------
# Case 5: alternative integrators (single_gym, sampler_RHMC.py:592-783) and
#         post-processing (utils.py:86-209)
# ----------------------------------------------------------------------------
def case_solvers(S, U):
    out = {}
    for name, solver, stars_t, stars_m, dt, nsteps in [
        ("hmc", None, [[17., 8.3, 7.9]], [[17.2, 8.6, 7.7]], 0.02, 60),
        ("naive", "naive", [[19., 8.3, 7.9]], [[19.3, 8.6, 7.7]], 0.02, 60),
        ("leap_frog", "leap_frog", [[19., 8.3, 7.9]], [[19.3, 8.6, 7.7]], 0.05, 60),
        ("leap_frog_k2", "leap_frog", [[18., 5.3, 6.9], [19.5, 10.2, 9.1]],
         [[18.2, 5.6, 6.6], [19.9, 10.0, 9.4]], 0.05, 40),
        ("naive_wall", "naive", [[22.9, 8.3, 7.9]], [[22.95, 8.6, 7.7]], 0.3, 60),
    ]:
        np.random.seed(77)
        g = S.single_gym(dt=0., Nsteps=0, g_xx=1., g_ff=1.)
        g.num_rows = g.num_cols = 16
        g.fmin = g.mag2flux_converter(20.)
        g.fmax = g.mag2flux_converter(15.)
        g.gen_mock_data(np.array(stars_t))
        g.Nsteps, g.dt = nsteps, dt
        np.random.seed(5)
        with contextlib.redirect_stdout(io.StringIO()):
            if solver is None:
                g.run_single_HMC(q_model_0=np.array(stars_m), f_pos=False)
            else:
                g.run_single_RHMC(q_model_0=np.array(stars_m), f_pos=True, solver=solver)
        res = dict(D=g.D, q_chain=g.q_chain, p_chain=g.p_chain, E_chain=g.E_chain,
                   V_chain=g.V_chain, T_chain=g.T_chain, nsteps=nsteps)
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))

    # convergence_stats / variogram / acceptance_rate on synthetic chains
    rs = np.random.RandomState(9)
    for name, shape, ar in [("iid", (4, 400, 3), 0.0), ("ar", (3, 501, 2), 0.9),
                            ("ar_hi", (5, 300, 4), 0.98)]:
        e = rs.randn(*shape)
        x = np.empty(shape)
        x[:, 0] = e[:, 0]
        for t in range(1, shape[1]):
            x[:, t] = ar * x[:, t - 1] + np.sqrt(1 - ar * ar) * e[:, t]
        x += rs.randn(shape[0], 1, shape[2]) * 0.1       # small between-chain offsets
        R, neff = U.convergence_stats(x, thin_rate=2, warm_up_num=10)
        R1, neff1 = U.convergence_stats(x, thin_rate=1, warm_up_num=0)
        chains = [x[0, :100], x[1, :100]]
        vg = np.array([U.variogram(chains, 1, t) for t in (1, 2, 5)])
        dec = (rs.rand(shape[0], shape[1], 1) < 0.7).astype(float)
        acc = U.acceptance_rate(dec)
        acc2 = U.acceptance_rate(dec, start=10, end=50)
        out.update(pack("conv_" + name + "/", dict(x=x, R=R, neff=neff, R1=R1, neff1=neff1,
                                                   vg=vg, dec=dec, acc=acc, acc2=acc2)))
    return out


def case_datagen(S, U):
    """gen_model (sampler_RHMC.py:101-116), gen_mock_data (:77-99) and
    gen_noise_profile (:118-144) outputs.  gen_noise_profile calls
    np.histogram(normed=True), removed in NumPy 2: it is run with a shim that
    maps normed to density (equal-width bins: the same normalisation)."""
    out = {}
    cases = [("k1_48", "multi", 48, [[19., 24.3, 23.8]]),
             ("k1_32", "single", 32, [[17.5, 16.2, 15.7]]),
             ("k2_16", "single", 16, [[18., 5.3, 6.9], [19.5, 10.2, 9.1]])]
    g = make_gym(S, "multi", 48)
    np.random.seed(12)
    K = 10
    mags = 15. + 8.3 * np.random.rand(K)
    xy = np.random.rand(K, 2) * 46. + 1.
    cases.append(("k10_48", "multi", 48, np.column_stack([mags, xy]).tolist()))
    orig_hist = np.histogram

    def hist_shim(a, bins=10, range=None, normed=None, weights=None, density=None):
        return orig_hist(a, bins=bins, range=range, weights=weights,
                         density=bool(normed) or bool(density))
    for name, cls, n, stars in cases:
        g = make_gym(S, cls, n)
        qm = np.array(stars, dtype=float)
        model = g.gen_model(qm)
        np.random.seed(31)
        D = g.gen_mock_data(qm, return_data=True)
        np.random.seed(32)
        np.histogram = hist_shim
        try:
            g.gen_noise_profile(qm, N_trial=8, sig_fac=10)
        finally:
            np.histogram = orig_hist
        out.update(pack(name + "/", dict(stars=qm, q=stars_to_q(g, qm.copy()).reshape(-1, 3),
                                         model=model, D=D, hist=g.hist_noise,
                                         centers=g.centers_noise)))
        out.update(pack(name + "/par_", gym_params(g)))
    return out


def case_hmc_random(S, U, L):
    """samplers.lightsource_gym.HMC_random (samplers.py:460-572): the older
    sampler API's unit-mass HMC with a per-coordinate dt vector, random
    trajectory lengths and the flux wall (with its sticky-iflip / stale-p
    quirks, exercised by the "wall" cases).  The global NumPy RNG is seeded
    right before the call, so a test can replay the draws."""
    out = {}
    for name, n, stars_t, stars_m, dt3, niter, smin, smax, f_lim in [
        ("k1", 16, [[1500., 8.3, 7.9]], [[1400., 8.6, 7.7]], (8.0, 0.08, 0.08), 40, 5, 15, 0.),
        ("k2", 24, [[2500., 9.3, 10.9], [900., 14.2, 12.1]],
         [[2400., 9.6, 10.7], [1000., 14.0, 12.4]], (8.0, 0.06, 0.06), 30, 8, 20, 0.),
        ("wall", 16, [[60., 8.3, 7.9]], [[45., 8.6, 7.7]], (6., 0.05, 0.05), 40, 5, 15, 40.),
        ("wall2", 20, [[70., 6.3, 7.9], [1800., 12.2, 11.1]],
         [[48., 6.6, 7.7], [1750., 12.0, 11.4]], (8., 0.05, 0.05), 40, 4, 12, 44.),
    ]:
        g = L.lightsource_gym()
        g.num_rows = g.num_cols = n
        np.random.seed(77)
        g.gen_mock_data(np.array(stars_t))
        K = len(stars_m)
        g.Nobjs = K
        g.d = 3 * K
        g.dt = np.tile(np.array(dt3, dtype=float), K)
        q0 = np.array(stars_m, dtype=float)
        np.random.seed(5)
        with contextlib.redirect_stdout(io.StringIO()):
            g.HMC_random(q_model_0=q0, Nchain=1, Niter=niter, steps_min=smin,
                         steps_max=smax, f_lim=f_lim)
        out.update(pack(name + "/", dict(
            D=g.D, dt=g.dt, q0=q0.reshape(-1), Niter=niter, steps_min=smin, steps_max=smax,
            f_lim=f_lim, seed=5, q_chain=g.q_chain[0], E_chain=g.E_chain[0],
            dE_chain=g.dE_chain[0], A_chain=g.A_chain[0], B_count=g.B_count,
            fwhm_pix=g.PSF_FWHM_pix)))
    return out


def case_rj(S, U):
    """multi_gym.run_RHMC with the reversible-jump moves on (P_move[1:] != 0,
    sampler_RHMC.py:1089-1187; birth_death_move :1200-1270, split_merge_move
    :1273-1445, scipy Beta for the split fraction).  A seed whose run hits
    one of the reference's own dead ends (no star left, nothing mergeable) is
    skipped; the seed used is recorded."""
    out = {}
    for name, stars_t, stars_m, P_move, niter, nsteps, seeds in [
        ("rj_bd", [[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4]], [0.4, 0.6, 0.], 40, 8, range(100, 140)),
        ("rj_sm", [[18., 10.2, 12.7], [19., 20.3, 18.1], [19.5, 11., 14.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4]], [0.4, 0., 0.6], 40, 8, range(200, 240)),
        ("rj_all", [[18., 10.2, 12.7], [19., 20.3, 18.1], [20., 15., 25.]],
         [[18.3, 10.5, 12.2], [19.4, 20.0, 18.4], [19.6, 15.3, 24.6]], [0.4, 0.3, 0.3], 50, 6,
         range(300, 340)),
    ]:
        for seed in seeds:
            np.random.seed(77)
            g = make_gym(S, n=32, g_xx=0.05, g_ff=4., g_ff2=4., prior=True)
            g.gen_mock_data(np.array(stars_t))
            np.random.seed(seed)
            try:
                with contextlib.redirect_stdout(io.StringIO()), np.errstate(all="ignore"):
                    g.run_RHMC(np.array(stars_m), f_pos=True, delta=1e-6, Niter=niter,
                               Nsteps=nsteps, dt=0.05, N_max=8, P_move=P_move)
            except Exception:
                continue
            moves = np.bincount(g.move_chain, minlength=5)
            acc = np.bincount(g.move_chain[g.A_chain], minlength=5)
            if (P_move[1] > 0 and (acc[1] == 0 or acc[2] == 0 and moves[2] == 0)) or \
               (P_move[2] > 0 and (moves[3] == 0 or moves[4] == 0)):
                continue          # want every move type proposed (and some jumps accepted)
            break
        else:
            raise RuntimeError("no usable seed for " + name)
        res = dict(D=g.D, q_model=np.array(stars_m), q_chain=g.q_chain, p_chain=g.p_chain,
                   E_chain=g.E_chain, V_chain=g.V_chain, T_chain=g.T_chain,
                   A_chain=g.A_chain.astype(np.int32), move_chain=g.move_chain,
                   N_chain=g.N_chain, P_move=np.array(P_move), niter=niter, nsteps=nsteps,
                   seed=seed, dt=0.05, N_max=8)
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))
        print(name, "seed", seed, "moves", np.bincount(g.move_chain, minlength=5),
              "accepted", np.bincount(g.move_chain[g.A_chain], minlength=5),
              "N", g.N_chain.min(), g.N_chain.max())
    return out


def _jitter_model(stars, rs, dmag=0.05, dpos=0.2):
    m = np.array(stars, dtype=float).copy()
    m[:, 0] += dmag * rs.randn(len(m))
    m[:, 1:] += dpos * rs.randn(len(m), 2)
    return m


def case_mh_bigk(S, U):
    """multi_gym.run_RHMC move-0 (P_move = [1, 0, 0], f_pos = True,
    sampler_RHMC.py:1018-1083) at many stars, every start above the flux wall
    (V finite, sampler_RHMC.py:303-309), so that proposals are really accepted
    and rejected — the generator requires 0 < acceptance < 1 and tries seeds
    until a run has both (the seed used is recorded).

    d51: RHMC-big-sim4.py's geometry and parameters (32x32, 51 true stars from
         its power law, mags 15-20, g_xx 0.05, g_ff = g_ff2 = 4, prior on,
         RHMC-big-sim4.py:5-47), the model the truth jittered;
    w64: the C5 geometry (256x256, K = 64, big-sim4 parameters, prior), mags
         in [15, 22] (all above the wall at mag 23)."""
    out = {}
    for name, n, K, mags, niter, nsteps, seeds in [
        ("d51", 32, 51, (20., 15.), 10, 5, range(500, 540)),
        ("w64", 256, 64, (22., 15.), 8, 5, range(600, 640)),
    ]:
        np.random.seed(77)
        g = make_gym(S, n=n, g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True,
                     fminmax=mags)
        stars = powlaw_stars(U, g, K, n, mag_lo=mags[1], mag_hi=mags[0])
        g.gen_mock_data(stars)
        model = _jitter_model(stars, np.random.RandomState(K))
        assert (g.format_q(model.copy())[0::3] > 1.5 * g.f_lim).all()
        for seed in seeds:
            np.random.seed(seed)
            with contextlib.redirect_stdout(io.StringIO()):
                g.run_RHMC(model.copy(), f_pos=True, delta=1e-6, Niter=niter,
                           Nsteps=nsteps, dt=0.05, N_max=K)
            rate = g.A_chain.mean()
            if 0 < rate < 1:
                break
        else:
            raise RuntimeError("no seed with 0 < acceptance < 1 for " + name)
        assert np.isfinite(g.E_chain).all()
        res = dict(D=g.D, q_model=model, q_chain=g.q_chain, p_chain=g.p_chain,
                   E_chain=g.E_chain, V_chain=g.V_chain, T_chain=g.T_chain,
                   A_chain=g.A_chain.astype(np.int32), niter=niter, nsteps=nsteps,
                   seed=seed, dt=0.05)
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))
        print(name, "seed", seed, "accepted", g.A_chain.sum(), "of", niter + 1)
    return out


def case_rj_big(S, U):
    """run_RHMC with the reversible-jump moves across K = 64 (the register-slot
    boundary of the engine's one-wave-per-chain kernels): a 32x32 image of 100
    true stars from RHMC-big-sim4.py's power law (alpha 2, mags 15-20), 64
    model stars (the first 64 true stars, jittered; every flux above the wall,
    so V is finite), RHMC-big-sim4.py's move parameters (P_move
    [0.6, 0.2, 0.2], K_split 1, beta_a = beta_b = 4, N_max 120, prior on;
    :10, :42-47, :77), 2 steps per trajectory.  The generator requires the
    chain to grow past 65 stars and 0 < acceptance < 1."""
    np.random.seed(77)
    g = make_gym(S, n=32, g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True)
    g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
    stars = powlaw_stars(U, g, 100, 32, mag_lo=15., mag_hi=20.)
    g.gen_mock_data(stars)
    model = _jitter_model(stars[:64], np.random.RandomState(64))
    assert (g.format_q(model.copy())[0::3] > 1.5 * g.f_lim).all()
    niter, nsteps, P_move = 30, 2, [0.6, 0.2, 0.2]
    for seed in range(800, 900):
        np.random.seed(seed)
        try:
            with contextlib.redirect_stdout(io.StringIO()), np.errstate(all="ignore"):
                g.run_RHMC(model.copy(), f_pos=True, delta=1e-6, Niter=niter, Nsteps=nsteps,
                           dt=0.05, N_max=120, P_move=P_move)
        except Exception:
            continue
        if g.N_chain.max() > 65 and 0 < g.A_chain.mean() < 1:
            break
    else:
        raise RuntimeError("no seed grows past 64 stars")
    res = dict(D=g.D, q_model=model, q_chain=g.q_chain, p_chain=g.p_chain,
               E_chain=g.E_chain, V_chain=g.V_chain, T_chain=g.T_chain,
               A_chain=g.A_chain.astype(np.int32), move_chain=g.move_chain,
               N_chain=g.N_chain, P_move=np.array(P_move), niter=niter, nsteps=nsteps,
               seed=seed, dt=0.05, N_max=120, K_split=1., beta_a=4., beta_b=4.)
    out = pack("b64/", res)
    out.update(pack("b64/par_", gym_params(g)))
    print("rj_big seed", seed, "moves", np.bincount(g.move_chain, minlength=5),
          "accepted", np.bincount(g.move_chain[g.A_chain], minlength=5),
          "N", g.N_chain.min(), g.N_chain.max())
    return {"rj_big": out}


def case_flagship(S, U, niter=40, compact=False):
    """The reference's flagship run, RHMC-big-sim4.py, as written except
    Niter (40 instead of 10000) and verbose (off: it only prints and plots,
    which draws nothing from the RNG): seed 77, 32x32, 51 true stars from the
    power law (alpha 2, mags 15-20), 5 model stars, gen_mock_data,
    gen_noise_profile(N_trial = 1000) (with the normed -> density shim), then
    run_RHMC(f_pos, delta 1e-6, Nsteps 10, dt 0.05, P_move [0.6, 0.2, 0.2],
    N_max 120) with K_split 1, beta_a = beta_b = 4, prior on
    (RHMC-big-sim4.py:5-21, :39-47, :60-77).

    Recorded: the data image, the truth and model stars, NumPy's global
    stream state right before run_RHMC (so that a GPU test starts from it
    without re-running the 1000 noise realisations) and right after
    gen_mock_data, the noise histogram, and every chain record."""
    g = S.multi_gym(dt=0., Nsteps=0, g_xx=0.05, g_ff=4., g_ff2=4.)
    np.random.seed(77)
    g.num_rows = g.num_cols = 32
    n_true, n_model = int(32 ** 2 * 0.05), 5
    alpha, mag_max, mag_min = 2., 20., 15.
    fmin, fmax = g.mag2flux_converter(mag_max), g.mag2flux_converter(mag_min)
    mag = g.flux2mag_converter(U.gen_pow_law_sample(alpha, fmin, fmax, n_true))
    q_true = np.zeros((n_true, 3))
    for i in range(n_true):
        x = np.random.random() * (g.num_rows - 2.) + 1.
        y = np.random.random() * (g.num_cols - 2.) + 1.
        q_true[i] = np.array([mag[i], x, y])
    g.fmin, g.fmax = fmin, fmax
    g.K_split, g.beta_a, g.beta_b = 1., 4., 4.
    g.use_prior, g.alpha = True, alpha
    q_model = np.zeros((n_model, 3))
    q_model[:, 0] = g.flux2mag_converter(U.gen_pow_law_sample(alpha, fmin, fmax, n_model))
    q_model[:, 1] = np.random.random(size=n_model) * (g.num_rows - 2.) + 1.
    q_model[:, 2] = np.random.random(size=n_model) * (g.num_cols - 2.) + 1.
    g.gen_mock_data(q_true)
    st_data = np.random.get_state()
    orig_hist = np.histogram

    def hist_shim(a, bins=10, range=None, normed=None, weights=None, density=None):
        return orig_hist(a, bins=bins, range=range, weights=weights,
                         density=bool(normed) or bool(density))
    np.histogram = hist_shim
    try:
        g.gen_noise_profile(q_true, N_trial=1000)
    finally:
        np.histogram = orig_hist
    st_run = np.random.get_state()
    nsteps, dt, N_max, P_move = 10, 5e-2, 120, [0.6, 0.2, 0.2]
    with contextlib.redirect_stdout(io.StringIO()):
        g.run_RHMC(q_model.copy(), f_pos=True, delta=1e-6, Niter=niter, Nsteps=nsteps,
                   dt=dt, save_traj=False, verbose=False, q_true=q_true,
                   schedule_beta=None, P_move=P_move, N_max=N_max)
    if compact:  # the written length: records that say where two runs part
        res = dict(D=g.D, q_true=q_true, q_model=q_model,
                   rng_key=st_run[1], rng_pos=st_run[2],
                   rng_gauss=np.array([st_run[3], st_run[4]]),
                   E_chain=g.E_chain, V_chain=g.V_chain, T_chain=g.T_chain,
                   A_chain=g.A_chain.astype(np.int32), move_chain=g.move_chain,
                   N_chain=g.N_chain, q_every100=g.q_chain[::100], P_move=np.array(P_move),
                   niter=niter, nsteps=nsteps, dt=dt, N_max=N_max,
                   K_split=g.K_split, beta_a=g.beta_a, beta_b=g.beta_b)
        out = pack("", res)
        out.update(pack("par_", gym_params(g)))
        print("flagship_long moves", np.bincount(g.move_chain, minlength=5),
              "accepted", np.bincount(g.move_chain[g.A_chain], minlength=5),
              "N", g.N_chain.min(), g.N_chain.max())
        return {"flagship_long": out}
    res = dict(D=g.D, q_true=q_true, q_model=q_model,
               rng_data_key=st_data[1], rng_data_pos=st_data[2],
               rng_data_gauss=np.array([st_data[3], st_data[4]]),
               rng_key=st_run[1], rng_pos=st_run[2],
               rng_gauss=np.array([st_run[3], st_run[4]]),
               hist_noise=g.hist_noise, centers_noise=g.centers_noise,
               q_chain=g.q_chain, p_chain=g.p_chain, E_chain=g.E_chain,
               V_chain=g.V_chain, T_chain=g.T_chain, A_chain=g.A_chain.astype(np.int32),
               move_chain=g.move_chain, N_chain=g.N_chain, P_move=np.array(P_move),
               niter=niter, nsteps=nsteps, dt=dt, N_max=N_max,
               K_split=g.K_split, beta_a=g.beta_a, beta_b=g.beta_b)
    out = pack("", res)
    out.update(pack("par_", gym_params(g)))
    print("flagship moves", np.bincount(g.move_chain, minlength=5),
          "accepted", np.bincount(g.move_chain[g.A_chain], minlength=5),
          "N", g.N_chain.min(), g.N_chain.max())
    return {"flagship": out}


def case_hugek(S, U):
    """K > 256 stars per chain: the engine's slotted kernels with their factor
    tables in global memory (8 register slots up to 512 stars, 16 up to
    1024).  The reference's dVdq / V / RHMC_single_step are vectorised over
    any K (sampler_RHMC.py:365-425, :294-351, :522-566).

    hugek.npz: per-function vectors (dVdq, dphidq, V, T, H) at K = 300 (64 px)
    and K = 700 (128 px), big-sim4 parameters + prior, 3 states each.
    traj_hugek.npz: 1 chain x 3 steps at 64 px, K = 300; traj_hugek700.npz:
    1 chain x 2 steps at 128 px, K = 700."""
    out = {}
    rs = np.random.RandomState(9)
    for name, n, K in (("h300", 64, 300), ("h700", 128, 700)):
        np.random.seed(77)
        g = make_gym(S, n=n, g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True)
        stars = powlaw_stars(U, g, K, n)
        g.gen_mock_data(np.array(stars))
        g.Nobjs, g.d = K, 3 * K
        q_true = stars_to_q(g, stars)
        qs, ps = [], []
        for t in range(3):
            q = q_true.copy()
            q[0::3] *= np.exp(0.2 * rs.randn(K))
            q[1::3] += 0.5 * rs.randn(K)
            q[2::3] += 0.5 * rs.randn(K)
            qs.append(q)
            ps.append(rs.randn(3 * K) * np.sqrt(np.abs(g.H(q))))
        qs, ps = np.array(qs), np.array(ps)
        res = dict(D=g.D, q=qs, p=ps)
        res["dVdq"] = np.array([g.dVdq(q) for q in qs])
        res["H"] = np.array([g.H(q) for q in qs])
        res["dphidq"] = np.array([g.dphidq(q) for q in qs])
        res["V"] = np.array([g.V(q, f_pos=False) for q in qs])
        res["Vpos"] = np.array([g.V(q, f_pos=True) for q in qs])
        res["T"] = np.array([g.T(p, g.H(q)) for q, p in zip(qs, ps)])
        out.update(pack(name + "/", res))
        out.update(pack(name + "/par_", gym_params(g)))
        print("hugek", name, "done")
    cases = {"hugek": out}
    big = dict(g_xx=0.05, g_ff=4., g_ff2=4., dt=0.05, prior=True)
    cases["traj_hugek"] = traj_case(
        S, U, 64, lambda g: powlaw_stars(U, g, 300, 64),
        lambda g, c: powlaw_stars(U, g, 300, 64), big, 1, 3)
    cases["traj_hugek700"] = traj_case(
        S, U, 128, lambda g: powlaw_stars(U, g, 700, 128),
        lambda g, c: powlaw_stars(U, g, 700, 128), big, 1, 2)
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    S, U, L, tmp = load_reference(args.ref)
    try:
        jobs = {"functions": case_functions, "steps": case_steps,
                "mh": case_mh, "mh_sched": case_mh_sched, "solvers": case_solvers,
                "datagen": case_datagen}
        for name, fn in jobs.items():
            if args.only and args.only != name:
                continue
            np.savez_compressed(os.path.join(HERE, name + ".npz"), **fn(S, U))
            print("wrote", name)
        if not args.only or args.only == "rj":
            np.savez_compressed(os.path.join(HERE, "rj.npz"), **case_rj(S, U))
            print("wrote rj")
        if not args.only or args.only == "hmc_random":
            np.savez_compressed(os.path.join(HERE, "hmc_random.npz"), **case_hmc_random(S, U, L))
            print("wrote hmc_random")
        if not args.only or args.only == "trajs":
            for name, d in case_trajs(S, U).items():
                np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
                print("wrote", name)
        if not args.only or args.only == "mh_bigk":
            np.savez_compressed(os.path.join(HERE, "mh_bigk.npz"), **case_mh_bigk(S, U))
            print("wrote mh_bigk")
        # subsets of the above, regenerated on their own (--only c5 / bigk)
        if args.only == "flagship_long":   # RHMC-big-sim4.py at Niter = 10000 (minutes)
            for name, d in case_flagship(S, U, niter=10000, compact=True).items():
                np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
                print("wrote", name)
        for job, fn in (("c5", case_c5), ("bigk", case_bigk), ("flagship", case_flagship),
                        ("rj_big", case_rj_big), ("hugek", case_hugek)):
            if args.only == job or (not args.only and job in ("bigk", "flagship", "rj_big",
                                                              "hugek")):
                for name, d in fn(S, U).items():
                    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
                    print("wrote", name)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
