"""The reference's `sampler_RHMC` entry points, routed to the MI355X engine.

Mirrors jaekor91/HMC-stellar-toy-model `sampler_RHMC.py` (file:line cited per
method): same class names, constructor arguments, attributes (set them after
construction exactly like the reference scripts do, e.g.
`gym.num_rows = gym.num_cols = 32; gym.use_prior = True`), method names,
argument meaning, global-NumPy-RNG draw order and return values.

What runs where:
  * RHMC_single_step, dVdq, dphidq, V and the batched RHMC_steps run in
    librhmc.so (HIP kernels, rhmc_amd.capi).  There is no CPU fallback:
    without a GPU these raise.
  * O(K) scalar helpers (H, H_ff, H_xx, T, dtaudq, dtaudp, dVdq_RHMC) and the
    MH bookkeeping stay on the host, as NumPy, like in the reference.

Quirks kept on purpose: g0/g1/g2 are computed once at
construction on the default 48x48 grid and NOT recomputed when num_rows is
changed later; single_gym ignores its g_ff2 argument; V needs fmin/fmax for
its prior constant (computed and cached on the first V call); use_Vc needs
f_expnt to be set (TypeError otherwise, like the reference).

Out of scope here: plotting (display_image, diagnostics_*).
"""
import sys

import numpy as np

from . import capi
from .photometry import (default_exp_setup, factors, flux2mag, gauss_PSF,
                         gen_pow_law_sample, mag2flux, poisson_realization)


class base_class(object):
    """sampler_RHMC.py:27-566."""

    def __init__(self, dt=1., g_xx=10, g_ff=10, g_ff2=2):
        self._D = None
        self._ctx = None
        self._ctx_shape = None
        self.M = None
        (self.num_rows, self.num_cols, self.flux_to_count, self.PSF_FWHM_pix,
         self.B_count, self.arcsec_to_pix, self.mB, self.f_lim) = default_exp_setup()
        self.dt = dt
        self.g_xx = g_xx
        self.g_ff = g_ff
        self.g_ff2 = g_ff2
        self.compute_factors()
        self.vmin = None
        self.vmax = None
        self.use_prior = False
        self.alpha = 2.
        self.use_Vc = False
        self.beta = 1.
        self.f_expnt = None
        self.Vc_r_pow = 1.
        self.V_prior_const = None
        self.K_split = 1.
        self.beta_a = 2.
        self.beta_b = 2.
        self.move_types = {0: "within", 1: "birth", 2: "death", 3: "split", 4: "merge"}
        self.device = 0

    # ---------------------------------------------------------------- data
    @property
    def D(self):
        return self._D

    @D.setter
    def D(self, value):
        self._D = None if value is None else np.ascontiguousarray(value, dtype=np.float64)
        self._ctx_shape = None        # re-upload on next use

    def _context(self):
        if self._D is None:
            raise ValueError("no data image: call gen_mock_data() or set .D first")
        if self._ctx is None:
            self._ctx = capi.Context(self._D, device=self.device)
        elif self._ctx_shape is None:
            self._ctx.set_image(self._D)
        self._ctx_shape = self._D.shape
        return self._ctx

    def _params(self, delta=1e-6, counter_max=1000, for_energy=False):
        vpc = 0.
        if for_energy:
            if self.V_prior_const is None:     # :320-321 (evaluated unconditionally)
                self.V_prior_const = np.log(self.num_rows * self.num_cols) - np.log(
                    (1 - self.alpha) / (self.fmax ** (1 - self.alpha) - self.fmin ** (1 - self.alpha)))
            vpc = self.V_prior_const
        if self.use_Vc and self.f_expnt is None:
            # the reference raises here too (:388, None ** ... TypeError)
            raise TypeError("use_Vc requires f_expnt to be set")
        return capi.make_params(
            dt=self.dt, delta=delta, counter_max=counter_max, B_count=self.B_count,
            f_lim=self.f_lim, f_low=self.mag2flux_converter(self.mB + 2),
            fwhm_pix=self.PSF_FWHM_pix, g_xx=self.g_xx, g_ff=self.g_ff, g_ff2=self.g_ff2,
            g0=self.g0, g1=self.g1, g2=self.g2, use_prior=self.use_prior, alpha=self.alpha,
            use_Vc=self.use_Vc, beta=self.beta, Vc_r_pow=self.Vc_r_pow, V_prior_const=vpc)

    def _check_geometry(self):
        if self._D is not None and self._D.shape != (self.num_rows, self.num_cols):
            raise ValueError("D has shape %s but num_rows/num_cols are %d/%d"
                             % (self._D.shape, self.num_rows, self.num_cols))

    def gen_mock_data(self, q_true=None, return_data=False, rng="numpy", seed=0):
        """sampler_RHMC.py:77-99.  rng="numpy": the reference's global NumPy
        RNG, row-major Poisson draws (bit-identical data).  rng="device": model
        and Poisson draw on the GPU (rhmc_gen_image, Philox keyed by `seed`);
        without return_data the image is installed in the device context
        directly (no host->device upload) and mirrored to .D."""
        if rng == "device":
            self._check_square()
            ctx = self._gen_context()
            data = ctx.gen_image(self._gen_params(), self._counts(q_true), self.num_rows,
                                 self.num_cols, n_real=1, seed=seed,
                                 install=not return_data)[0]
            if return_data:
                return data
            self._D = np.ascontiguousarray(data)
            self._ctx_shape = data.shape
            return None
        if rng != "numpy":
            raise ValueError("rng must be 'numpy' or 'device'")
        data = np.ones((self.num_rows, self.num_cols), dtype=float) * self.B_count
        for i in range(q_true.shape[0]):
            mag, x, y = q_true[i]
            data += self.mag2flux_converter(mag) * gauss_PSF(
                self.num_rows, self.num_cols, x, y, FWHM=self.PSF_FWHM_pix)
        data = poisson_realization(data)
        if return_data:
            return data
        self.D = data

    def gen_model(self, q_model, device=False):
        """sampler_RHMC.py:101-116 (device=True: rhmc_gen_image, n_real=0)."""
        if device:
            self._check_square()
            return self._gen_context().gen_image(self._gen_params(), self._counts(q_model),
                                                 self.num_rows, self.num_cols, n_real=0)
        model = np.ones((self.num_rows, self.num_cols), dtype=float) * self.B_count
        for i in range(q_model.shape[0]):
            mag, x, y = q_model[i]
            model += self.mag2flux_converter(mag) * gauss_PSF(
                self.num_rows, self.num_cols, x, y, FWHM=self.PSF_FWHM_pix)
        return model

    def gen_noise_profile(self, q_true, N_trial=1000, sig_fac=10, rng="numpy", seed=0):
        """sampler_RHMC.py:118-145 (`normed=` is NumPy's `density=` today).
        rng="device": the N_trial realisations are one rhmc_gen_image launch."""
        if rng == "device":
            self._check_square()
            ctx = self._gen_context()
            gp = self._gen_params()
            q = self._counts(q_true)
            truth = ctx.gen_image(gp, q, self.num_rows, self.num_cols, n_real=0)
            res = (ctx.gen_image(gp, q, self.num_rows, self.num_cols, n_real=N_trial,
                                 seed=seed) - truth).ravel()
        elif rng == "numpy":
            truth = self.gen_model(q_true)
            res = np.vstack([poisson_realization(truth) - truth
                             for _ in range(N_trial)]).ravel()
        else:
            raise ValueError("rng must be 'numpy' or 'device'")
        sig = np.sqrt(self.B_count)
        bins = np.arange(-sig_fac * sig, sig_fac * sig, sig / 5.)
        hist, _ = np.histogram(res, bins=bins, density=True)
        self.hist_noise = hist
        self.centers_noise = (bins[1:] + bins[:-1]) / 2.

    def _counts(self, q_mag):
        """(K, 3) mag, x, y -> (K, 3) counts, x, y (like format_q, :209)."""
        q = np.array(q_mag, dtype=float).reshape(-1, 3)
        q[:, 0] = [self.mag2flux_converter(m) for m in q[:, 0]]
        return q

    def _check_square(self):
        if self.num_rows != self.num_cols:
            raise ValueError("square images only (gauss_PSF, utils.py:481-483)")

    def _gen_context(self):
        if self._ctx is None:
            self._ctx = capi.Context(None, device=self.device)
            self._ctx_shape = None        # .D (if any) is uploaded on first use
        return self._ctx

    def _gen_params(self):
        """rhmc_gen_image reads B_count and PSF_FWHM_pix only."""
        return capi.make_params(dt=self.dt, delta=1e-6, counter_max=1, B_count=self.B_count,
                                f_lim=self.f_lim, f_low=0., fwhm_pix=self.PSF_FWHM_pix,
                                g_xx=1., g_ff=1., g_ff2=1., g0=self.g0, g1=self.g1, g2=self.g2)

    def mag2flux_converter(self, mag):
        """sampler_RHMC.py:147-152"""
        return mag2flux(mag) * self.flux_to_count

    def flux2mag_converter(self, flux):
        """sampler_RHMC.py:154-159"""
        return flux2mag(flux / self.flux_to_count)

    def compute_factors(self):
        """sampler_RHMC.py:161-167 (on the grid current at call time)."""
        self.g0, self.g1, self.g2 = factors(self.num_rows, self.num_cols, self.num_rows / 2.,
                                            self.num_cols / 2., self.PSF_FWHM_pix)

    def default_exp_setup(self):
        """sampler_RHMC.py:169-201"""
        r, c, ftc, fwhm, B, a2p, mB, f_lim = default_exp_setup()
        self.mB, self.f_lim = mB, f_lim
        return r, c, ftc, fwhm, B, a2p

    def u_sample(self, d):
        """sampler_RHMC.py:203-207"""
        return np.random.randn(d)

    def format_q(self, q):
        """sampler_RHMC.py:209-217 (mutates q like the reference)."""
        for i in range(q.shape[0]):
            q[i, 0] = self.mag2flux_converter(q[i, 0])
        return q.reshape((q.size,))

    def _format_q_fast(self, q_model):
        """format_q on a copy, per star with Python floats: the same pow and
        product per element as mag2flux_converter (bit-equal), ~4x faster than
        the np.float64 scalar loop (the batched drivers convert thousands of
        chains)."""
        q = np.array(q_model, dtype=np.float64)
        ftc = self.flux_to_count
        q[:, 0] = [10 ** (0.4 * (22.5 - v)) * ftc for v in q[:, 0].tolist()]
        return q.reshape(-1)

    def reverse_format_q(self, q):
        """sampler_RHMC.py:219-227"""
        q = np.copy(q.reshape((-1, 3)))
        for i in range(q.shape[0]):
            q[i, 0] = self.flux2mag_converter(q[i, 0])
        return q

    # ---------------------------------------------------- O(K) host helpers
    def H(self, q, grad=False):
        """sampler_RHMC.py:229-258"""
        K = q.size // 3
        Hd = np.zeros(q.size)
        Hg = np.zeros(q.size)
        for i in range(K):
            f = q[3 * i]
            if grad:
                Hd[3 * i], Hg[3 * i] = self.H_ff(f, grad=True)
                v, g = self.H_xx(f, grad=True)
                Hd[3 * i + 1] = Hd[3 * i + 2] = v
                Hg[3 * i + 1] = Hg[3 * i + 2] = g
            else:
                Hd[3 * i] = self.H_ff(f)
                Hd[3 * i + 1] = Hd[3 * i + 2] = self.H_xx(f)
        return (Hd, Hg) if grad else Hd

    def _H_vec(self, q):
        """H(q, grad=False) with the per-star loop vectorised: the same IEEE
        operations in the same order per element (tests/test_sampler_host.py
        checks bit equality with H), for the batched runners' host work."""
        f = np.asarray(q, dtype=np.float64)[0::3]
        Hf = 1. / (f / self.g_ff2 + (self.B_count / self.g0) / self.g_ff)
        f_low = self.mag2flux_converter(self.mB + 2)
        fl = np.where(f < f_low, f_low, f)
        s = 1. / (self.g1 * fl) + self.B_count / (self.g2 * fl ** 2)
        Hx = self.g_xx * s ** -1
        Hd = np.empty(3 * f.size)
        Hd[0::3], Hd[1::3], Hd[2::3] = Hf, Hx, Hx
        return Hd

    def H_xx(self, f, grad=False):
        """sampler_RHMC.py:260-280"""
        f_low = self.mag2flux_converter(self.mB + 2)
        low = f < f_low
        if low:
            f = f_low
        s = 1. / (self.g1 * f) + self.B_count / (self.g2 * f ** 2)
        val = self.g_xx * s ** -1
        if not grad:
            return val
        g = 0 if low else self.g_xx * (1. / (self.g1 * f ** 2) + 2 * self.B_count
                                       / (self.g2 * f ** 3)) * s ** -2
        return val, g

    def H_ff(self, f, grad=False):
        """sampler_RHMC.py:283-292 (gradient ignores g_ff2, :292)"""
        val = 1. / (f / self.g_ff2 + (self.B_count / self.g0) / self.g_ff)
        if not grad:
            return val
        return val, -1. / (f + (self.B_count / self.g0) / self.g_ff) ** 2

    def T(self, p, H_diag):
        """sampler_RHMC.py:353-363"""
        return (np.sum(p ** 2 / H_diag) + np.sum(np.log(np.abs(H_diag)))) / 2.

    def dVdq_RHMC(self, q, p):
        """sampler_RHMC.py:427-446"""
        g = np.zeros_like(q)
        H, Hg = self.H(q, grad=True)
        for i in range(q.size // 3):
            t1 = (p[3 * i] ** 2) * (-Hg[3 * i] / H[3 * i] ** 2)
            t2 = (Hg[3 * i] / H[3 * i]) + (2 * Hg[3 * i + 1] / H[3 * i + 1])
            g[3 * i] = (t1 + t2) / 2.
        return g

    def dtaudq(self, q, p):
        """sampler_RHMC.py:467-483"""
        g = np.zeros_like(q)
        H, Hg = self.H(q, grad=True)
        for i in range(q.size // 3):
            g[3 * i] = ((p[3 * i] ** 2) * (-Hg[3 * i] / H[3 * i] ** 2)) / 2.
        return g

    def dtaudp(self, q, p):
        """sampler_RHMC.py:485-492"""
        return p / self.H(q, grad=False)

    # ---------------------------------------------------- device hot path
    def V(self, q, f_pos=False):
        """sampler_RHMC.py:294-351 on the GPU (rhmc_energy).  q: [3K] or [n, 3K]."""
        self._check_geometry()
        V, _ = self._context().energy(self._params(for_energy=True), q, None, f_pos=f_pos)
        return V

    def V_T(self, q, p, f_pos=False):
        """Batched V(q) and T(p, H(q)) in one launch: q, p [n, 3K] -> (V[n], T[n])."""
        self._check_geometry()
        return self._context().energy(self._params(for_energy=True), q, p, f_pos=f_pos)

    def dVdq(self, q):
        """sampler_RHMC.py:365-425 on the GPU (rhmc_gradient kind 0)."""
        self._check_geometry()
        return self._context().gradient(self._params(), q, kind=0)

    def dphidq(self, q):
        """sampler_RHMC.py:448-465 on the GPU (rhmc_gradient kind 1)."""
        self._check_geometry()
        return self._context().gradient(self._params(), q, kind=1)

    def RHMC_single_step(self, q_tmp, p_tmp, delta=1e-6, counter_max=1000):
        """sampler_RHMC.py:522-566 — one implicit generalized-leapfrog step with
        flux-wall / edge reflection.  Returns new (q, p); inputs untouched."""
        return self.RHMC_steps(q_tmp, p_tmp, 1, delta=delta, counter_max=counter_max)

    def RHMC_steps(self, q, p, n_steps, delta=1e-6, counter_max=1000, return_info=False):
        """Batched, fused: n_steps RHMC_single_step()s on every chain of
        q, p [n_chains, 3K] (or [3K]) in one launch.  With return_info also
        returns the per-chain (p-loop, q-loop) iteration sums and status bits."""
        self._check_geometry()
        return self._context().leapfrog(self._params(delta, counter_max), q, p, n_steps,
                                        return_info=return_info)

    def display_image(self, *args, **kwargs):
        raise NotImplementedError("plotting is out of scope of the MI355X engine")


class single_gym(base_class):
    """sampler_RHMC.py:569-879 (single trajectories)."""

    def __init__(self, Nsteps=100, dt=0.1, g_xx=1., g_ff=1., g_ff2=1.):
        base_class.__init__(self, dt=dt, g_xx=g_xx, g_ff=g_ff, g_ff2=1.)  # g_ff2 ignored (:578)
        self.Nsteps = Nsteps
        self.q_chain = self.p_chain = self.E_chain = self.V_chain = self.T_chain = None

    def run_single_HMC(self, q_model_0=None, f_pos=False):
        """sampler_RHMC.py:592-647 — plain HMC, naive leapfrog, unit metric."""
        self.Nobjs = q_model_0.shape[0]
        self.d = self.Nobjs * 3
        q_model_0 = self.format_q(q_model_0)
        n = self.Nsteps + 1
        self.q_chain = np.zeros((n, self.d))
        self.p_chain = np.zeros((n, self.d))
        self.E_chain = np.zeros(n)
        self.V_chain = np.zeros(n)
        self.T_chain = np.zeros(n)
        q_tmp = q_model_0
        p_tmp = self.u_sample(self.d)
        self.q_chain[0], self.p_chain[0] = q_tmp, p_tmp
        self.V_chain[0] = self.V(q_tmp, f_pos=f_pos)
        self.T_chain[0] = self.T(p_tmp, np.ones_like(p_tmp))
        self.E_chain[0] = self.V_chain[0] + self.T_chain[0]
        params = self._params()
        ctx = self._context()
        for i in range(1, n):
            # one plain-leapfrog step on the GPU (rhmc_integrate, SOLVER_HMC)
            q_tmp, p_tmp = ctx.integrate(params, capi.SOLVER_HMC, q_tmp, p_tmp, 1)
            self.q_chain[i], self.p_chain[i] = q_tmp, p_tmp
            self.V_chain[i] = self.V(q_tmp, f_pos=f_pos)
            self.T_chain[i] = self.T(p_tmp, np.ones_like(p_tmp))
            self.E_chain[i] = self.V_chain[i] + self.T_chain[i]

    def run_single_RHMC(self, q_model_0=None, f_pos=False, solver="naive", delta=1e-6,
                        p_initial=None, counter_max=100):
        """sampler_RHMC.py:649-783.  solver="implicit" is the engine's step
        (identical math to RHMC_single_step, :729-772); "naive" and
        "leap_frog" are the explicit RHMC integrators of rhmc_integrate."""
        if solver not in ("naive", "leap_frog", "implicit"):
            assert False
        self.Nobjs = q_model_0.shape[0]
        self.d = self.Nobjs * 3
        q_model_0 = self.format_q(q_model_0)
        n = self.Nsteps + 1
        self.q_chain = np.zeros((n, self.d))
        self.p_chain = np.zeros((n, self.d))
        self.E_chain = np.zeros(n)
        self.V_chain = np.zeros(n)
        self.T_chain = np.zeros(n)
        q_tmp = q_model_0
        H_diag = self.H(q_tmp)
        if p_initial is None:
            p_initial = self.u_sample(self.d) * np.sqrt(H_diag)
        p_tmp = p_initial
        self.q_chain[0], self.p_chain[0] = q_tmp, p_tmp
        V0 = self.V(q_tmp, f_pos=f_pos)
        T0 = self.T(p_tmp, H_diag)
        for i in range(1, n):
            if solver == "implicit":
                q_tmp, p_tmp = self.RHMC_single_step(q_tmp, p_tmp, delta=delta,
                                                     counter_max=counter_max)
                H_diag = self.H(q_tmp)
            else:
                sol = capi.SOLVER_RHMC_NAIVE if solver == "naive" else capi.SOLVER_RHMC_LEAPFROG
                q_tmp, p_tmp = self._context().integrate(self._params(), sol, q_tmp, p_tmp, 1,
                                                         f_pos=f_pos)
                H_diag = self.H(q_tmp)
            self.q_chain[i], self.p_chain[i] = q_tmp, p_tmp
            self.V_chain[i] = self.V(q_tmp, f_pos=f_pos) - V0
            self.T_chain[i] = self.T(p_tmp, H_diag) - T0
            self.E_chain[i] = self.V_chain[i] + self.T_chain[i]


class multi_gym(base_class):
    """sampler_RHMC.py:883-1473 (fixed-dimension RHMC MCMC)."""

    def __init__(self, Nsteps=100, dt=0.1, g_xx=1., g_ff=1., g_ff2=1.):
        base_class.__init__(self, dt=dt, g_xx=g_xx, g_ff=g_ff, g_ff2=g_ff2)
        self.Nsteps = Nsteps
        self.q_chain = self.p_chain = self.E_chain = self.V_chain = self.T_chain = None
        self.A_chain = None
        self.fmin = None
        self.fmax = None

    def run_RHMC(self, q_model_0, f_pos=True, delta=1e-6, Niter=100, Nsteps=100, dt=1e-1,
                 save_traj=False, counter_max=1000, verbose=False, q_true=None,
                 schedule_g_ff2=None, N_max=50, P_move=[1., 0., 0.], schedule_beta=None):
        """sampler_RHMC.py:937-1198.  Each batch of Nsteps leapfrog steps is ONE
        fused launch.  Same global NumPy RNG stream as the reference: per
        iteration randn(d), the move-type choice (one uniform), then for
        move 0 random(1); for the reversible-jump moves (P_move[1:] != 0) the
        grow/shrink choice, the move's own draws (birth_death_move /
        split_merge_move) and random(1)."""
        if save_traj:
            assert False                                  # :966-968
        self.dt, self.Niter, self.Nsteps = dt, Niter, Nsteps
        self.save_traj, self.P_move, self.N_max = save_traj, P_move, N_max
        self.Nobjs = q_model_0.shape[0]
        self.d = self.Nobjs * 3
        q_model_0 = self.format_q(q_model_0)
        self.q_chain = np.zeros((Niter + 1, N_max * 3))
        self.p_chain = np.zeros((Niter + 1, N_max * 3))
        self.E_chain = np.zeros(Niter + 1)
        self.V_chain = np.zeros(Niter + 1)
        self.T_chain = np.zeros(Niter + 1)
        self.A_chain = np.zeros(Niter + 1, dtype=bool)
        self.move_chain = np.zeros(Niter + 1, dtype=int)
        self.N_chain = np.zeros(Niter + 1, dtype=int)
        q_tmp = np.copy(q_model_0)
        for l in range(Niter + 1):
            if schedule_g_ff2 is not None and l < schedule_g_ff2.size:
                self.g_ff2 = schedule_g_ff2[l]
            if schedule_beta is not None and l < schedule_beta.size:
                self.beta = schedule_beta[l]
            H_diag = self.H(q_tmp, grad=False)
            p_tmp = self.u_sample(self.d) * np.sqrt(H_diag)
            V_initial = self.V(q_tmp, f_pos=f_pos)
            T_initial = self.T(p_tmp, H_diag)
            E_initial = V_initial + T_initial
            self.q_chain[l, :self.d] = q_tmp
            self.p_chain[l, :self.d] = p_tmp
            self.V_chain[l] = V_initial
            self.E_chain[l] = E_initial
            self.T_chain[l] = T_initial
            self.N_chain[l] = self.Nobjs
            move_type = np.random.choice([0, 1, 2], p=self.P_move, size=1)[0]
            if move_type == 0:                            # :1048-1088
                self.move_chain[l] = 0
                q_tmp, p_tmp = self.RHMC_steps(q_tmp, p_tmp, self.Nsteps, delta=delta,
                                               counter_max=counter_max)
                H_diag = self.H(q_tmp, grad=False)
                E_final = self.V(q_tmp, f_pos=f_pos) + self.T(p_tmp, H_diag)
                dE = E_final - E_initial
                lnu = np.log(np.random.random(1))
                if (dE < 0) or (lnu < -dE):
                    self.A_chain[l] = 1
                else:
                    q_tmp = self.q_chain[l, :self.d]
            else:
                # reversible-jump moves (:1089-1187): Nsteps RHMC steps, momentum
                # flip, the dimension-changing proposal, Nsteps steps, flip, then
                # accept with ln alpha0 = -dE + factor
                grow = np.random.choice([True, False], p=[0.5, 0.5])
                self.move_chain[l] = (1 if grow else 2) if move_type == 1 else (3 if grow else 4)
                q_tmp, p_tmp = self.RHMC_steps(q_tmp, p_tmp, self.Nsteps, delta=delta,
                                               counter_max=counter_max)
                p_tmp = -p_tmp
                move = self.birth_death_move if move_type == 1 else self.split_merge_move
                q_tmp, p_tmp, factor = move(q_tmp, p_tmp, grow)
                q_tmp, p_tmp = self.RHMC_steps(q_tmp, p_tmp, self.Nsteps, delta=delta,
                                               counter_max=counter_max)
                p_tmp = -p_tmp
                H_diag = self.H(q_tmp, grad=False)
                E_final = self.V(q_tmp, f_pos=f_pos) + self.T(p_tmp, H_diag)
                ln_alpha0 = -(E_final - E_initial) + factor
                lnu = np.log(np.random.random(1))
                if (ln_alpha0 > 0) or (lnu < ln_alpha0):
                    self.A_chain[l] = 1
                else:                                         # undo the dimension change
                    self.Nobjs += -1 if grow else 1
                    self.d = 3 * self.Nobjs
                    q_tmp = self.q_chain[l, :self.d]
            if verbose and (l % 50) == 0:                 # :1183-1186, every move type
                print("/---- Completed iteration %d" % l)
                print("N_objs: %d\n" % self.Nobjs)
                self.R_accept_report(idx_iter=l, run_window=10)
        print("Finished. Final report.")                  # :1195-1196
        self.R_accept_report(idx_iter=-1, running=False)

    # ------------------------------------------------ reversible-jump moves
    def _one_star_T(self, q3, p3):
        """T of a single star (q3, p3 of length 3) at its own metric."""
        H3 = self.H(q3, grad=False)
        return self.T(p3, H3), H3

    def birth_death_move(self, q_tmp, p_tmp, birth_death=None):
        """sampler_RHMC.py:1200-1270.  Birth (True): a new star with x, y
        uniform on [1, n-1), flux from the power-law prior, momentum from its
        own metric, appended last.  Death (False): a uniformly chosen star is
        removed.  Returns (q, p, ln-acceptance correction); updates Nobjs, d."""
        if birth_death is None or self.alpha is None or self.fmin is None or self.fmax is None:
            assert False                                  # :1205-1207 (prior required)
        if birth_death:
            x = np.random.random() * (self.num_rows - 2.) + 1.
            y = np.random.random() * (self.num_cols - 2.) + 1.
            f = gen_pow_law_sample(self.alpha, self.fmin, self.fmax, 1)[0]
            q_new = np.array([f, x, y])
            H3 = self.H(q_new, grad=False)
            p_new = self.u_sample(3) * np.sqrt(H3)
            q = np.concatenate([q_tmp, q_new])
            p = np.concatenate([p_tmp, p_new])
            factor = (self.alpha * np.log(f) - 3 / 2. + self.T(p_new, H3)
                      + self.V_prior_const)
            self.Nobjs += 1
        else:
            k = np.random.randint(0, self.Nobjs, size=1)[0]
            sl = slice(3 * k, 3 * k + 3)
            T_k, _ = self._one_star_T(q_tmp[sl], p_tmp[sl])
            factor = -self.alpha * np.log(q_tmp[3 * k]) + 3 / 2. - T_k - self.V_prior_const
            q = np.delete(q_tmp, np.s_[sl])
            p = np.delete(p_tmp, np.s_[sl])
            self.Nobjs -= 1
        self.d = 3 * self.Nobjs
        return q, p, factor

    def split_merge_move(self, q_tmp, p_tmp, split_merge=None):
        """sampler_RHMC.py:1273-1445.  Split (True): star i (uniform) becomes
        (F f, x + (1-F) dx, y + (1-F) dy) in place and ((1-F) f, x - F dx,
        y - F dy) appended, F ~ Beta(beta_a, beta_b), (dx, dy) ~ N(0,
        K_split^2); fresh momenta for both.  Merge (False): a pair (i, j)
        chosen with probability ~ Beta(F_ij) N(r_ij) (self-pairs excluded),
        removed, and the flux-weighted merged star appended with a fresh
        momentum.  Returns (q, p, ln-acceptance correction)."""
        from scipy.stats import beta as BETA
        if split_merge is None:
            assert False
        a, b, Ks = self.beta_a, self.beta_b, self.K_split
        ln_q_dxdy = np.log(2 * np.pi * Ks ** 2)
        if split_merge:
            i = np.random.randint(0, self.Nobjs, size=1)[0]
            f_s, x_s, y_s = q_tmp[3 * i:3 * i + 3]
            q_star = np.copy(q_tmp[3 * i:3 * i + 3])
            p_star = np.copy(p_tmp[3 * i:3 * i + 3])
            dx, dy = np.random.randn(2) * Ks
            dr_sq = dx ** 2 + dy ** 2
            F = BETA.rvs(a, b, size=1)[0]
            q_1 = np.array([F * f_s, x_s + (1 - F) * dx, y_s + (1 - F) * dy])
            q_2 = np.array([(1 - F) * f_s, x_s - F * dx, y_s - F * dy])
            H1 = self.H(q_1, grad=False)
            p_1 = self.u_sample(3) * np.sqrt(H1)
            H2 = self.H(q_2, grad=False)
            p_2 = self.u_sample(3) * np.sqrt(H2)
            T_star, _ = self._one_star_T(q_star, p_star)
            q = np.concatenate([q_tmp, q_2])
            p = np.concatenate([p_tmp, p_2])
            q[3 * i:3 * i + 3] = q_1
            p[3 * i:3 * i + 3] = p_1
            factor = ((-3 / 2.) + np.log(f_s) - BETA.logpdf(F, a, b) + ln_q_dxdy
                      + (dr_sq / (2 * Ks ** 2)) + self.T(p_1, H1) + self.T(p_2, H2) - T_star)
            self.Nobjs += 1
        else:
            n = self.Nobjs
            f_v, x_v, y_v = q_tmp[0::3][:n], q_tmp[1::3][:n], q_tmp[2::3][:n]
            F_m = f_v / (f_v.reshape((n, 1)) + f_v)
            P = BETA.pdf(F_m, a, b)
            P[np.abs(F_m - 0.5) < 1e-6] = 0.              # no self-merging
            R_sq = (x_v.reshape((n, 1)) - x_v) ** 2 + (y_v.reshape((n, 1)) - y_v) ** 2
            P = P * (np.exp(-R_sq / (2. * Ks ** 2)) / (2. * np.pi * Ks ** 2))
            P /= np.sum(P)
            pair = np.random.choice(range(n ** 2), p=P.ravel())
            i1, i2 = pair // n, pair % n
            q_1, p_1 = np.copy(q_tmp[3 * i1:3 * i1 + 3]), np.copy(p_tmp[3 * i1:3 * i1 + 3])
            q_2, p_2 = np.copy(q_tmp[3 * i2:3 * i2 + 3]), np.copy(p_tmp[3 * i2:3 * i2 + 3])
            F = q_1[0] / (q_1[0] + q_2[0])
            dx, dy = q_1[1] - q_2[1], q_1[2] - q_2[2]
            dr_sq = dx ** 2 + dy ** 2
            q_star = np.array([q_1[0] + q_2[0], F * q_1[1] + (1 - F) * q_2[1],
                               F * q_1[2] + (1 - F) * q_2[2]])
            T_1, _ = self._one_star_T(q_1, p_1)
            T_2, _ = self._one_star_T(q_2, p_2)
            H_s = self.H(q_star, grad=False)
            p_star = self.u_sample(3) * np.sqrt(H_s)
            T_star = self.T(p_star, H_s)
            lo, hi = min(i1, i2), max(i1, i2)
            keep = [np.s_[:3 * lo], np.s_[3 * lo + 3:3 * hi], np.s_[3 * hi + 3:]]
            q = np.concatenate([q_tmp[k] for k in keep] + [q_star])
            p = np.concatenate([p_tmp[k] for k in keep] + [p_star])
            factor = ((3 / 2.) - np.log(q_star[0]) + BETA.logpdf(F, a, b) - ln_q_dxdy
                      - (dr_sq / (2 * Ks ** 2)) - T_1 - T_2 + T_star)
            self.Nobjs -= 1
        self.d = 3 * self.Nobjs
        return q, p, factor

    def run_RHMC_batched(self, q_model_0, f_pos=True, delta=1e-6, Niter=100, Nsteps=100,
                         dt=1e-1, counter_max=1000, rng="numpy", seeds=None, seed=0,
                         schedule_g_ff2=None, schedule_beta=None):
        """Many independent chains of run_RHMC's move-0 loop, entirely on the GPU
        (rhmc_mh): Niter+1 MH iterations of Nsteps fused leapfrog steps.
        schedule_g_ff2 / schedule_beta: run_RHMC's schedules
        (sampler_RHMC.py:1010-1016) — iteration l runs with schedule[l] while l
        < its size, then with its last value; afterwards self.g_ff2 / self.beta
        hold the last value applied, as after run_RHMC.

        q_model_0: [n_chains, K, 3] (mag, x, y) or [K, 3] (one chain).
        rng="numpy": host randoms in the reference's per-iteration order
            (randn(d), the move-type uniform, the accept uniform); from the
            global np.random stream (iteration-major, chain-minor) or, with
            seeds=[...], from one RandomState per chain — then chain c equals
            run_RHMC after np.random.seed(seeds[c]).
        rng="device": Philox-4x32-10 on the device, keyed by `seed`.
        Sets q_chain/p-less E/V/T_chain [Niter+1, n_chains(, 3K)], A_chain
        [Niter+1, n_chains] and returns the final q [n_chains, 3K]."""
        q0 = np.array(q_model_0, dtype=np.float64)
        if q0.ndim == 2:
            q0 = q0[None]
        n, K = q0.shape[0], q0.shape[1]
        q0 = q0.copy()
        q0[:, :, 0] = self.mag2flux_converter(q0[:, :, 0])
        q0 = q0.reshape(n, 3 * K)
        self.dt, self.Niter, self.Nsteps, self.Nobjs, self.d = dt, Niter, Nsteps, K, 3 * K
        n_iter = Niter + 1
        z = u = None
        if rng == "numpy":
            z = np.empty((n_iter, n, 3 * K))
            u = np.empty((n_iter, n))
            streams = [np.random.RandomState(s) for s in seeds] if seeds is not None else None
            for l in range(n_iter):
                for c in range(n):
                    r = streams[c] if streams is not None else np.random
                    z[l, c] = r.randn(3 * K)          # u_sample (:1022)
                    r.random_sample()                 # np.random.choice move type (:1046)
                    u[l, c] = r.random_sample()       # np.random.random(1) (:1075)
        elif rng != "device":
            raise ValueError("rng must be 'numpy' or 'device'")
        self._check_geometry()
        out = self._context().mh(self._params(delta, counter_max, for_energy=True), q0, n_iter,
                                 Nsteps, f_pos=f_pos, z=z, u=u, seed=seed, record=True,
                                 schedule_g_ff2=schedule_g_ff2, schedule_beta=schedule_beta)
        for name, sched in (("g_ff2", schedule_g_ff2), ("beta", schedule_beta)):
            if sched is not None and np.size(sched) > 0:        # :1010-1016
                setattr(self, name, float(np.ravel(sched)[min(n_iter, np.size(sched)) - 1]))
        self.q_chain, self.E_chain = out["q_chain"], out["E_chain"]
        self.V_chain, self.T_chain = out["V_chain"], out["T_chain"]
        self.A_chain = out["accept"].astype(bool)
        return out["q"]

    def run_RHMC_rj_batched(self, q_models_0, seeds, f_pos=True, delta=1e-6, Niter=100,
                            Nsteps=100, dt=1e-1, counter_max=1000, N_max=50,
                            P_move=[1., 0., 0.], schedule_g_ff2=None, schedule_beta=None,
                            engine="native", n_threads=0, n_pipes=0, rng_states=None,
                            reuse_records=False):
        """Many independent chains of run_RHMC WITH the reversible-jump moves
        (sampler_RHMC.py:937-1198; birth_death_move :1200-1270, split_merge_move
        :1273-1445), each chain at its own, changing, star count.  Chain c is
        run_RHMC after np.random.seed(seeds[c]): its draws come from its own
        NumPy stream in the reference's order (swapped into the global stream
        around its host work, so the moves' np.random / scipy Beta draws are
        the reference's own), while the GPU work of every phase — V(q) at the
        iteration start, the Nsteps trajectories before and after a jump, V(q')
        — runs batched over the chains, one launch per distinct star count
        (chains grouped by K, so the kernels see ordinary fixed-K batches).

        q_models_0: a list of [K_c, 3] (mag, x, y) arrays, or of the flat
        flux-count q vectors a run returned (taken as they are: a resume); or
        one [n, K, 3] array when every chain starts with K stars (packed in one
        pass, without a Python object per chain).
        Returns a list of the chains' final q; sets q_chain / p_chain [Niter+1, n, 3 N_max],
        E/V/T_chain, A_chain, move_chain, N_chain [Niter+1, n] (iteration-major,
        like run_RHMC_batched).

        engine="native" (default) runs the same algorithm in librhmc_rj.so
        (include/rhmc_rj.h): per-chain host work in C++ on n_threads host
        threads (0: up to 16) with a bit-identical replica of each chain's
        NumPy stream, and flag_chain [Niter+1, n] marks the iterations whose
        proposal was a dead end (see the header); n_pipes = 2..8 (the default:
        2 from 1,024 chains, 3 from 2,048, 4 from 4,096, 8 from 16,384) runs the chains in
        that many parts whose host and GPU phases overlap, 1 in one pass;
        rng_states (native only): the chains' streams to start from instead of
        the seeds — a list of numpy RandomState objects or the rj_rng_states
        array an earlier run left (run it from that run's final q: the draws of
        one uninterrupted run); engine="python" is the NumPy loop below (the
        reference's own draws through np.random)."""
        n = len(q_models_0)
        # any array-like schedule, on either engine (the NumPy loop reads .size)
        if schedule_g_ff2 is not None:
            schedule_g_ff2 = np.ravel(np.asarray(schedule_g_ff2, dtype=np.float64))
        if schedule_beta is not None:
            schedule_beta = np.ravel(np.asarray(schedule_beta, dtype=np.float64))
        if engine == "native":
            if rng_states is None and (seeds is None or len(seeds) != n):
                raise ValueError("one seed per chain")
            return self._rj_native(q_models_0, seeds, f_pos, delta, Niter, Nsteps, dt,
                                   counter_max, N_max, P_move, schedule_g_ff2, schedule_beta,
                                   n_threads, n_pipes, rng_states, reuse_records)
        if engine != "python":
            raise ValueError("engine must be 'native' or 'python'")
        if rng_states is not None:
            raise ValueError("rng_states needs engine='native'")
        if len(seeds) != n:
            raise ValueError("one seed per chain")
        self.dt, self.Niter, self.Nsteps = dt, Niter, Nsteps
        self.P_move, self.N_max = P_move, N_max
        n_it = Niter + 1
        self.q_chain = np.zeros((n_it, n, N_max * 3))
        self.p_chain = np.zeros((n_it, n, N_max * 3))
        self.E_chain, self.V_chain, self.T_chain = (np.zeros((n_it, n)) for _ in range(3))
        self.A_chain = np.zeros((n_it, n), dtype=bool)
        self.move_chain = np.zeros((n_it, n), dtype=int)
        self.N_chain = np.zeros((n_it, n), dtype=int)
        saved = np.random.get_state()
        streams = [np.random.RandomState(s) for s in seeds]   # == np.random.seed(s)
        q = [self._start_q(m) for m in q_models_0]
        p = [None] * n
        move = [0] * n
        grow = [False] * n
        E0 = np.zeros(n)
        factor = np.zeros(n)

        def host(c, fn):               # chain c's stream as the global one (the moves'
            np.random.set_state(streams[c].get_state())   # np.random / scipy draws)
            try:
                return fn()
            finally:
                streams[c].set_state(np.random.get_state())

        def by_k(idx, fn):             # fn(list of chains with one K) per distinct K
            groups = {}
            for c in idx:
                groups.setdefault(q[c].size, []).append(c)
            for cs in groups.values():
                fn(cs)

        def energies(idx):
            out = {}

            def run(cs):
                V = np.atleast_1d(self.V(np.stack([q[c] for c in cs]), f_pos=f_pos))
                out.update(zip(cs, V))
            by_k(idx, run)
            return out

        def trajectories(idx):
            def run(cs):
                qq, pp = self.RHMC_steps(np.stack([q[c] for c in cs]),
                                         np.stack([p[c] for c in cs]), Nsteps, delta=delta,
                                         counter_max=counter_max)
                qq, pp = np.atleast_2d(qq), np.atleast_2d(pp)
                for i, c in enumerate(cs):
                    q[c], p[c] = qq[i], pp[i]
            by_k(idx, run)

        try:
            for l in range(n_it):
                if schedule_g_ff2 is not None and l < schedule_g_ff2.size:
                    self.g_ff2 = schedule_g_ff2[l]
                if schedule_beta is not None and l < schedule_beta.size:
                    self.beta = schedule_beta[l]
                everyone = range(n)
                # momentum, move type and (for a jump) grow/shrink: :1020-1047, :1094
                for c in everyone:
                    r = streams[c]
                    H = self._H_vec(q[c])
                    p[c] = r.randn(q[c].size) * np.sqrt(H)          # u_sample (:1022)
                    move[c] = r.choice([0, 1, 2], p=self.P_move, size=1)[0]
                    grow[c] = (r.choice([True, False], p=[0.5, 0.5]) if move[c] != 0
                               else False)
                    self.T_chain[l, c] = self.T(p[c], H)
                V0 = energies(everyone)
                for c in everyone:
                    d = q[c].size
                    self.V_chain[l, c] = V0[c]
                    E0[c] = self.E_chain[l, c] = V0[c] + self.T_chain[l, c]
                    self.q_chain[l, c, :d], self.p_chain[l, c, :d] = q[c], p[c]
                    self.N_chain[l, c] = d // 3
                    self.move_chain[l, c] = (0 if move[c] == 0 else
                                             (1 if grow[c] else 2) if move[c] == 1 else
                                             (3 if grow[c] else 4))
                trajectories(everyone)
                jump = [c for c in everyone if move[c] != 0]
                for c in jump:                              # :1096-1104, the proposal
                    def propose(c=c):
                        self.Nobjs, self.d = q[c].size // 3, q[c].size
                        mv = self.birth_death_move if move[c] == 1 else self.split_merge_move
                        return mv(q[c], -p[c], grow[c])
                    q[c], p[c], factor[c] = host(c, propose)
                trajectories(jump)
                for c in jump:
                    p[c] = -p[c]
                V1 = energies(everyone)
                for c in everyone:
                    E1 = V1[c] + self.T(p[c], self._H_vec(q[c]))
                    u = np.log(streams[c].random_sample(1))
                    if move[c] == 0:                        # :1075-1083
                        dE = E1 - E0[c]
                        acc = (dE < 0) or (u < -dE)
                    else:                                   # :1160-1181
                        ln_alpha0 = -(E1 - E0[c]) + factor[c]
                        acc = (ln_alpha0 > 0) or (u < ln_alpha0)
                    self.A_chain[l, c] = bool(acc)
                    if not acc:
                        d = 3 * self.N_chain[l, c]
                        q[c] = self.q_chain[l, c, :d].copy()
        finally:
            np.random.set_state(saved)
        self.Nobjs = self.d = None
        return q

    def _start_q(self, m):
        """A chain's start for run_RHMC_rj_batched: [K, 3] (mag, x, y) rows are
        formatted (format_q); a flat q (what the run returns) is used as is."""
        m = np.asarray(m, dtype=np.float64)
        if m.ndim == 1:
            if m.size % 3:
                raise ValueError("a flat q holds 3 values per star")
            return m.copy()
        return self._format_q_fast(m)

    def _rj_native(self, q_models_0, seeds, f_pos, delta, Niter, Nsteps, dt, counter_max, N_max,
                   P_move, schedule_g_ff2, schedule_beta, n_threads, n_pipes=0,
                   rng_states=None, reuse_records=False):
        """run_RHMC_rj_batched through librhmc_rj.so (rhmc_rj_run)."""
        from . import rj_native
        self._check_geometry()
        self.dt, self.Niter, self.Nsteps = dt, Niter, Nsteps
        self.P_move, self.N_max = P_move, N_max
        jumps = P_move[1] != 0 or P_move[2] != 0
        if jumps and (self.alpha is None or self.fmin is None or self.fmax is None):
            assert False                                  # :1205-1207 (prior required)
        # the starts in one native pass: [K, 3] (mag, x, y) rows through format_q's
        # mag2flux (bit-identical to _start_q), flat q vectors (a resume) as they are.
        # With reuse_records the previous run's packed [n][3 N_max] array takes
        # them when nothing else holds it (the returned q views keep it alive)
        qbuf = self.__dict__.get("_rj_qbuf") if reuse_records else None
        kbuf = self.__dict__.get("_rj_kbuf") if reuse_records else None
        if not (isinstance(qbuf, np.ndarray) and sys.getrefcount(qbuf) <= 3):
            qbuf = kbuf = None
        self._rj_qbuf = self._rj_kbuf = None
        if isinstance(q_models_0, np.ndarray) and q_models_0.ndim == 3:
            packed = rj_native.pack_starts(q_models_0, N_max, self.flux_to_count, out=qbuf,
                                           K_prev=kbuf)
            dims = None
        else:
            dims = {np.ndim(m) for m in q_models_0}
        if dims is None:
            pass
        elif dims <= {2}:
            packed = rj_native.pack_starts(q_models_0, N_max, self.flux_to_count, out=qbuf,
                                           K_prev=kbuf)
        elif dims <= {1}:
            packed = rj_native.pack_starts(q_models_0, N_max, out=qbuf, K_prev=kbuf)
        else:
            packed = rj_native.pack_starts([self._start_q(m) for m in q_models_0], N_max,
                                           out=qbuf, K_prev=kbuf)
        qbuf = kbuf = None
        P = self._params(delta, counter_max, for_energy=True)
        # reuse_records (opt-in): the previous run's q_chain / p_chain memory
        # takes this run's records when nothing but this sampler holds it (no
        # caller reference, no view: the attribute, `a` and getrefcount's
        # argument) — fresh arrays of this size cost a page fault per 4 KiB
        # inside the run.  The attributes are detached until the run succeeds,
        # so a failed run leaves None, not half-overwritten records.
        # The q_chain / p_chain records such a run returns are read-only and
        # zero past 3 N_chain in every row, and their int32 star counts stay
        # with them (_rj_nstars): the next run writes only the columns a row
        # can have used (records_zero_padded) instead of all 3 N_max
        out, padded = {}, True
        for key, attr in ((("q_chain", "q_chain"), ("p_chain", "p_chain"),
                           ("E_chain", "E_chain"), ("V_chain", "V_chain"),
                           ("T_chain", "T_chain"), ("flags", "flag_chain"),
                           ("n_stars", "_rj_nstars"),
                           ("states", "rj_rng_states")) if reuse_records else ()):
            a = self.__dict__.get(attr)
            if (isinstance(a, np.ndarray) and a.base is None and sys.getrefcount(a) <= 3
                    and not (key == "states" and rng_states is not None)):
                if key in ("q_chain", "p_chain") and a.flags.writeable:
                    padded = False   # not this path's read-only records: no claim on them
                a.flags.writeable = True
                out[key] = a
                setattr(self, attr, None)
            a = None
        self._rj_nstars = None
        import time
        t0 = time.perf_counter()
        q_end, rec = rj_native.run(
            P, None, seeds, Niter, Nsteps, N_max, P_move, capi.V_FLUX_WALL if f_pos else 0,
            self.num_rows, self.num_cols, self.fmin if jumps else 1., self.fmax if jumps else 1.,
            self.K_split, self.beta_a, self.beta_b, schedule_g_ff2=schedule_g_ff2,
            schedule_beta=schedule_beta, ctx=self._context(), n_threads=n_threads,
            n_pipes=n_pipes, states=(None if rng_states is None else
                                     rng_states if isinstance(rng_states, np.ndarray)
                                     else rj_native.states_from(rng_states)), packed=packed,
            out=out, zero_padded=padded and "n_stars" in out, starts_zero_padded=True)
        out = None
        self.rj_native_s = time.perf_counter() - t0     # the library call (records included)
        n_it = Niter + 1
        for name, sched in (("g_ff2", schedule_g_ff2), ("beta", schedule_beta)):
            if sched is not None and np.size(sched) > 0:    # the value of the last iteration
                setattr(self, name, float(np.ravel(sched)[min(n_it, np.size(sched)) - 1]))
        self.q_chain, self.p_chain = rec["q_chain"], rec["p_chain"]
        self.E_chain, self.V_chain, self.T_chain = rec["E_chain"], rec["V_chain"], rec["T_chain"]
        self.A_chain = rec["accept"].astype(bool)
        self.move_chain = rec["move"].astype(int)
        self.N_chain = rec["n_stars"].astype(int)
        self.flag_chain = rec["flags"]
        self.rj_rng_states = rec["states"]     # every chain's stream at the end (resume)
        if reuse_records:
            self._rj_qbuf, self._rj_kbuf = packed   # final q rows, zero past 3 K
            self._rj_nstars = rec["n_stars"]
            self.q_chain.flags.writeable = False
            self.p_chain.flags.writeable = False
        self.rj_phase_s = dict(zip(("draws", "V0", "steps1", "proposals", "steps2", "V1",
                                    "accept"), rec["phase_s"]))
        self.Nobjs = self.d = None
        return q_end

    def R_accept_report(self, idx_iter, cumulative=True, running=True, run_window=10):
        """sampler_RHMC.py:1447-1473"""
        def rep(A, M):
            for i in range(5):
                b = M == i
                n = np.sum(b)
                if n > 0:
                    a = np.sum(A[b])
                    print("%10s: %.2f%% (%d / %d)" % (self.move_types[i], a / float(n) * 100, a, n))
        if cumulative:
            print("/--Acceptance rate (cumulative)")
            rep(self.A_chain[:idx_iter], self.move_chain[:idx_iter])
        if running:
            print("/--Acceptance rate (running: %d)" % run_window)
            rep(self.A_chain[idx_iter - run_window:idx_iter],
                self.move_chain[idx_iter - run_window:idx_iter])
