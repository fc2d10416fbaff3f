"""The reference's older `samplers` API on the sampling path, routed to the
MI355X engine: `lightsource_gym` with unit-mass HMC (`HMC_random`).

Mirrors jaekor91/HMC-stellar-toy-model `samplers.py` (file:line per method):
same class name, attributes (set after construction, like the reference's
scripts: `gym.Nobjs`, `gym.d = 3 * Nobjs`, `gym.dt = <vector [d]>`), method
names, argument meaning, global-NumPy-RNG draw order and results.

What runs where:
  * dVdq, V and the HMC_random trajectories run in librhmc.so
    (rhmc_gradient kind 0, rhmc_energy without the position check,
    rhmc_hmc_random).  No CPU fallback.
  * E, K, p_sample and the MH bookkeeping stay on the host (NumPy), like the
    reference.

Quirks kept on purpose (samplers.py:519-552): the flux-wall flip mask is
never cleared inside a trajectory, and a trajectory whose last step flipped
is evaluated with the momentum it started from.  HMC_random requires
Nchain == 1 (assert, like the reference); HMC_random_batched runs many chains
at once and, with one chain, draws exactly what HMC_random draws.

Out of scope: find_peaks / HMC_find_best_dt (seed and step-size
search), RHMC_random_diag / RHMC_random, the GMM testbed and the plots.
"""
import numpy as np

from . import capi
from .photometry import default_exp_setup, gauss_PSF, mag2flux, poisson_realization


class lightsource_gym(object):
    """samplers.py:3-43."""

    def __init__(self):
        self._D = None
        self._ctx = None
        self._ctx_shape = None
        self.M = None
        (self.num_rows, self.num_cols, self.flux_to_count, self.PSF_FWHM_pix,
         self.B_count, self.arcsec_to_pix, self.mB, _) = default_exp_setup()
        self.Nchain = None
        self.Niter = None
        self.thin_rate = None
        self.Nwarmup = None
        self.q_chain = None
        self.p_chain = None
        self.V_chain = None
        self.E_chain = None
        self.dE_chain = None
        self.A_chain = None
        self.dt = None           # per-coordinate step vector [d]
        self.Nobjs = None
        self.d = None
        self.f_lim = 0.
        self.q_seed = None
        self.device = 0

    # ---------------------------------------------------------------- data
    @property
    def D(self):
        return self._D

    @D.setter
    def D(self, value):
        self._D = None if value is None else np.ascontiguousarray(value, dtype=np.float64)
        self._ctx_shape = None

    def _context(self):
        if self._D is None:
            raise ValueError("no data image: call gen_mock_data() or set .D first")
        if self._D.shape != (self.num_rows, self.num_cols):
            raise ValueError("D has shape %s but num_rows/num_cols are %d/%d"
                             % (self._D.shape, self.num_rows, self.num_cols))
        if self._ctx is None:
            self._ctx = capi.Context(self._D, device=self.device)
        elif self._ctx_shape is None:
            self._ctx.set_image(self._D)
        self._ctx_shape = self._D.shape
        return self._ctx

    def _params(self, dt=1.0):
        # Only B, the PSF width and f_lim are read by the kernels used here;
        # the metric constants are placeholders (unit metric).
        return capi.make_params(
            dt=dt, delta=1e-6, counter_max=1000, B_count=self.B_count, f_lim=self.f_lim,
            f_low=mag2flux(self.mB + 2) * self.flux_to_count, fwhm_pix=self.PSF_FWHM_pix,
            g_xx=1., g_ff=1., g_ff2=1., g0=1., g1=1., g2=1., use_prior=False, alpha=2.,
            use_Vc=False, beta=1., Vc_r_pow=1., V_prior_const=0.)

    def gen_mock_data(self, q_true=None, return_data=False):
        """samplers.py:44-67: q_true (Nobjs, 3) = (f counts, x, y); the global
        NumPy RNG draws the Poisson realisation (bit-identical data)."""
        data = np.ones((self.num_rows, self.num_cols), dtype=float) * self.B_count
        for i in range(q_true.shape[0]):
            f, x, y = q_true[i]
            data += f * gauss_PSF(self.num_rows, self.num_cols, x, y, FWHM=self.PSF_FWHM_pix)
        data = poisson_realization(data)
        if return_data:
            return data
        self.D = data

    # ------------------------------------------------------------ potential
    def dVdq(self, objs_flat):
        """samplers.py:1108-1135 on the GPU (rhmc_gradient kind 0)."""
        return self._context().gradient(self._params(), objs_flat, kind=0)

    def V(self, objs_flat):
        """samplers.py:1137-1150 on the GPU: -sum(D ln Lambda - Lambda), no
        prior, no position check."""
        return self._context().energy(self._params(), objs_flat, None, f_pos=False,
                                      pos_check=False)[0]

    def E(self, q, p, mass_matrix=None):
        """samplers.py:1152-1161."""
        Nobjs = q.size // 3
        for l in range(Nobjs):
            if q[3 * l] < self.f_lim:
                return np.inf
        return self.V(q) + self.K(p, mass_matrix)

    def K(self, p, mass_matrix=None):
        """samplers.py:1163-1175."""
        if mass_matrix is None:
            return np.dot(p, p) / 2.
        return (np.sum(p ** 2 / mass_matrix) + np.log(np.abs(np.prod(mass_matrix)))) / 2.

    def p_sample(self):
        """samplers.py:1177-1181."""
        return np.random.randn(self.d)

    def leap_frog(self, p_old, q_old, dt):
        """samplers.py:1183-1191."""
        p_half = p_old - dt * self.dVdq(q_old) / 2.
        q_new = q_old + dt * p_half
        p_new = p_half - dt * self.dVdq(q_new) / 2.
        return p_new, q_new

    # ------------------------------------------------------------- sampling
    def _trajectories(self, q, p, steps):
        """Batched samplers.py:519-552 on the GPU (rhmc_hmc_random)."""
        dt = np.ascontiguousarray(np.broadcast_to(np.asarray(self.dt, np.float64), (self.d,)))
        return self._context().hmc_random(self._params(), dt, q, p,
                                          np.asarray(steps, np.int32))

    def _set_f_lim(self, f_lim, f_lim_default):
        if f_lim_default:
            self.f_lim = mag2flux(self.mB - 1.) * self.flux_to_count
        else:
            self.f_lim = f_lim

    def HMC_random(self, q_model_0=None, Nchain=1, Niter=1000, thin_rate=0, Nwarmup=0,
                   steps_min=10, steps_max=50, f_lim=0., f_lim_default=False):
        """samplers.py:460-572.  Sets q_chain [1, Niter+1, d], E_chain,
        dE_chain [1, Niter+1, 1] and A_chain [1, Niter, 1]."""
        assert Nchain == 1  # Currently we do not support any other.
        self.Nchain = Nchain
        self.Niter = Niter
        self.thin_rate = thin_rate
        self.Nwarmup = Nwarmup
        assert self.d is not None
        self._set_f_lim(f_lim, f_lim_default)
        if q_model_0 is None:
            print("Use found seeds for inference.")
            q_model_0 = self.q_seed
        q_model_0 = np.asarray(q_model_0, dtype=float).reshape((self.d,))
        self._run(q_model_0[None, :], Niter, steps_min, steps_max)
        print("Chain %d Acceptance rate: %.2f%%"
              % (0, np.sum(self.A_chain[0, :] * 100) / float(self.Niter)))

    def HMC_random_batched(self, q_model_0, Niter=1000, steps_min=10, steps_max=50, f_lim=0.,
                           f_lim_default=False):
        """HMC_random over many independent chains at once (q_model_0
        [Nchain, d]); per iteration the global NumPy RNG draws randn(Nchain, d),
        randint(steps_min, steps_max, Nchain) and random(Nchain) — with one
        chain exactly the reference's draws."""
        assert self.d is not None
        self._set_f_lim(f_lim, f_lim_default)
        q0 = np.asarray(q_model_0, dtype=float).reshape(-1, self.d)
        self.Nchain = q0.shape[0]
        self.Niter = Niter
        self._run(q0, Niter, steps_min, steps_max)

    def _E_batch(self, q, p):
        V = self._context().energy(self._params(), q, None, f_pos=False, pos_check=False)[0]
        E = V + np.sum(p * p, axis=1) / 2.
        E[(q[:, 0::3] < self.f_lim).any(axis=1)] = np.inf
        return E

    def _run(self, q0, Niter, steps_min, steps_max):
        n, d = q0.shape
        self.q_chain = np.zeros((n, Niter + 1, d))
        self.E_chain = np.zeros((n, Niter + 1, 1))
        self.dE_chain = np.zeros((n, Niter + 1, 1))
        self.A_chain = np.zeros((n, Niter, 1))
        self.q_chain[:, 0, :] = q0
        p_initial = np.random.randn(n, d)
        self.E_chain[:, 0, 0] = self._E_batch(q0, p_initial)
        E_previous = self.E_chain[:, 0, 0].copy()
        q_tmp = q0.copy()
        for i in range(1, Niter + 1):
            q_initial = q_tmp
            p_tmp = np.random.randn(n, d)
            E_initial = self._E_batch(q_tmp, p_tmp)
            self.E_chain[:, i, 0] = E_initial
            self.dE_chain[:, i, 0] = E_initial - E_previous
            steps = np.random.randint(low=steps_min, high=steps_max, size=n)
            q_new, p_new = self._trajectories(q_tmp, p_tmp, steps)
            E_final = self._E_batch(q_new, p_new)
            with np.errstate(invalid="ignore"):
                dE = E_final - E_initial
            E_previous = E_initial
            lnu = np.log(np.random.random(n))
            with np.errstate(invalid="ignore"):
                acc = (dE < 0) | (lnu < -dE)
            self.A_chain[:, i - 1, 0] = acc
            q_tmp = np.where(acc[:, None], q_new, q_initial)
            self.q_chain[:, i, :] = q_tmp
