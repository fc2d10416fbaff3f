"""The reference's flagship run, RHMC-big-sim4.py, as a setup function.

RHMC-big-sim4.py (the reference's largest driver) builds a 32x32 image of
51 stars and runs the reversible-jump sampler from 5 model stars:

  * seed 77 (:18), 32x32 (:19), Nobjs = int(32**2 * 0.05) = 51 true stars and
    Nobjs_model = 5 (:20-21);
  * multi_gym(dt=0, Nsteps=0, g_xx=0.05, g_ff=4, g_ff2=4) (:15), fluxes from
    the power law alpha = 2 on mags [15, 20] (:29-34), positions uniform on
    [1, 31) (:35-38);
  * fmin / fmax, K_split = 1, beta_a = beta_b = 4 (:39-44), the prior on with
    alpha = 2 (:45-47);
  * the model stars from the same law (:58-65), gen_mock_data (:68) and
    gen_noise_profile(N_trial=1000) (:72);
  * run_RHMC(q_model, f_pos=True, delta=1e-6, Niter, Nsteps=10, dt=0.05,
    P_move=[0.6, 0.2, 0.2], N_max=120) (:5-11, :75-77).

`setup()` performs the same calls in the same order on NumPy's global
stream (the draws are the reference's, bit for bit — tests/test_flagship_host.py
checks the image, the stars, the noise histogram and the stream state
against the reference's own run, tests/golden/flagship.npz), so that the
caller's next `gym.run_RHMC(q_model, **RUN_KW)` is the reference's run.
"""
import numpy as np

from .photometry import gen_pow_law_sample
from .sampler import multi_gym

# run_RHMC's arguments in RHMC-big-sim4.py (:5-11, :75-77); Niter is the caller's
# (10000 in the script)
RUN_KW = dict(f_pos=True, delta=1e-6, Nsteps=10, dt=5e-2, P_move=[0.6, 0.2, 0.2], N_max=120)
N_TRUE = int(32 ** 2 * 0.05)
N_MODEL = 5


def setup(seed=77, noise_trials=1000):
    """-> (gym, q_true [51, 3], q_model [5, 3]) with NumPy's global stream
    where RHMC-big-sim4.py leaves it before run_RHMC (mags, not counts)."""
    gym = multi_gym(dt=0., Nsteps=0, g_xx=0.05, g_ff=4., g_ff2=4.)
    np.random.seed(seed)
    gym.num_rows = gym.num_cols = 32
    alpha, mag_max, mag_min = 2., 20., 15.
    fmin = gym.mag2flux_converter(mag_max)
    fmax = gym.mag2flux_converter(mag_min)
    mag = gym.flux2mag_converter(gen_pow_law_sample(alpha, fmin, fmax, N_TRUE))
    q_true = np.zeros((N_TRUE, 3))
    for i in range(N_TRUE):
        x = np.random.random() * (gym.num_rows - 2.) + 1.
        y = np.random.random() * (gym.num_cols - 2.) + 1.
        q_true[i] = np.array([mag[i], x, y])
    gym.fmin, gym.fmax = fmin, fmax
    gym.K_split, gym.beta_a, gym.beta_b = 1., 4., 4.
    gym.use_prior, gym.alpha = True, alpha
    q_model = np.zeros((N_MODEL, 3))
    q_model[:, 0] = gym.flux2mag_converter(gen_pow_law_sample(alpha, fmin, fmax, N_MODEL))
    q_model[:, 1] = np.random.random(size=N_MODEL) * (gym.num_rows - 2.) + 1.
    q_model[:, 2] = np.random.random(size=N_MODEL) * (gym.num_cols - 2.) + 1.
    gym.gen_mock_data(q_true)
    if noise_trials:
        gym.gen_noise_profile(q_true, N_trial=noise_trials)
    return gym, q_true, q_model
