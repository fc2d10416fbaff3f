"""Drop-in module name: `from samplers import *` (as the reference's older
driver scripts do) gets the MI355X-backed lightsource_gym (HMC_random)."""
from rhmc_amd.photometry import *  # noqa: F401,F403
from rhmc_amd.samplers import lightsource_gym  # noqa: F401
import numpy as np  # noqa: F401
