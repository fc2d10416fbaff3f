"""Drop-in module name: `from sampler_RHMC import *` (as the reference's
driver scripts do) gets the MI355X-backed base_class / single_gym / multi_gym."""
from rhmc_amd.photometry import *  # noqa: F401,F403
from rhmc_amd.sampler import base_class, multi_gym, single_gym  # noqa: F401
import numpy as np  # noqa: F401
