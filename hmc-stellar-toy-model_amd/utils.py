"""Drop-in module name for the reference's `from utils import *`: the
photometry helpers the hot path's inputs are built with."""
from rhmc_amd.photometry import (factors, flux2mag, gauss_PSF, gen_pow_law_sample,  # noqa: F401
                                 mag2flux, poisson_realization)
import numpy as np  # noqa: F401
