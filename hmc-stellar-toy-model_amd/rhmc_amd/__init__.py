"""rhmc_amd — MI355X-native RHMC leapfrog engine for the stellar-photometry
posterior of jaekor91/HMC-stellar-toy-model.

Layout:
  capi        ctypes binding of librhmc.so (the HIP kernels, include/rhmc.h)
  sampler     base_class / single_gym / multi_gym — the reference's
              sampler_RHMC entry points, routed to the GPU
  photometry  host-side input helpers (mag2flux, gauss_PSF, factors, ...)
  workloads   synthetic BASELINE configs C1..C5
"""
from . import capi  # noqa: F401  (fails loudly if librhmc.so is missing)

__all__ = ["capi"]
