// rhmc_datagen.hpp — device data generation:
//   gen_model     (sampler_RHMC.py:101-116): B + sum_k f_k PSF_k on the full
//                 image, per pixel exactly the reference's expression
//                 exp(-((i+.5-x)^2 + (j+.5-y)^2) / (2 sigma^2)) / (2 pi sigma^2)
//                 (utils.py:475-486), stars added in index order;
//   gen_mock_data (:77-99): a Poisson draw of that image (utils.py:488-496).
// Poisson variates use the same algorithms as NumPy's legacy generator
// (multiplication method below lam = 10, Hormann's PTRS at and above) on a
// Philox-4x32-10 stream keyed by (seed, pixel): same distribution, not the
// same stream — the host path keeps NumPy's stream for parity tests.
#pragma once
#include "rhmc_mh.hpp"
#include "rhmc_wave.hpp"

namespace rhmc {

struct DataArgs {
  const double* q;  // [K][3] flux (counts), x, y
  double* out;      // [rows][cols]
  int K, rows, cols, poisson, n_real;
  unsigned long long seed;
  Consts c;
};

// Sequential uniform stream of one pixel: Philox blocks (pixel, counter).
struct PixelRng {
  unsigned long long seed;
  long long pixel;
  unsigned ctr;
  __device__ double next() {
    const U4 r = philox4x32_10(U4{ctr++, 0x5eedu, (unsigned)pixel, (unsigned)(pixel >> 32)},
                               (unsigned)seed, (unsigned)(seed >> 32));
    return u01(r.x, r.y);  // (0, 1]
  }
};

// log(k!) for the PTRS acceptance test.
__device__ __forceinline__ double log_factorial(double k) { return lgamma(k + 1.0); }

__device__ double poisson_draw(double lam, PixelRng& rng) {
  if (!(lam > 0.0)) return 0.0;
  if (lam < 10.0) {  // multiplication method
    const double enlam = exp(-lam);
    double prod = 1.0;
    double k = 0.0;
    for (int it = 0; it < 1000; ++it) {
      prod *= rng.next();
      if (prod > enlam) k += 1.0;
      else return k;
    }
    return k;
  }
  // PTRS (Hormann 1993), the transformed-rejection sampler NumPy uses
  const double slam = sqrt(lam), loglam = log(lam);
  const double b = 0.931 + 2.53 * slam;
  const double a = -0.059 + 0.02483 * b;
  const double invalpha = 1.1239 + 1.1328 / (b - 3.4);
  const double vr = 0.9277 - 3.6224 / (b - 2.0);
  for (int it = 0; it < 100000; ++it) {
    const double U = rng.next() - 0.5;
    const double V = rng.next();
    const double us = 0.5 - fabs(U);
    const double k = floor((2.0 * a / us + b) * U + lam + 0.43);
    if (us >= 0.07 && V <= vr) return k;
    if (k < 0.0 || (us < 0.013 && V > us)) continue;
    if (log(V) + log(invalpha) - log(a / (us * us) + b) <= -lam + k * loglam - log_factorial(k))
      return k;
  }
  return floor(lam);
}

// One thread per (realisation, pixel); element e = r * rows*cols + pixel is
// also the Philox stream index, so realisation 0 does not depend on n_real.
__global__ void __launch_bounds__(256) datagen_kernel(DataArgs a) {
  const long long npix = (long long)a.rows * a.cols;
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= npix * (a.poisson ? a.n_real : 1)) return;
  const long long pix = e % npix;
  const int i = (int)(pix / a.cols), j = (int)(pix - (long long)i * a.cols);
  const double xv = i + 0.5, yv = j + 0.5;
  double lam = a.c.B;  // np.ones(...) * B_count
  for (int k = 0; k < a.K; ++k) {
    const double f = a.q[3 * k], x = a.q[3 * k + 1], y = a.q[3 * k + 2];
    const double dxv = xv - x, dyv = yv - y;
    const double psf = exp(-(dxv * dxv + dyv * dyv) / a.c.two_sig2) / a.c.psf_norm;
    lam += f * psf;
  }
  if (a.poisson) {
    PixelRng rng{a.seed, e, 0u};
    lam = poisson_draw(lam, rng);
  }
  a.out[e] = lam;
}

}  // namespace rhmc
