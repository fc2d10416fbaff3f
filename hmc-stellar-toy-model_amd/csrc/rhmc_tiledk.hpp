// rhmc_tiledk.hpp — multi-star gradient on small images (C3: 48x48, K = 10).
//
// Same 8 x 8 lane tiling and lane-tiled LDS image as the single-star kernel
// (rhmc_tiled.hpp).  Stars 0..K-1 live in lanes 0..K-1; the template bound
// KMAX >= K pads with phantom stars whose PSF tables are zero (f = 0), so
// every star loop is a compile-time unrolled, branch-free loop.  Per pixel:
//   Lambda = B + sum_k f_k ex_k[row] ey_k[col]        (:373-376)
//   r = D / Lambda,  w_k = psf_k (r - 1)              (:379, :404)
// accumulated per star as a row sum (x moment = sum_rows dx_k[row] * rowsum)
// and a running y moment; the row factors of the lane's current row stay in
// registers, the column factors and offsets are read from the per-wave LDS
// tables.  Three wave all-reduces per star.
#pragma once
#include "rhmc_tiled.hpp"
#include "rhmc_wave.hpp"
#include "rhmc_windowed.hpp"

namespace rhmc {

template <int IMG, int KMAX>
struct TiledK {
  static constexpr int T = IMG / 8;
  static constexpr int NPIX = IMG * IMG;
  static constexpr int TAB = 4 * KMAX * IMG;  // EX, DX, EY, DY: [KMAX][IMG] each
  static_assert(IMG % 8 == 0 && IMG <= 64, "IMG multiple of 8, <= 64");

  static __host__ __device__ constexpr size_t lds_doubles(int waves) {
    return (size_t)NPIX + (size_t)waves * TAB;
  }

  static __device__ __forceinline__ void build_tables(double* tab, int K, double x, double y,
                                                      const LeanConsts& lc) {
    const int lane = lane_id();
    constexpr int per_star = 2 * IMG;
    constexpr int total = KMAX * per_star;
    double* EX = tab;
    double* DX = tab + KMAX * IMG;
    double* EY = tab + 2 * KMAX * IMG;
    double* DY = tab + 3 * KMAX * IMG;
#pragma unroll 1
    for (int m = 0; m < (total + kWave - 1) / kWave; ++m) {
      const int e = lane + kWave * m;
      const int k = min(e / per_star, KMAX - 1);
      const int ks = min(k, K - 1);
      const double xk = __shfl(x, ks, kWave), yk = __shfl(y, ks, kWave);
      if (e < total) {
        const int r = e - k * per_star;
        const int axis = r / IMG, d = r - axis * IMG;
        double val = 0.0, off = 0.0;
        if (k < K) {
          const double c = axis == 0 ? xk : yk;
          const double v = (d + 0.5) - c;
          val = exp(-(v * v) * lc.inv_two_sig2);
          if (axis == 1) val *= lc.inv_norm;
          off = ((double)d - c) + 0.5;
        }
        (axis == 0 ? EX : EY)[k * IMG + d] = val;
        (axis == 0 ? DX : DY)[k * IMG + d] = off;
      }
    }
    wave_lds_sync();
  }

  // dphidq for the wave's chain; lane k < K receives star k's components.
  static __device__ __forceinline__ void gradient(const double* __restrict__ sDl, double* tab,
                                                  int K, double f, double x, double y,
                                                  const Consts& c, const LeanConsts& lc,
                                                  double& gf, double& gx, double& gy) {
    const int lane = lane_id();
    const int ta = lane >> 3, tb = lane & 7;
    build_tables(tab, K, x, y, lc);
    const double* EX = tab;
    const double* DX = tab + KMAX * IMG;
    const double* EY = tab + 2 * KMAX * IMG;
    const double* DY = tab + 3 * KMAX * IMG;

    double fk[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) fk[k] = (k < K) ? bcast(f, k) : 0.0;
    double acc0[KMAX], acc1[KMAX], acc2[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) acc0[k] = acc1[k] = acc2[k] = 0.0;

    // Pixel loops stay rolled: unrolling them lets the compiler hoist every
    // table read of the block and spill (star loops are unrolled instead).
#pragma unroll 1
    for (int ii = 0; ii < T; ++ii) {
      const int row = ta * T + ii;
      double exr[KMAX], rows[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        exr[k] = EX[k * IMG + row];
        rows[k] = 0.0;
      }
#pragma unroll 1
      for (int jj = 0; jj < T; ++jj) {
        const int col = tb * T + jj;
        const double dv = sDl[(ii * T + jj) * 64];
        double psf[KMAX];
        double lam = c.B;
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
          psf[k] = exr[k] * EY[k * IMG + col];
          lam = fma(fk[k], psf[k], lam);                  // (:373-376)
        }
        const double r = fast_div(dv, lam);                // D/Lambda (:379)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
          const double w = fma(psf[k], r, -psf[k]);       // rho * PSF_k
          rows[k] += w;
          acc2[k] = fma(w, DY[k * IMG + col], acc2[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        acc0[k] += rows[k];
        acc1[k] = fma(rows[k], DX[k * IMG + row], acc1[k]);
      }
    }
    gf = gx = gy = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        const double s0 = wave_sum_dpp(acc0[k]);
        const double s1 = wave_sum_dpp(acc1[k]);
        const double s2 = wave_sum_dpp(acc2[k]);
        if (lane == k) {
          gf = -s0;                       // :404
          gx = -s1 * f * lc.inv_var;      // :405
          gy = -s2 * f * lc.inv_var;      // :406
        }
      }
    }
    if (c.use_prior) gf += c.alpha / f;              // :408-409
    if (c.use_Vc) vc_gradient(K, x, y, c, gx, gy);   // :411-418
    gf += metric_flux_term(f, c);                    // :459-463
    wave_lds_sync();
  }
};

}  // namespace rhmc
