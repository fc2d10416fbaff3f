// rhmc_windowed.hpp — the large-image / many-star path (C5: 256x256, K = 64).
//
// The reference evaluates every star's PSF on the full image (sampler_RHMC.py
// :373-406), i.e. N_pix*K = 4.2 M terms per gradient at C5.  Here each star's
// PSF is evaluated on a 32 x 32 window: rows floor(x)-16 .. floor(x)+15 (same
// for columns).  Every excluded pixel centre is >= 15.5 px from the star, where
// PSF/peak <= exp(-15.5^2 / (2 sigma^2)) = 2.4e-24 at the reference's
// sigma = 3.5/2.354 px: f*PSF <= 7e-21 for f <= 4e4 (mag 15), far below one
// ulp of Lambda >= B = 25 — the truncated terms do not change Lambda's fp64
// value, and their contribution to the gradient sums is below 1e-20 of them.
//
// Gradient, star-major: for star k (wave-uniform), lane (r = l>>5, c = l&31)
// owns window column c and rows r, r+2, .., r+30 (16 pixels); Lambda at those
// pixels sums over the stars whose windows overlap star k's window (a 64-bit
// neighbour mask built per gradient), in ascending star order like the
// reference; one division per pixel; three wave sums per star.
// D stays in global memory (512 KB at 256x256, L2-resident and shared by all
// chains).  Per-wave LDS: windowed PSF factor tables, 2 x K x 33 doubles.
#pragma once
#include "rhmc_wave.hpp"

namespace rhmc {

constexpr int kWin = 32;         // window side in pixels
constexpr int kWinHalf = 16;     // rows floor(x)-16 .. floor(x)+15
constexpr int kTabW = kWin + 1;  // table row + one zero entry (clamped index)

__host__ __device__ inline size_t win_table_doubles(int K) { return (size_t)2 * K * kTabW; }

struct WinTables {
  double* ex;  // [K][kTabW]  exp(-((i+.5)-x)^2/(2s^2)), i = bx + d
  double* ey;  // [K][kTabW]  same for columns, times 1/(2 pi s^2)
};

// Window origin of a star coordinate; a non-finite or absurd coordinate gets
// an origin far outside any image (empty window).
__device__ __forceinline__ int win_base(double v) {
  if (!(fabs(v) < 1.0e7)) return -(1 << 28);
  return (int)floor(v) - kWinHalf;
}

__device__ __forceinline__ int readlane_i(int v, int src) {
  return __builtin_amdgcn_readlane(v, src);
}

__device__ __forceinline__ unsigned long long readlane_u64(unsigned long long v, int src) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, src);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), src);
  return ((unsigned long long)hi << 32) | lo;
}

// Windowed PSF factor tables for K stars (lane k < K holds star k); the
// entries are flattened over (star, axis, index) so all 64 lanes work.
__device__ __forceinline__ void win_build_tables(const WinTables& t, int K, double x, double y,
                                                 int bx, int by, const LeanConsts& lc) {
  const int lane = lane_id();
  const int per_star = 2 * kTabW;
  const int total = K * per_star;
  const int iters = (total + kWave - 1) / kWave;
  for (int m = 0; m < iters; ++m) {  // uniform trip count: shuffles see all lanes
    const int e = lane + kWave * m;
    const int k = min(e / per_star, K - 1);
    const double xk = __shfl(x, k, kWave), yk = __shfl(y, k, kWave);
    const int bxk = __shfl(bx, k, kWave), byk = __shfl(by, k, kWave);
    if (e < total) {
      const int r = e - k * per_star;
      const int axis = r / kTabW, d = r - axis * kTabW;
      double val = 0.0;
      if (d < kWin) {
        if (axis == 0) {
          const double v = ((double)(bxk + d) + 0.5) - xk;
          val = exp(-(v * v) * lc.inv_two_sig2);
        } else {
          const double v = ((double)(byk + d) + 0.5) - yk;
          val = exp(-(v * v) * lc.inv_two_sig2) * lc.inv_norm;
        }
      }
      (axis == 0 ? t.ex : t.ey)[k * kTabW + d] = val;
    }
  }
  wave_lds_sync();
}

// Lane k: bit j set when star j's window overlaps star k's window.
__device__ __forceinline__ unsigned long long win_neighbours(int K, int bx, int by) {
  unsigned long long m = 0ull;
  for (int j = 0; j < K; ++j) {
    const int bxj = readlane_i(bx, j), byj = readlane_i(by, j);
    if (abs(bx - bxj) < kWin && abs(by - byj) < kWin) m |= 1ull << j;
  }
  return m;
}

// Repulsion gradient (sampler_RHMC.py:411-418), lanes = stars.
__device__ __forceinline__ void vc_gradient(int K, double x, double y, const Consts& c,
                                            double& gx, double& gy) {
  double sx = 0.0, sy = 0.0;
  for (int jj = 0; jj < K; ++jj) {
    const double X = bcast(x, jj), Y = bcast(y, jj);
    const double ddx = X - x, ddy = Y - y;
    double R = sqrt(ddx * ddx + ddy * ddy);
    if (fabs(R) < 1e-10) R = 1e32;
    const double tr = pow(1.0 / R, c.vc_pow + 2.0);
    sx += tr * ddx;
    sy += tr * ddy;
  }
  gx += c.beta * sx * c.vc_pow;
  gy += c.beta * sy * c.vc_pow;
}

// dVdq (+ dphidq metric term) of the wave's chain; lane k < K gets star k's.
__device__ void win_gradient(const double* __restrict__ D, const WinTables& t, int K, double f,
                             double x, double y, int rows, int cols, const Consts& c,
                             const LeanConsts& lc, bool with_metric, double& gf, double& gx,
                             double& gy) {
  const int lane = lane_id();
  const int bx = win_base(x), by = win_base(y);
  win_build_tables(t, K, x, y, bx, by, lc);
  const unsigned long long nb = win_neighbours(K, bx, by);
  const int lrow = lane >> 5, lcol = lane & 31;
  gf = gx = gy = 0.0;

  for (int k = 0; k < K; ++k) {
    const double xk = bcast(x, k), fk = bcast(f, k);
    const int bxk = readlane_i(bx, k), byk = readlane_i(by, k);
    const unsigned long long mk = readlane_u64(nb, k);
    const int j = byk + lcol;
    const bool colok = (unsigned)j < (unsigned)cols;

    double lam[16], psk[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      lam[s] = c.B;
      psk[s] = 0.0;
    }
    // Lambda = B + sum_{stars overlapping this window} f PSF, ascending order (:373-376)
    unsigned long long mm = mk;
    while (mm) {
      const int kk = __builtin_ctzll(mm);
      mm &= mm - 1;
      const double fkk = bcast(f, kk);
      const int bxkk = readlane_i(bx, kk), bykk = readlane_i(by, kk);
      const unsigned v = min((unsigned)(j - bykk), (unsigned)kWin);
      const double eyv = t.ey[kk * kTabW + v];
      const double* exrow = t.ex + kk * kTabW;
      const int u0 = bxk + lrow - bxkk;
      if (kk == k) {
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const unsigned u = min((unsigned)(u0 + 2 * s), (unsigned)kWin);
          const double p = exrow[u] * eyv;
          psk[s] = p;
          lam[s] = fma(fkk, p, lam[s]);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const unsigned u = min((unsigned)(u0 + 2 * s), (unsigned)kWin);
          lam[s] = fma(fkk, exrow[u] * eyv, lam[s]);
        }
      }
    }
    // rho * PSF_k and its three moments over this lane's 16 pixels
    double a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int s = 0; s < 16; s += 2) {
      const int i1 = bxk + lrow + 2 * s, i2 = i1 + 2;
      const bool ok1 = colok && (unsigned)i1 < (unsigned)rows;
      const bool ok2 = colok && (unsigned)i2 < (unsigned)rows;
      const double d1 = ok1 ? D[(size_t)i1 * cols + j] : 0.0;
      const double d2 = ok2 ? D[(size_t)i2 * cols + j] : 0.0;
      const double l1 = lam[s], l2 = lam[s + 1];
      const double L = l1 * l2;
      double r = __builtin_amdgcn_rcp(L);
      r = fma(r, fma(-L, r, 1.0), r);
      const double r1 = l2 * r, r2 = l1 * r;
      double q1 = d1 * r1, q2 = d2 * r2;
      q1 = fma(r1, fma(-l1, q1, d1), q1);
      q2 = fma(r2, fma(-l2, q2, d2), q2);
      const double p1 = ok1 ? psk[s] : 0.0, p2 = ok2 ? psk[s + 1] : 0.0;
      const double w1 = fma(p1, q1, -p1), w2 = fma(p2, q2, -p2);
      a0 += w1;
      a1 = fma(w1, ((double)i1 - xk) + 0.5, a1);
      a0 += w2;
      a1 = fma(w2, ((double)i2 - xk) + 0.5, a1);
    }
    const double yk = bcast(y, k);
    const double a2 = a0 * (((double)j - yk) + 0.5);  // the lane's column is fixed
    const double s0 = wave_sum_dpp(a0);
    const double s1 = wave_sum_dpp(a1);
    const double s2 = wave_sum_dpp(a2);
    if (lane == k) {
      gf = -s0;                      // :404
      gx = -s1 * fk * lc.inv_var;    // :405
      gy = -s2 * fk * lc.inv_var;    // :406
    }
  }
  if (c.use_prior) gf += c.alpha / f;               // :408-409
  if (c.use_Vc) vc_gradient(K, x, y, c, gx, gy);    // :411-418
  if (with_metric) gf += metric_flux_term(f, c);    // :459-463
  wave_lds_sync();
}

// V of the wave's chain on a large image (sampler_RHMC.py:294-351), pixel-major:
// image row i (uniform), lanes over columns; only the stars whose window rows
// contain i contribute (ballot over the star lanes).
__device__ double win_potential(const double* __restrict__ D, const WinTables& t, int K,
                                double f, double x, double y, int rows, int cols,
                                const Consts& c, const LeanConsts& lc) {
  const int lane = lane_id();
  const bool owner = lane < K;
  const int bx = win_base(x), by = win_base(y);
  win_build_tables(t, K, x, y, bx, by, lc);
  double v = 0.0;
  for (int i = 0; i < rows; ++i) {
    unsigned long long rm = __ballot(owner && bx <= i && i < bx + kWin);
    for (int cb = 0; cb < cols; cb += kWave) {
      const int j = cb + lane;
      if (j < cols) {
        double lam = c.B;
        unsigned long long mm = rm;
        while (mm) {
          const int kk = __builtin_ctzll(mm);
          mm &= mm - 1;
          const double fkk = bcast(f, kk);
          const int u = i - readlane_i(bx, kk);
          const unsigned vv = min((unsigned)(j - readlane_i(by, kk)), (unsigned)kWin);
          lam = fma(fkk, t.ex[kk * kTabW + u] * t.ey[kk * kTabW + vv], lam);
        }
        v += lam - D[(size_t)i * cols + j] * log(lam);
      }
    }
  }
  wave_lds_sync();
  return wave_sum_dpp(v);
}

}  // namespace rhmc
