// rhmc_kernels.hip — MI355X (gfx950) kernels of the RHMC leapfrog engine and
// the C-ABI declared in include/rhmc.h.
//
// Work decomposition: one wave64 per chain; a workgroup of W waves shares the
// data image D, staged once into LDS with coalesced loads.  After that single
// workgroup barrier every wave runs its chain independently (only wave-local
// LDS hand-offs), n_steps steps fused in one launch with (q, p) in registers.
//
// Per gradient evaluation (the inner loop, sampler_RHMC.py:365-425):
//   * the Gaussian PSF is separable: PSF[i][j] = ex[i]*ey[j] with
//     ex[i] = exp(-((i+.5)-x)^2/(2s^2)), ey[j] = exp(-((j+.5)-y)^2/(2s^2))/(2 pi s^2)
//     -> (R + C) exps per star instead of R*C (utils.py:475-486);
//   * the per-wave LDS tables hold ex, ey and the offsets (i-x)+.5, (j-y)+.5;
//   * lane l owns pixels l, l+64, ...: Lambda = B + sum_k f_k psf_k,
//     w_k = psf_k*(D/Lambda - 1), three running sums per star;
//   * one butterfly all-reduce per sum.
// The end-of-step gradient (sampler_RHMC.py:551) is evaluated at the same q
// as the next step's first one (:525) — reflection only flips p — so it is
// carried over: one gradient per step, bit-identical to recomputing it.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rhmc.h"
#ifndef RHMC_KERNELS_ONLY  // (their non-template kernels belong to this unit only)
#include "rhmc_datagen.hpp"
#include "rhmc_mh.hpp"
#endif
#include "rhmc_tiledl.hpp"
#include "rhmc_tiledr.hpp"
#include "rhmc_tiledrk.hpp"
#ifndef RHMC_KERNELS_ONLY
#include "rhmc_mhk1.hpp"
#include "rhmc_mhpk.hpp"
#endif
#include "rhmc_pixk.hpp"
#include "rhmc_wave.hpp"
#include "rhmc_windowed.hpp"
#include "rhmc_dense.hpp"
#ifndef RHMC_KERNELS_ONLY
#include "rhmc_rows.hpp"
#endif

namespace rhmc {

struct Geometry {
  int rows, cols, npix, npl;  // npl = ceil(npix / 64) pixels per lane
  int di, dj;                 // pixel index step of 64 as (rows, cols)
  double* work;               // WinGG's per-chain factor tables (from 65 stars), else null
};

struct Tables {  // per-wave LDS tables, K stars
  double* ex;  // [K][rows]
  double* dx;  // [K][rows]
  double* ey;  // [K][cols]  (carries 1/(2 pi s^2))
  double* dy;  // [K][cols]
};

__device__ __forceinline__ Tables carve_tables(double* base, int K, const Geometry& g) {
  Tables t;
  t.ex = base;
  t.dx = base + K * g.rows;
  t.ey = base + 2 * K * g.rows;
  t.dy = base + 2 * K * g.rows + K * g.cols;
  return t;
}

__host__ __device__ inline size_t table_doubles(int K, int rows, int cols) {
  return (size_t)2 * K * (rows + cols);
}

// Build the separable PSF tables of K stars (lane k < K holds star k).
__device__ __forceinline__ void build_tables(const Tables& t, int K, double x, double y,
                                             const Geometry& g, const Consts& c) {
  const int lane = lane_id();
  const int span = g.rows + g.cols;
  for (int k = 0; k < K; ++k) {
    const double xk = bcast(x, k), yk = bcast(y, k);
    for (int e = lane; e < span; e += kWave) {
      if (e < g.rows) {
        const double v = (e + 0.5) - xk;
        t.ex[k * g.rows + e] = exp(-(v * v) / c.two_sig2);
        t.dx[k * g.rows + e] = ((double)e - xk) + 0.5;
      } else {
        const int j = e - g.rows;
        const double v = (j + 0.5) - yk;
        t.ey[k * g.cols + j] = exp(-(v * v) / c.two_sig2) / c.psf_norm;
        t.dy[k * g.cols + j] = ((double)j - yk) + 0.5;
      }
    }
  }
  wave_lds_sync();
}

// dVdq (optionally + the dphidq metric term) for the chain of this wave.
// Returns lane k's (g_f, g_x, g_y) for k < K; other lanes get junk.
template <int MAXK>
__device__ void gradient(const double* __restrict__ sD, const Tables& t, int K, double f,
                         double x, double y, const Geometry& g, const Consts& c,
                         bool with_metric, double& gf, double& gx, double& gy) {
  const int lane = lane_id();
  build_tables(t, K, x, y, g, c);

  double fk[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) fk[k] = (k < K) ? bcast(f, k) : 0.0;

  double acc[MAXK][3];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) acc[k][0] = acc[k][1] = acc[k][2] = 0.0;

  int i = lane / g.cols, j = lane - (lane / g.cols) * g.cols;
  for (int tt = 0; tt < g.npl; ++tt) {
    const int pix = lane + kWave * tt;
    if (pix < g.npix) {
      const double dv = sD[pix];
      double psf[MAXK];
      double lam = c.B;  // Lambda = B + sum_k f_k PSF_k (:373-376)
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        if (k < K) {
          psf[k] = t.ex[k * g.rows + i] * t.ey[k * g.cols + j];
          lam = fma(fk[k], psf[k], lam);
        }
      }
      const double r = dv / lam;  // rho + 1 = D/Lambda (:379)
#pragma unroll
      for (int k = 0; k < MAXK; ++k) {
        if (k < K) {
          const double w = fma(psf[k], r, -psf[k]);  // rho * PSF
          acc[k][0] += w;
          acc[k][1] = fma(w, t.dx[k * g.rows + i], acc[k][1]);
          acc[k][2] = fma(w, t.dy[k * g.cols + j], acc[k][2]);
        }
      }
    }
    j += g.dj;
    i += g.di;
    if (j >= g.cols) {
      j -= g.cols;
      ++i;
    }
  }

  gf = gx = gy = 0.0;
#pragma unroll
  for (int k = 0; k < MAXK; ++k) {
    if (k < K) {
      const double s0 = wave_sum(acc[k][0]);
      const double s1 = wave_sum(acc[k][1]);
      const double s2 = wave_sum(acc[k][2]);
      // K == 1: every lane mirrors star 0, so the chain state stays
      // wave-uniform and the fixed-point loops never diverge.
      if (MAXK == 1 || lane == k) {
        gf = -s0;
        gx = -s1 * f / c.var;
        gy = -s2 * f / c.var;
      }
    }
  }
  if (c.use_prior) gf += c.alpha / f;  // :408-409
  if (c.use_Vc) {                      // :411-418 (O(K^2), lanes = stars)
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
  if (with_metric) gf += metric_flux_term(f, c);  // dphidq (:459-463)
  // Tables are rebuilt by the next gradient call; make sure every lane has
  // finished reading before they are overwritten.
  wave_lds_sync();
}

struct LeapArgs {
  double* q;
  double* p;
  int32_t* fp_iters;
  int32_t* status;
  const double* D;
  int64_t n_chains;
  int K, n_steps;
  Geometry g;
  Consts c;
  // ragged sets (rhmc_leapfrog_ragged_device, the slotted kernels only): chain
  // i is row rows[i] (NULL: row i) of [*][ld] arrays with Kc[row] stars; K is
  // then the largest star count of the launch (it sizes LDS).  Kc NULL: every
  // chain has K stars in rows of 3K.
  const int32_t* Kc = nullptr;
  const int64_t* rows = nullptr;
  int64_t ld = 0;
};

// Row, star count and row stride of launch chain i (LeapArgs / EnergyArgs).
template <class A>
__device__ __forceinline__ void chain_row(const A& a, int64_t i, int64_t& row, int& K,
                                          int64_t& ld) {
  row = a.rows ? a.rows[i] : i;
  K = a.Kc ? a.Kc[row] : a.K;
  ld = a.Kc ? a.ld : 3 * (int64_t)K;
}

// Stage D into LDS (coalesced, whole workgroup) and return this wave's chain.
__device__ __forceinline__ int64_t stage_image(double* sD, const double* __restrict__ D,
                                               int npix, int waves_per_wg) {
  for (int e = threadIdx.x; e < npix; e += blockDim.x) sD[e] = D[e];
  __syncthreads();
  return (int64_t)blockIdx.x * waves_per_wg + (threadIdx.x / kWave);
}

// Chain state of one wave: lane k < K owns star k (UNIFORM: K == 1 and every
// lane mirrors star 0, so no cross-lane reduction is needed).
struct StarState {
  double f, x, y, pf, px, py;
};

// n_steps implicit generalized-leapfrog steps (sampler_RHMC.py:522-566) with a
// single gradient call site: the end-of-step gradient (:551) is the next
// step's opening one (:525).  `grad(f, x, y, gf, gx, gy)` returns dphidq.
template <bool UNIFORM, class Grad>
__device__ __forceinline__ void run_steps(StarState& s, bool owner, int n_steps, int rows,
                                          int cols, const Consts& c, int& it_p, int& it_q,
                                          unsigned& st, Grad grad) {
  const double hdt = c.hdt;
  for (int step = 0;; ++step) {
    double gf, gx, gy;
    grad(s.f, s.x, s.y, gf, gx, gy);
    if (step > 0) {
      // (5) closing half kick of the previous step (:551), (6) reflection (:554-564)
      s.pf = s.pf - hdt * gf;
      s.px = s.px - hdt * gx;
      s.py = s.py - hdt * gy;
      if (s.f < c.f_lim) {
        s.pf = -s.pf;
        st |= RHMC_STATUS_REFLECT_F;
        if (s.f >= c.near_f) st |= RHMC_STATUS_NEAR_WALL;
      }
      if (s.x < 0.0 || s.x > (double)(rows - 1)) {
        s.px = -s.px;
        st |= RHMC_STATUS_REFLECT_XY;
        if (near_edge(s.x, (double)(rows - 1))) st |= RHMC_STATUS_NEAR_WALL;
      }
      if (s.y < 0.0 || s.y > (double)(cols - 1)) {
        s.py = -s.py;
        st |= RHMC_STATUS_REFLECT_XY;
        if (near_edge(s.y, (double)(cols - 1))) st |= RHMC_STATUS_NEAR_WALL;
      }
    }
    if (step == n_steps) break;
    // (1) opening half kick (:525)
    s.pf = s.pf - hdt * gf;
    s.px = s.px - hdt * gx;
    s.py = s.py - hdt * gy;
    // (2) p fixed point, flux slots only (:528-535); x/y slots change by 0
    {
      const double coef = dtaudq_coef(s.f, c);
      const double rho = s.pf;
      double dp;
      int n = 0;
      do {
        const double pp = rho - hdt * ((s.pf * s.pf) * coef / 2.0);
        const double d = (UNIFORM || owner) ? fabs(s.pf - pp) : 0.0;
        dp = UNIFORM ? d : wave_nanmax(d);
        s.pf = pp;
        ++n;
      } while (dp > c.delta && n < c.counter_max);
      it_p += n;
      if (dp > c.delta) st |= RHMC_STATUS_PLOOP_CAP;
    }
    // (3) q fixed point (:538-545): q' = sig + dt/2 (p/H(sig) + p/H(q))
    {
      const double sf = s.f, sx = s.x, sy = s.y;
      const double hff0 = H_ff(sf, c), hxx0 = H_xx(sf, c);
      const double af = s.pf / hff0, ax = s.px / hxx0, ay = s.py / hxx0;
      double dq;
      int n = 0;
      do {
        const double hff = H_ff(s.f, c), hxx = H_xx(s.f, c);
        const double nf = sf + hdt * (af + s.pf / hff);
        const double nx = sx + hdt * (ax + s.px / hxx);
        const double ny = sy + hdt * (ay + s.py / hxx);
        double d = nanmax2(nanmax2(fabs(s.f - nf), fabs(s.x - nx)), fabs(s.y - ny));
        d = (UNIFORM || owner) ? d : 0.0;
        dq = UNIFORM ? d : wave_nanmax(d);
        s.f = nf;
        s.x = nx;
        s.y = ny;
        ++n;
      } while (dq > c.delta && n < c.counter_max);
      it_q += n;
      if (dq > c.delta) st |= RHMC_STATUS_QLOOP_CAP;
    }
    // (4) p -= dt/2 dtaudq(q, p) (:548)
    s.pf = s.pf - hdt * ((s.pf * s.pf) * dtaudq_coef(s.f, c) / 2.0);
  }
}

__device__ __forceinline__ StarState load_chain(const LeapArgs& a, int64_t chain, int K,
                                                bool owner, int64_t& base) {
  base = chain * 3 * (int64_t)K + 3 * (owner ? lane_id() : 0);
  StarState s;
  s.f = a.q[base];
  s.x = a.q[base + 1];
  s.y = a.q[base + 2];
  s.pf = a.p[base];
  s.px = a.p[base + 1];
  s.py = a.p[base + 2];
  return s;
}

__device__ __forceinline__ void store_chain(const LeapArgs& a, int64_t chain, int64_t base,
                                            bool owner, const StarState& s, int it_p, int it_q,
                                            unsigned st) {
  if (owner) {
    if (!(isfinite(s.f) && isfinite(s.x) && isfinite(s.y) && isfinite(s.pf) &&
          isfinite(s.px) && isfinite(s.py)))
      st |= RHMC_STATUS_NONFINITE;
    a.q[base] = s.f;
    a.q[base + 1] = s.x;
    a.q[base + 2] = s.y;
    a.p[base] = s.pf;
    a.p[base + 1] = s.px;
    a.p[base + 2] = s.py;
  }
  // OR the star lanes' status bits
  unsigned all = owner ? st : 0u;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) all |= (unsigned)__shfl_xor((int)all, m, kWave);
  if (lane_id() == 0) {
    if (a.status) a.status[chain] = (int32_t)all;
    if (a.fp_iters) {
      a.fp_iters[2 * chain] = it_p;
      a.fp_iters[2 * chain + 1] = it_q;
    }
  }
}

// Generic kernel: image in LDS, K <= MAXK <= 16, reference-form metric.
template <int MAXK>
__global__ void __launch_bounds__(256) leapfrog_kernel(LeapArgs a) {
  extern __shared__ double lds[];
  const Geometry& g = a.g;
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  double* sD = lds;
  const int64_t chain = stage_image(sD, a.D, g.npix, W);
  if (chain >= a.n_chains) return;
  const int K = a.K;
  const Tables tab = carve_tables(
      lds + g.npix + (threadIdx.x / kWave) * table_doubles(K, g.rows, g.cols), K, g);
  const bool owner = lane_id() < K;
  int64_t base;
  StarState s = load_chain(a, chain, K, owner, base);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  run_steps<MAXK == 1>(s, owner, a.n_steps, g.rows, g.cols, c, it_p, it_q, st,
                       [&](double f, double x, double y, double& gf, double& gx, double& gy) {
                         gradient<MAXK>(sD, tab, K, f, x, y, g, c, true, gf, gx, gy);
                       });
  store_chain(a, chain, base, owner, s, it_p, it_q, st);
}

// ---------------------------------------------------------------------------
// Windowed kernels (rhmc_windowed.hpp): any square image, 1 <= K <= 256, one
// wave per chain, star 64 s + lane in register slot s (SLOTS = 1, 2, 4).
template <int SLOTS>
struct WinState {
  double f[SLOTS], x[SLOTS], y[SLOTS], pf[SLOTS], px[SLOTS], py[SLOTS];
  bool own[SLOTS];
};

// Lanes without a star in a slot carry a copy of star 0 (finite, never read).
// The chain's stars start at element row * ld of q and p.
template <int SLOTS>
__device__ __forceinline__ void win_load(const LeapArgs& a, int64_t row, int64_t ld, int K,
                                         WinState<SLOTS>& s) {
  const int lane = lane_id();
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    s.own[t] = kWave * t + lane < K;
    const int64_t e = row * ld + 3 * (s.own[t] ? kWave * t + lane : 0);
    s.f[t] = a.q[e];
    s.x[t] = a.q[e + 1];
    s.y[t] = a.q[e + 2];
    s.pf[t] = a.p[e];
    s.px[t] = a.p[e + 1];
    s.py[t] = a.p[e + 2];
  }
}

template <int SLOTS>
__device__ __forceinline__ void win_store(const LeapArgs& a, int64_t chain, int64_t row,
                                          int64_t ld, int K, const WinState<SLOTS>& s, int it_p,
                                          int it_q, unsigned st) {
  const int lane = lane_id();
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    if (!s.own[t]) continue;
    if (!(isfinite(s.f[t]) && isfinite(s.x[t]) && isfinite(s.y[t]) && isfinite(s.pf[t]) &&
          isfinite(s.px[t]) && isfinite(s.py[t])))
      st |= RHMC_STATUS_NONFINITE;
    const int64_t e = row * ld + 3 * (kWave * t + lane);
    a.q[e] = s.f[t];
    a.q[e + 1] = s.x[t];
    a.q[e + 2] = s.y[t];
    a.p[e] = s.pf[t];
    a.p[e + 1] = s.px[t];
    a.p[e + 2] = s.py[t];
  }
  unsigned all = s.own[0] ? st : 0u;  // status bits are only set for owned slots
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) all |= (unsigned)__shfl_xor((int)all, m, kWave);
  if (lane == 0) {
    if (a.status) a.status[chain] = (int32_t)all;
    if (a.fp_iters) {
      a.fp_iters[2 * chain] = it_p;
      a.fp_iters[2 * chain + 1] = it_q;
    }
  }
}

// n_steps RHMC_single_step()s (sampler_RHMC.py:522-566) on the slotted state,
// the reference-form metric of run_steps; the fixed-point tests take np.max
// over all 3K coordinates (NaN propagates) with one wave max per iteration.
template <int SLOTS, class Grad>
__device__ __forceinline__ void run_steps_win(WinState<SLOTS>& s, int n_steps, int rows,
                                              int cols, const Consts& c, int& it_p, int& it_q,
                                              unsigned& st, Grad grad) {
  const double hdt = c.hdt;
  for (int step = 0;; ++step) {
    double gf[SLOTS], gx[SLOTS], gy[SLOTS];
    grad(s.f, s.x, s.y, gf, gx, gy);
    if (step > 0) {
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        // (5) closing half kick of the previous step (:551), (6) reflection (:554-564)
        s.pf[t] = s.pf[t] - hdt * gf[t];
        s.px[t] = s.px[t] - hdt * gx[t];
        s.py[t] = s.py[t] - hdt * gy[t];
        unsigned b = 0u;
        if (s.f[t] < c.f_lim) {
          s.pf[t] = -s.pf[t];
          b |= RHMC_STATUS_REFLECT_F;
          if (s.f[t] >= c.near_f) b |= RHMC_STATUS_NEAR_WALL;
        }
        if (s.x[t] < 0.0 || s.x[t] > (double)(rows - 1)) {
          s.px[t] = -s.px[t];
          b |= RHMC_STATUS_REFLECT_XY;
          if (near_edge(s.x[t], (double)(rows - 1))) b |= RHMC_STATUS_NEAR_WALL;
        }
        if (s.y[t] < 0.0 || s.y[t] > (double)(cols - 1)) {
          s.py[t] = -s.py[t];
          b |= RHMC_STATUS_REFLECT_XY;
          if (near_edge(s.y[t], (double)(cols - 1))) b |= RHMC_STATUS_NEAR_WALL;
        }
        if (s.own[t]) st |= b;
      }
    }
    if (step == n_steps) break;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {  // (1) opening half kick (:525)
      s.pf[t] = s.pf[t] - hdt * gf[t];
      s.px[t] = s.px[t] - hdt * gx[t];
      s.py[t] = s.py[t] - hdt * gy[t];
    }
    {  // (2) p fixed point, flux slots only (:528-535); x/y slots change by 0
      double coef[SLOTS], rho[SLOTS];
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        coef[t] = dtaudq_coef(s.f[t], c);
        rho[t] = s.pf[t];
      }
      double dp;
      int n = 0;
      do {
        double d = 0.0;
#pragma unroll
        for (int t = 0; t < SLOTS; ++t) {
          const double pp = rho[t] - hdt * ((s.pf[t] * s.pf[t]) * coef[t] / 2.0);
          const double dd = s.own[t] ? fabs(s.pf[t] - pp) : 0.0;
          d = t == 0 ? dd : nanmax2(d, dd);
          s.pf[t] = pp;
        }
        dp = wave_nanmax(d);
        ++n;
      } while (dp > c.delta && n < c.counter_max);
      it_p += n;
      if (dp > c.delta) st |= RHMC_STATUS_PLOOP_CAP;
    }
    {  // (3) q fixed point (:538-545): q' = sig + dt/2 (p/H(sig) + p/H(q))
      double sf[SLOTS], sx[SLOTS], sy[SLOTS], af[SLOTS], ax[SLOTS], ay[SLOTS];
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        sf[t] = s.f[t];
        sx[t] = s.x[t];
        sy[t] = s.y[t];
        const double hff0 = H_ff(sf[t], c), hxx0 = H_xx(sf[t], c);
        af[t] = s.pf[t] / hff0;
        ax[t] = s.px[t] / hxx0;
        ay[t] = s.py[t] / hxx0;
      }
      double dq;
      int n = 0;
      do {
        double d = 0.0;
#pragma unroll
        for (int t = 0; t < SLOTS; ++t) {
          const double hff = H_ff(s.f[t], c), hxx = H_xx(s.f[t], c);
          const double nf = sf[t] + hdt * (af[t] + s.pf[t] / hff);
          const double nx = sx[t] + hdt * (ax[t] + s.px[t] / hxx);
          const double ny = sy[t] + hdt * (ay[t] + s.py[t] / hxx);
          double dd =
              nanmax2(nanmax2(fabs(s.f[t] - nf), fabs(s.x[t] - nx)), fabs(s.y[t] - ny));
          dd = s.own[t] ? dd : 0.0;
          d = t == 0 ? dd : nanmax2(d, dd);
          s.f[t] = nf;
          s.x[t] = nx;
          s.y[t] = ny;
        }
        dq = wave_nanmax(d);
        ++n;
      } while (dq > c.delta && n < c.counter_max);
      it_q += n;
      if (dq > c.delta) st |= RHMC_STATUS_QLOOP_CAP;
    }
#pragma unroll
    for (int t = 0; t < SLOTS; ++t)  // (4) p -= dt/2 dtaudq(q, p) (:548)
      s.pf[t] = s.pf[t] - hdt * ((s.pf[t] * s.pf[t]) * dtaudq_coef(s.f[t], c) / 2.0);
  }
}


// Leapfrog on the slotted state (1 <= K <= 64 SLOTS) with gradient policy G:
// WinG (windowed, any square image, D from global memory) or DenseG<IMG>
// (rhmc_dense.hpp: 32/48-px images, many stars).
template <class G, int SLOTS>
__global__ void __launch_bounds__(256) leapfrog_win_kernel(LeapArgs a) {
  extern __shared__ double lds[];
  const typename G::Ctx gctx = G::setup(lds, a.D, a.K, a.g.rows, a.g.cols, a.g.work);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  int64_t row, ld;
  int K;
  chain_row(a, chain, row, K, ld);
  const LeanConsts lc = lean_consts(c);
  WinState<SLOTS> s;
  win_load<SLOTS>(a, row, ld, K, s);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  const int rows = a.g.rows, cols = a.g.cols;
  run_steps_win<SLOTS>(
      s, a.n_steps, rows, cols, c, it_p, it_q, st,
      [&](const double(&f)[SLOTS], const double(&x)[SLOTS], const double(&y)[SLOTS],
          double(&gf)[SLOTS], double(&gx)[SLOTS], double(&gy)[SLOTS]) {
        G::template gradient<SLOTS>(gctx, K, f, x, y, c, lc, true, gf, gx, gy);
      });
  win_store<SLOTS>(a, chain, row, ld, K, s, it_p, it_q, st);
}

struct GradArgs {
  const double* q;
  double* grad;
  const double* D;
  int64_t n_chains;
  int K, with_metric;
  Geometry g;
  Consts c;
};

template <int MAXK>
__global__ void __launch_bounds__(256) gradient_kernel(GradArgs a) {
  extern __shared__ double lds[];
  const int W = blockDim.x / kWave;
  const int64_t chain = stage_image(lds, a.D, a.g.npix, W);
  if (chain >= a.n_chains) return;
  const int lane = lane_id();
  const int K = a.K;
  const Tables tab = carve_tables(lds + a.g.npix + (threadIdx.x / kWave) * table_doubles(K, a.g.rows, a.g.cols), K, a.g);
  const bool owner = lane < K;
  const int64_t base = chain * 3 * (int64_t)K + 3 * (owner ? lane : 0);
  const double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double gf, gx, gy;
  gradient<MAXK>(lds, tab, K, f, x, y, a.g, a.c, a.with_metric != 0, gf, gx, gy);
  if (owner) {
    a.grad[base] = gf;
    a.grad[base + 1] = gx;
    a.grad[base + 2] = gy;
  }
}

struct EnergyArgs {
  const double* q;
  const double* p;
  double* V;
  double* T;
  const double* D;
  int64_t n_chains;
  int K, f_pos;
  Geometry g;
  Consts c;
  // ragged sets (rhmc_energy_ragged_device, slotted kernels only), as LeapArgs
  const int32_t* Kc = nullptr;
  const int64_t* rows = nullptr;
  int64_t ld = 0;
};

// V (sampler_RHMC.py:294-351) and T at H(q) (:353-363), one wave per chain.
// Ragged sets (a.Kc): the chain's row and star count; the wave's table region
// is sized by the set's largest K (a.K), laid out by the chain's.
template <int MAXK>
__global__ void __launch_bounds__(256) energy_kernel(EnergyArgs a) {
  extern __shared__ double lds[];
  const Geometry& g = a.g;
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t chain = stage_image(lds, a.D, g.npix, W);
  if (chain >= a.n_chains) return;
  const int lane = lane_id();
  int64_t row, ld;
  int K;
  chain_row(a, chain, row, K, ld);
  const Tables tab = carve_tables(
      lds + g.npix + (threadIdx.x / kWave) * table_doubles(a.K, g.rows, g.cols), K, g);
  const bool owner = lane < K;
  const int64_t base = row * ld + 3 * (owner ? lane : 0);
  const double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];

  if (a.T) {
    double t1 = 0.0, t2 = 0.0;
    if (owner) {
      const double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
      const double hff = H_ff(f, c), hxx = H_xx(f, c);
      t1 = pf * pf / hff + px * px / hxx + py * py / hxx;
      t2 = log(fabs(hff)) + log(fabs(hxx)) + log(fabs(hxx));
    }
    t1 = wave_sum(t1);
    t2 = wave_sum(t2);
    if (lane == 0) a.T[chain] = (t1 + t2) / 2.0;
  }
  if (!a.V) return;

  // Infinite potential outside the support (:303-317)
  bool bad = false;
  if (owner) {
    if ((a.f_pos & RHMC_V_FLUX_WALL) && f < c.f_lim) bad = true;
    if (!(a.f_pos & RHMC_V_NO_POSCHECK) &&
        (x < -1.0 || x > (double)(g.rows + 1) || y < -1.0 || y > (double)(g.cols + 1)))
      bad = true;
  }
  if (__any(bad)) {
    if (lane == 0) a.V[chain] = INFINITY;
    return;
  }

  build_tables(tab, K, x, y, g, c);
  double fk[MAXK];
#pragma unroll
  for (int k = 0; k < MAXK; ++k) fk[k] = (k < K) ? bcast(f, k) : 0.0;
  double v = 0.0;
  int i = lane / g.cols, j = lane - (lane / g.cols) * g.cols;
  for (int tt = 0; tt < g.npl; ++tt) {
    const int pix = lane + kWave * tt;
    if (pix < g.npix) {
      double lam = c.B;
#pragma unroll
      for (int k = 0; k < MAXK; ++k)
        if (k < K) lam = fma(fk[k], tab.ex[k * g.rows + i] * tab.ey[k * g.cols + j], lam);
      v += lam - lds[pix] * log(lam);
    }
    j += g.dj;
    i += g.di;
    if (j >= g.cols) {
      j -= g.cols;
      ++i;
    }
  }
  v = wave_sum(v);
  if (c.use_prior) {  // V_prior accumulated per star, added after the sum (:326, :329-330)
    const double vp = wave_sum(owner ? c.alpha * log(f) + c.vprior : 0.0);
    v += vp;
  }
  if (c.use_Vc) {  // 0.5 beta sum_{a,b} R_ab^-pow with R_aa -> 1e32 (:332-349)
    double s = 0.0;
    for (int jj = 0; jj < K; ++jj) {
      const double X = bcast(x, jj), Y = bcast(y, jj);
      double R = sqrt((X - x) * (X - x) + (Y - y) * (Y - y));
      if (fabs(R) < 1e-10) R = 1e32;
      s += pow(1.0 / R, c.vc_pow);
    }
    v += 0.5 * c.beta * wave_sum(owner ? s : 0.0);
  }
  if (lane == 0) a.V[chain] = v;
}

// ---------------------------------------------------------------------------
// Alternative integrators, windowed gradient, lanes = stars:
//   HMC:        single_gym.run_single_HMC leapfrog, unit metric (:628-645)
//   RHMC_NAIVE: run_single_RHMC solver="naive"     (:690-708)
//   RHMC_LF:    run_single_RHMC solver="leap_frog" (:709-728)
// The gradient at the end of a step is the next step's first one (same q).
// dVdq_RHMC (:427-446): flux slot ((p_f^2 (-H_ff'/H_ff^2)) + H_ff'/H_ff + 2 H_xx'/H_xx)/2.
__device__ __forceinline__ double dVdq_rhmc_f(double f, double pf, const Consts& c) {
  const double hff = H_ff(f, c), hffg = H_ff_grad(f, c);
  const double hxx = H_xx(f, c), hxxg = H_xx_grad(f, c);
  const double t1 = (pf * pf) * (-hffg / (hff * hff));
  const double t2 = (hffg / hff) + (2.0 * hxxg / hxx);
  return (t1 + t2) / 2.0;
}

template <class G, int SOLVER, int SLOTS>
__global__ void __launch_bounds__(256) integrate_win_kernel(LeapArgs a, int f_pos) {
  extern __shared__ double lds[];
  const typename G::Ctx gctx = G::setup(lds, a.D, a.K, a.g.rows, a.g.cols, a.g.work);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  const int K = a.K;
  const LeanConsts lc = lean_consts(c);
  WinState<SLOTS> s;
  win_load<SLOTS>(a, chain, 3 * (int64_t)K, K, s);
  const double dt = c.dt;
  unsigned st = 0u;
  double gf[SLOTS], gx[SLOTS], gy[SLOTS];
  // One gradient call site (the gradient is most of the kernel: a second
  // copy is not inlined and its array arguments go to scratch).  Pass `step`
  // closes step - 1 and opens step; the gradient at the end of a step is the
  // next step's first one (same q).
  for (int step = 0;; ++step) {
    if (SOLVER == RHMC_SOLVER_RHMC_NAIVE && step == a.n_steps) break;
    G::template gradient<SLOTS>(gctx, K, s.f, s.x, s.y, c, lc, false, gf, gx, gy);
    if (SOLVER == RHMC_SOLVER_RHMC_NAIVE) {  // :690-708, the gradient at the step's start
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        const double hff = H_ff(s.f[t], c), hxx = H_xx(s.f[t], c);
        const double nf = s.f[t] + dt * s.pf[t] / hff, nx = s.x[t] + dt * s.px[t] / hxx,
                     ny = s.y[t] + dt * s.py[t] / hxx;
        const double pf_old = s.pf[t];
        s.pf[t] = s.pf[t] - dt * (gf[t] + dVdq_rhmc_f(s.f[t], s.pf[t], c));
        s.px[t] = s.px[t] - dt * (gx[t] + 0.0);
        s.py[t] = s.py[t] - dt * (gy[t] + 0.0);
        if (f_pos && nf < c.f_lim) {
          s.pf[t] = pf_old * -1.0;
          if (s.own[t]) st |= RHMC_STATUS_REFLECT_F;
        }
        s.f[t] = nf;
        s.x[t] = nx;
        s.y[t] = ny;
      }
      continue;
    }
    if (step > 0) {  // second half kick of step - 1 (p holds the half-step momentum)
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        if (SOLVER == RHMC_SOLVER_HMC) {  // :628-638
          s.pf[t] = s.pf[t] - dt * gf[t] / 2.0;
        } else {                          // :709-728
          const double hf = s.pf[t];
          s.pf[t] = hf - dt * (gf[t] + dVdq_rhmc_f(s.f[t], hf, c)) / 2.0;
          if (f_pos && s.f[t] < c.f_lim) {
            s.pf[t] = hf * -1.0;
            if (s.own[t]) st |= RHMC_STATUS_REFLECT_F;
          }
        }
        s.px[t] = s.px[t] - dt * (gx[t] + 0.0) / 2.0;
        s.py[t] = s.py[t] - dt * (gy[t] + 0.0) / 2.0;
      }
    }
    if (step == a.n_steps) break;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {  // first half kick and drift of step
      if (SOLVER == RHMC_SOLVER_HMC) {
        const double hf = s.pf[t] - dt * gf[t] / 2.0, hx = s.px[t] - dt * gx[t] / 2.0,
                     hy = s.py[t] - dt * gy[t] / 2.0;
        s.f[t] = s.f[t] + dt * hf;
        s.x[t] = s.x[t] + dt * hx;
        s.y[t] = s.y[t] + dt * hy;
        s.pf[t] = hf;
        s.px[t] = hx;
        s.py[t] = hy;
      } else {
        const double hff = H_ff(s.f[t], c), hxx = H_xx(s.f[t], c);
        const double hf = s.pf[t] - dt * (gf[t] + dVdq_rhmc_f(s.f[t], s.pf[t], c)) / 2.0;
        const double hx = s.px[t] - dt * (gx[t] + 0.0) / 2.0,
                     hy = s.py[t] - dt * (gy[t] + 0.0) / 2.0;
        s.f[t] = s.f[t] + dt * hf / hff;
        s.x[t] = s.x[t] + dt * hx / hxx;
        s.y[t] = s.y[t] + dt * hy / hxx;
        s.pf[t] = hf;
        s.px[t] = hx;
        s.py[t] = hy;
      }
    }
  }
  win_store<SLOTS>(a, chain, chain, 3 * (int64_t)K, K, s, 0, 0, st);
}

// samplers.lightsource_gym.HMC_random's trajectory (samplers.py:519-552):
// unit-mass leapfrog with a per-coordinate step vector dt[3K] and a per-chain
// trajectory length steps[chain] >= 1, flux wall at c.f_lim with the
// reference's quirks kept: the flip mask `iflip` is never cleared within a
// trajectory (a star once below the wall has its flux momentum flipped on
// every later step in which ANY star is below it, :529-541), and when the
// last step flipped, p_tmp keeps the momentum the trajectory started from
// (:547-550 update p_half, not p_tmp) — status bit RHMC_STATUS_REFLECT_F
// marks those chains.  One wave per chain, star 64 s + lane in slot s.
template <class G, int SLOTS>
__global__ void __launch_bounds__(256) hmc_random_win_kernel(LeapArgs a,
                                                             const double* __restrict__ dtv,
                                                             const int32_t* __restrict__ steps) {
  extern __shared__ double lds[];
  const typename G::Ctx gctx = G::setup(lds, a.D, a.K, a.g.rows, a.g.cols, a.g.work);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  const int K = a.K;
  const LeanConsts lc = lean_consts(c);
  const int lane = lane_id();
  WinState<SLOTS> s;
  win_load<SLOTS>(a, chain, 3 * (int64_t)K, K, s);
  double dtf[SLOTS], dtx[SLOTS], dty[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    const int ks = s.own[t] ? kWave * t + lane : 0;
    dtf[t] = dtv[3 * ks];
    dtx[t] = dtv[3 * ks + 1];
    dty[t] = dtv[3 * ks + 2];
  }
  double gf[SLOTS], gx[SLOTS], gy[SLOTS];
  G::template gradient<SLOTS>(gctx, K, s.f, s.x, s.y, c, lc, false, gf, gx, gy);
  double hf[SLOTS], hx[SLOTS], hy[SLOTS];
  bool iflip[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {  // :519
    hf[t] = s.pf[t] - dtf[t] * gf[t] / 2.0;
    hx[t] = s.px[t] - dtx[t] * gx[t] / 2.0;
    hy[t] = s.py[t] - dty[t] * gy[t] / 2.0;
    iflip[t] = false;
  }
  bool flip = false;
  const int n = steps[chain];
  for (int i = 0; i < n; ++i) {
    bool below_any = false;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      s.f[t] = s.f[t] + dtf[t] * hf[t];                                 // :523
      s.x[t] = s.x[t] + dtx[t] * hx[t];
      s.y[t] = s.y[t] + dty[t] * hy[t];
      const bool below = s.own[t] && s.f[t] < c.f_lim;                  // :526-529
      iflip[t] = iflip[t] || below;
      below_any = below_any || below;
    }
    flip = __builtin_amdgcn_ballot_w64(below_any) != 0;
    G::template gradient<SLOTS>(gctx, K, s.f, s.x, s.y, c, lc, false, gf, gx, gy);
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      const double kept = -hf[t];                                       // :531
      hf[t] = hf[t] - dtf[t] * gf[t];                                   // :532, :535
      hx[t] = hx[t] - dtx[t] * gx[t];
      hy[t] = hy[t] - dty[t] * gy[t];
      if (flip && iflip[t]) hf[t] = kept;                               // :533
    }
  }
  unsigned st = 0u;
  if (flip) {
    st |= RHMC_STATUS_REFLECT_F;  // p_tmp stays the starting momentum (:547-550)
  } else {                        // :551-552, dVdq at the same q as the last step
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      s.pf[t] = hf[t] + dtf[t] * gf[t] / 2.0;
      s.px[t] = hx[t] + dtx[t] * gx[t] / 2.0;
      s.py[t] = hy[t] + dty[t] * gy[t] / 2.0;
    }
  }
  win_store<SLOTS>(a, chain, chain, 3 * (int64_t)K, K, s, 0, 0, st);
}

// Star 64 t + lane's (f, x, y) of a chain (lanes without a star: star 0's).
template <int SLOTS>
__device__ __forceinline__ void win_load_q(const double* q, int64_t row, int64_t ld, int K,
                                           double (&f)[SLOTS], double (&x)[SLOTS],
                                           double (&y)[SLOTS], bool (&own)[SLOTS]) {
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    own[t] = win_own(t, K);
    const int64_t e = row * ld + 3 * (own[t] ? kWave * t + lane_id() : 0);
    f[t] = q[e];
    x[t] = q[e + 1];
    y[t] = q[e + 2];
  }
}

// Large-image gradient (windowed), one wave per chain.
template <class G, int SLOTS>
__global__ void __launch_bounds__(256) gradient_win_kernel(GradArgs a) {
  extern __shared__ double lds[];
  const typename G::Ctx gctx = G::setup(lds, a.D, a.K, a.g.rows, a.g.cols, a.g.work);
  const int W = blockDim.x / kWave;
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  const int K = a.K;
  const LeanConsts lc = lean_consts(a.c);
  double f[SLOTS], x[SLOTS], y[SLOTS], gf[SLOTS], gx[SLOTS], gy[SLOTS];
  bool own[SLOTS];
  win_load_q<SLOTS>(a.q, chain, 3 * (int64_t)K, K, f, x, y, own);
  G::template gradient<SLOTS>(gctx, K, f, x, y, a.c, lc, a.with_metric != 0, gf, gx, gy);
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    if (!own[t]) continue;
    const int64_t e = chain * 3 * (int64_t)K + 3 * (kWave * t + lane_id());
    a.grad[e] = gf[t];
    a.grad[e + 1] = gx[t];
    a.grad[e + 2] = gy[t];
  }
}

// Large-image V and T (windowed tables, pixel-major V).
template <class G, int SLOTS>
__global__ void __launch_bounds__(256) energy_win_kernel(EnergyArgs a) {
  extern __shared__ double lds[];
  const typename G::Ctx gctx = G::setup(lds, a.D, a.K, a.g.rows, a.g.cols, a.g.work);
  const Geometry& g = a.g;
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  const int lane = lane_id();
  int64_t row, ld;
  int K;
  chain_row(a, chain, row, K, ld);
  const LeanConsts lc = lean_consts(c);
  double f[SLOTS], x[SLOTS], y[SLOTS];
  bool own[SLOTS];
  win_load_q<SLOTS>(a.q, row, ld, K, f, x, y, own);
  if (a.T) {
    double t1 = 0.0, t2 = 0.0;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      if (!own[t]) continue;
      const int64_t e = row * ld + 3 * (kWave * t + lane);
      const double pf = a.p[e], px = a.p[e + 1], py = a.p[e + 2];
      const double hff = H_ff(f[t], c), hxx = H_xx(f[t], c);
      t1 += pf * pf / hff + px * px / hxx + py * py / hxx;
      t2 += log(fabs(hff)) + log(fabs(hxx)) + log(fabs(hxx));
    }
    t1 = wave_sum(t1);
    t2 = wave_sum(t2);
    if (lane == 0) a.T[chain] = (t1 + t2) / 2.0;
  }
  if (!a.V) return;
  bool bad = false;
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    if (!own[t]) continue;
    if ((a.f_pos & RHMC_V_FLUX_WALL) && f[t] < c.f_lim) bad = true;
    if (!(a.f_pos & RHMC_V_NO_POSCHECK) &&
        (x[t] < -1.0 || x[t] > (double)(g.rows + 1) || y[t] < -1.0 ||
         y[t] > (double)(g.cols + 1)))
      bad = true;
  }
  if (__any(bad)) {
    if (lane == 0) a.V[chain] = INFINITY;
    return;
  }
  double v = G::template potential<SLOTS>(gctx, K, f, x, y, c, lc);
  if (c.use_prior) {
    double vp = 0.0;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t)
      if (own[t]) vp += c.alpha * log(f[t]) + c.vprior;
    v += wave_sum(vp);
  }
  if (c.use_Vc) {  // 0.5 beta sum_{a,b} R_ab^-pow with R_aa -> 1e32 (:332-349)
    double sl = 0.0;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      double sv = 0.0;
#pragma unroll
      for (int t2 = 0; t2 < SLOTS; ++t2) {
        for (int jl = 0; jl < kWave && kWave * t2 + jl < K; ++jl) {
          const double X = bcast(x[t2], jl), Y = bcast(y[t2], jl);
          double R = sqrt((X - x[t]) * (X - x[t]) + (Y - y[t]) * (Y - y[t]));
          if (fabs(R) < 1e-10) R = 1e32;
          sv += pow(1.0 / R, c.vc_pow);
        }
      }
      if (own[t]) sl += sv;
    }
    v += 0.5 * c.beta * wave_sum(sl);
  }
  if (lane == 0) a.V[chain] = v;
}

#ifndef RHMC_KERNELS_ONLY
// The dense kernel's one-slot leapfrog (K <= 64 on 32/48-px images: B4, the
// reference's big-sim4 run) is compiled in rhmc_dense_ilp.hip with the max-ILP
// scheduler; this translation unit only launches it.
extern template __global__ void leapfrog_win_kernel<DenseG<32>, 1>(LeapArgs);
extern template __global__ void leapfrog_win_kernel<DenseG<48>, 1>(LeapArgs);
#endif

}  // namespace rhmc

#ifndef RHMC_KERNELS_ONLY
// ============================================================================
// Host side: C-ABI
// ============================================================================
using namespace rhmc;

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                               \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      return fail(RHMC_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct rhmc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int rows = 0, cols = 0;
  double* d_D = nullptr;
  float* d_Df = nullptr;   // D in fp32, valid when img_f32
  int* d_flag = nullptr;
  bool img_f32 = false;    // every pixel of D is exactly representable in fp32
  // scratch for the host-pointer entry points
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* mh_scratch = nullptr;      // MH driver work arrays (q', p, V, V', E0)
  size_t mh_scratch_bytes = 0;
  int max_lds = 0;
  int n_cu = 0;
  int kernel = RHMC_KERNEL_AUTO;   // RHMC_OPT_KERNEL
  int mh_fused = 1;                // RHMC_OPT_MH_FUSED
  int window_split = 0;            // RHMC_OPT_WINDOW_SPLIT (0: by batch size)
  int table_mode = RHMC_TABLES_STREAM;  // RHMC_OPT_TABLES (diagnostic modes, rhmc.h)
  // WinGG factor tables, one buffer per stream (work_tables).  A launch holds a
  // lease (shared_ptr) on its buffer from the lookup until the launch is
  // enqueued, so a concurrent grow on the same stream cannot free it early.
  struct TabBuf {
    void* p = nullptr;
    size_t bytes = 0;
    hipStream_t s = nullptr;
    bool pooled = false;   // RHMC_TABLES_POOL*: stream-ordered, freed behind the launch
    bool synced = false;   // rhmc_ctx_destroy synchronised the device already
    bool sync_free = false;  // pooled: wait for the stream before hipFreeAsync
    ~TabBuf() {
      if (!p) return;
      if (pooled) {
        if (sync_free) (void)hipStreamSynchronize(s);  // RHMC_TABLES_POOL_SYNCFREE
        (void)hipFreeAsync(p, s);
        return;
      }
      if (!synced) (void)hipStreamSynchronize(s);  // the last launch reading it
      (void)hipFree(p);
    }
  };
  struct StreamTables {
    hipStream_t s;
    std::shared_ptr<TabBuf> buf;
  };
  mutable std::mutex tab_mu;
  mutable std::vector<StreamTables> tabs;
  mutable std::vector<std::shared_ptr<TabBuf>> kept;  // RHMC_TABLES_POOL_KEEP
};

namespace {

// Kernel selection is a context option (RHMC_OPT_KERNEL, rhmc.h); the parity
// tests run the same inputs through every family.  GENERIC / WINDOWED force
// the one-wave-per-chain kernels for every call.
bool per_wave_forced(const rhmc_ctx* ctx) {
  return ctx->kernel == RHMC_KERNEL_GENERIC || ctx->kernel == RHMC_KERNEL_WINDOWED;
}
bool force_windowed(const rhmc_ctx* ctx) { return ctx->kernel == RHMC_KERNEL_WINDOWED; }

// The 32-pixel windows (rhmc_windowed.hpp) drop pixel
// centres >= 15.5 px from a star; exact to fp64 only while their PSF factor
// exp(-15.5^2 / (2 sigma^2)) <= 2^-70, i.e. sigma <= 1.574 px (reference: 1.487).
bool window_exact(const Consts& c) { return 15.5 * 15.5 * c.inv_two_sig2 >= 48.5; }

int window_unsupported() {
  return fail(RHMC_ERR_UNSUPPORTED,
              "PSF wider than the 32-pixel window allows (sigma > 1.574 px) for a configuration "
              "that needs the windowed kernels (K > 16 or image larger than LDS)");
}


constexpr int kMaxKGeneric = 16;   // register accumulators of the LDS-image kernels
constexpr int kMaxKLds = 256;      // slotted kernels, LDS tables: 64 lanes x 4 star slots
constexpr int kMaxK = 1024;        // slotted kernels, global tables (WinGG): 8 / 16 slots
// The windowed path's first star count on the global-table policy (WinGG)
// instead of LDS tables (WinG, whose 2 K 33 doubles per wave cap a CU at one
// or two waves past 64 stars)
#ifndef RHMC_WINGG_FROM
#define RHMC_WINGG_FROM 65
#endif
constexpr int kWinGlobalFromK = RHMC_WINGG_FROM;
static_assert(kWinGlobalFromK == 65 || kWinGlobalFromK == 129 || kWinGlobalFromK == 257,
              "a register-slot boundary");

// Star slots per lane of the windowed kernels for K stars.
int win_slots(int K) {
  return K <= 64 ? 1 : K <= 128 ? 2 : K <= 256 ? 4 : K <= 512 ? 8 : 16;
}

// WinGG's per-chain factor tables (from kWinGlobalFromK stars): one buffer per
// (context, stream), grown on demand and kept until rhmc_ctx_destroy.  Launches
// on one stream run in order, so they can share it.  The caller keeps `lease`
// alive until its launch is enqueued: a grow by another thread on the same
// stream then replaces the context's buffer, and the old one is released only
// when its last lease goes (after a sync of its stream).  Every region a launch
// uses is written by that launch before it is read (win_build_tables,
// win_build_ey), which RHMC_TABLES_POISON checks.
using TableLease = std::shared_ptr<rhmc_ctx::TabBuf>;

int work_tables(const rhmc_ctx* ctx, int path, int K, int64_t n, hipStream_t st,
                double** out, TableLease* lease) {
  *out = nullptr;
  lease->reset();
  if (path != 0 || K < kWinGlobalFromK || n <= 0) return RHMC_OK;
  const size_t bytes = (size_t)n * WinGG::work_doubles(K) * sizeof(double);
  const int mode = ctx->table_mode;
  const bool poison = mode == RHMC_TABLES_STREAM_POISON || mode == RHMC_TABLES_POOL_POISON;
  if (mode == RHMC_TABLES_POOL || mode == RHMC_TABLES_POOL_POISON ||
      mode == RHMC_TABLES_POOL_KEEP || mode == RHMC_TABLES_POOL_SYNCFREE ||
      mode == RHMC_TABLES_POOL_BARRIER) {
    // Diagnostic: round 5's first scheme, one stream-ordered pool allocation
    // per launch, released behind it (~TabBuf: hipFreeAsync on st).
    auto b = std::make_shared<rhmc_ctx::TabBuf>();
    b->s = st;
    b->pooled = true;
    b->sync_free = mode == RHMC_TABLES_POOL_SYNCFREE;
    if (hipMallocAsync(&b->p, bytes, st) != hipSuccess) {
      b->p = nullptr;
      return fail(RHMC_ERR_NOMEM, "hipMallocAsync of " + std::to_string(bytes) +
                                      " B of windowed factor tables failed");
    }
    b->bytes = bytes;
    if (poison) HIP_TRY(hipMemsetAsync(b->p, 0xFF, bytes, st));
    if (mode == RHMC_TABLES_POOL_BARRIER) {  // the launch waits for everything before it
      hipEvent_t e;
      HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(e, st));
      HIP_TRY(hipStreamWaitEvent(st, e, 0));
      HIP_TRY(hipEventDestroy(e));
    }
    *out = (double*)b->p;
    if (mode == RHMC_TABLES_POOL_KEEP) {  // never reused: released at rhmc_ctx_destroy
      std::lock_guard<std::mutex> lk(ctx->tab_mu);
      ctx->kept.push_back(b);
    }
    *lease = std::move(b);
    return RHMC_OK;
  }
  std::lock_guard<std::mutex> lk(ctx->tab_mu);
  rhmc_ctx::StreamTables* t = nullptr;
  for (auto& e : ctx->tabs)
    if (e.s == st) t = &e;
  if (!t || !t->buf || t->buf->bytes < bytes) {
    auto b = std::make_shared<rhmc_ctx::TabBuf>();
    b->s = st;
    if (hipMalloc(&b->p, bytes) != hipSuccess) {
      b->p = nullptr;
      return fail(RHMC_ERR_NOMEM, "hipMalloc of " + std::to_string(bytes) +
                                      " B of windowed factor tables failed");
    }
    b->bytes = bytes;
    if (t)
      t->buf = std::move(b);  // the old buffer goes with its last lease
    else
      ctx->tabs.push_back({st, std::move(b)});
    t = nullptr;
    for (auto& e : ctx->tabs)
      if (e.s == st) t = &e;
  }
  // 0xFF bytes are NaN doubles: a read of an entry this launch did not write
  // turns its chain's result NaN (status NONFINITE) instead of reusing a
  // previous launch's value.
  if (poison) HIP_TRY(hipMemsetAsync(t->buf->p, 0xFF, bytes, st));
  *out = (double*)t->buf->p;
  *lease = t->buf;
  return RHMC_OK;
}

template <class G, int SLOTS>
void launch_integrate_win(int32_t solver, dim3 grid, dim3 block, size_t lds, hipStream_t s,
                          const LeapArgs& a, int fp) {
  if (solver == RHMC_SOLVER_HMC)
    hipLaunchKernelGGL((integrate_win_kernel<G, RHMC_SOLVER_HMC, SLOTS>), grid, block, lds, s, a,
                       fp);
  else if (solver == RHMC_SOLVER_RHMC_NAIVE)
    hipLaunchKernelGGL((integrate_win_kernel<G, RHMC_SOLVER_RHMC_NAIVE, SLOTS>), grid, block, lds,
                       s, a, fp);
  else
    hipLaunchKernelGGL((integrate_win_kernel<G, RHMC_SOLVER_RHMC_LEAPFROG, SLOTS>), grid, block,
                       lds, s, a, fp);
}

// The slotted one-wave-per-chain kernels run one of two gradient policies:
// WinG (windowed tables, any square image; needs window_exact) or DenseG<IMG>
// (rhmc_dense.hpp, 32/48-px images: full-image pixel-major Lambda, star-major
// sums).  A "path" names it: 0 = windowed, 32 / 48 = dense at that side.
template <class T> struct TypeTag { using type = T; };
template <int N> struct IntTag { static constexpr int value = N; };

template <class G, class F>
int with_slots(int K, F&& f) {
  switch (win_slots(K)) {
    case 1: return f(TypeTag<G>{}, IntTag<1>{});
    case 2: return f(TypeTag<G>{}, IntTag<2>{});
    default: return f(TypeTag<G>{}, IntTag<4>{});
  }
}
// K >= kWinGlobalFromK on the windowed path: the global-table policy (the
// only policy instantiated past 256 stars, 8 or 16 slots)
template <class F>
int with_big(int K, F&& f) {
  if constexpr (kWinGlobalFromK <= 64 * 2)
    if (K <= 128) return f(TypeTag<WinGG>{}, IntTag<2>{});
  if constexpr (kWinGlobalFromK <= 64 * 4)
    if (K <= 256) return f(TypeTag<WinGG>{}, IntTag<4>{});
  if (K <= 512) return f(TypeTag<WinGG>{}, IntTag<8>{});
  return f(TypeTag<WinGG>{}, IntTag<16>{});
}
// LDS-table policies below kWinGlobalFromK (windowed) / 256 (dense)
template <class G, class F>
int with_slots_lds(int K, F&& f) {
  if (K <= 64) return f(TypeTag<G>{}, IntTag<1>{});
  if constexpr (kWinGlobalFromK > 65 || !std::is_same<G, WinG>::value)
    if (K <= 128) return f(TypeTag<G>{}, IntTag<2>{});
  if constexpr (kWinGlobalFromK > 129 || !std::is_same<G, WinG>::value)
    return f(TypeTag<G>{}, IntTag<4>{});
  return fail(RHMC_ERR_ARG, "no LDS-table slotted kernel for K = " + std::to_string(K));
}
template <class F>
int with_path(int path, int K, F&& f) {
  if (path == 32) return with_slots<DenseG<32>>(K, f);  // dense_path: K <= 256
  if (path == 48) return with_slots<DenseG<48>>(K, f);
  if (K >= kWinGlobalFromK) return with_big(K, f);
  return with_slots_lds<WinG>(K, f);
}
// The windowed energy kernel's policy: column tables only (WinEG) below
// kWinGlobalFromK, the global tables from there
template <class F>
int with_energy_win(int K, F&& f) {
  if (K >= kWinGlobalFromK) return with_big(K, f);
  if (K <= 64) return f(TypeTag<WinEG>{}, IntTag<1>{});
  if constexpr (kWinGlobalFromK > 65)
    if (K <= 128) return f(TypeTag<WinEG>{}, IntTag<2>{});
  if constexpr (kWinGlobalFromK > 129) return f(TypeTag<WinEG>{}, IntTag<4>{});
  return fail(RHMC_ERR_ARG, "no LDS-table energy kernel for K = " + std::to_string(K));
}

// Which kernel family serves (K, image): the LDS-image kernels need D and the
// per-wave tables in LDS and K <= 16; everything else goes windowed.
bool use_windowed(const rhmc_ctx* ctx, int K) {
  if (K > kMaxKGeneric) return true;
  const size_t need = ((size_t)ctx->rows * ctx->cols + table_doubles(K, ctx->rows, ctx->cols)) *
                      sizeof(double);
  return need > (size_t)ctx->max_lds || force_windowed(ctx);
}

// Windowed kernels: W waves per workgroup, LDS = W * tables (K <= 256: 136 KB
// for one wave, within gfx950's 160 KB; a device with less LDS gets
// RHMC_ERR_UNSUPPORTED here, not a failed launch).
int pick_waves_win(const rhmc_ctx* ctx, int K, size_t* lds, int* W) {
  if (K >= kWinGlobalFromK) {  // WinGG: the exp table only
    *W = 4;
    *lds = WinGG::lds_bytes(4, K);
    return RHMC_OK;
  }
  int w = 4;
  while (w > 1 && WinG::lds_bytes(w, K) > (size_t)ctx->max_lds) w >>= 1;
  *W = w;
  *lds = WinG::lds_bytes(w, K);
  if (*lds > (size_t)ctx->max_lds)
    return fail(RHMC_ERR_UNSUPPORTED, "windowed PSF tables for K = " + std::to_string(K) +
                                          " exceed the device's LDS (" + std::to_string(*lds) +
                                          " B > " + std::to_string(ctx->max_lds) + " B)");
  return RHMC_OK;
}

// The slotted kernels' workgroup for a path (with_path): the windowed tables'
// LDS as above, or four waves of the dense kernel (32 px: 41.5 KB, 48 px:
// 92.6 KB).
int pick_waves_path(const rhmc_ctx* ctx, int path, int K, size_t* lds, int* W) {
  if (path == 32 || path == 48) {
    *W = 4;
    *lds = path == 32 ? DenseG<32>::lds_bytes(4) : DenseG<48>::lds_bytes(4);
    if (*lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "dense kernel LDS");
    return RHMC_OK;
  }
  return pick_waves_win(ctx, K, lds, W);
}

// The dense many-star kernel (rhmc_dense.hpp) for (K, image): by default from
// kDenseMinK stars on 32/48-px square images (where every star's window
// covers most of the image); RHMC_KERNEL_DENSE forces it on those images at
// any K, GENERIC / WINDOWED keep the per-wave families, MULTIWIN(_NOTAB)
// keeps the multi-star register-window kernel where it applies (K <= 64).
// Measured (4096 chains, 100 steps, chain-steps/s, profiles/r04_dense/):
// against the multi-star register-window kernel 32 px K = 12 1.15e8 vs 7.4e7,
// K = 24 8.1e7 vs 1.6e7; 48 px K = 12 5.6e7 vs 4.5e7, K = 24 3.6e7 vs 1.6e7,
// K = 40 2.3e7 vs 6.4e6; big-sim4 (32 px, K = 51) 5.1e7 vs 3.8e6, big-sim3
// (K = 100) 2.7e7 vs 1.7e5 for the windowed kernel.  At K <= 10 the
// pixel-major kernel stays (48 px K = 10: 2.2e8 vs 4.2e7).
constexpr int kDenseMinK = 11;
bool tiledrk_ok(const rhmc_ctx* ctx, int K, const Consts& c);
int dense_path(const rhmc_ctx* ctx, int K, const Consts& c) {
  if (K > kMaxKLds) return 0;  // four register slots at most
  if (ctx->rows != ctx->cols || (ctx->rows != 32 && ctx->rows != 48)) return 0;
  if (per_wave_forced(ctx)) return 0;
  if (ctx->kernel != RHMC_KERNEL_DENSE) {
    if (K < kDenseMinK) return 0;
    if ((ctx->kernel == RHMC_KERNEL_MULTIWIN || ctx->kernel == RHMC_KERNEL_MULTIWIN_NOTAB) &&
        tiledrk_ok(ctx, K, c))
      return 0;
  }
  return ctx->rows;
}

Geometry make_geometry(int rows, int cols) {
  Geometry g;
  g.rows = rows;
  g.cols = cols;
  g.npix = rows * cols;
  g.npl = (g.npix + kWave - 1) / kWave;
  g.di = kWave / cols;
  g.dj = kWave % cols;
  g.work = nullptr;
  return g;
}

int make_consts(const rhmc_params* P, Consts* c) {
  if (!P) return fail(RHMC_ERR_ARG, "params is NULL");
  if (P->reserved != 0) return fail(RHMC_ERR_ARG, "params.reserved must be 0");
  std::memset(c, 0, sizeof(*c));
  c->dt = P->dt;
  c->hdt = P->dt / 2.0;
  c->delta = P->delta;
  c->B = P->B_count;
  c->f_lim = P->f_lim;
  c->f_low = P->f_low;
  const double sigma = P->fwhm_pix / 2.354;  // utils.py:480
  c->two_sig2 = 2 * (sigma * sigma);         // 2*sigma**2 (:484)
  c->psf_norm = (M_PI * 2) * (sigma * sigma);
  const double sv = P->fwhm_pix / 2.354;
  c->var = sv * sv;  // (PSF_FWHM_pix/2.354)**2 (sampler_RHMC.py:384)
  c->g_xx = P->g_xx;
  c->g_ff = P->g_ff;
  c->g_ff2 = P->g_ff2;
  c->g0 = P->g0;
  c->g1 = P->g1;
  c->g2 = P->g2;
  c->c0 = (P->B_count / P->g0) / P->g_ff;
  c->alpha = P->alpha;
  c->beta = P->beta;
  c->vc_pow = P->Vc_r_pow;
  c->vprior = P->V_prior_const;
  c->inv_gff2 = 1.0 / c->g_ff2;
  c->inv_g1 = 1.0 / c->g1;
  c->Bg2 = c->B / c->g2;
  c->two_Bg2 = 2.0 * c->Bg2;
  c->inv_gxx = 1.0 / c->g_xx;
  c->inv_two_sig2 = 1.0 / c->two_sig2;
  c->inv_norm = 1.0 / c->psf_norm;
  c->inv_var = 1.0 / c->var;
  {  // PSF factor recurrences of the register-window kernels (rhmc_tiledr.hpp)
    const double ci = c->inv_two_sig2;
    c->k_row = std::exp(-2.0 * ci);
    c->k_col4 = std::exp(-32.0 * ci);
    // |v0| < rec_vmax keeps every base exp above the fp64 normal range
    // (c v0^2 < 700) and every ratio below e^700 over up to 8 rows (row
    // ratios: c (2 (|v0| + 8) + 1) < 700) or 8 columns 4 apart (column
    // ratios: c (8 (|w0| + 32) + 16) < 700); outside it the direct factors run
    double vm = std::sqrt(700.0 / ci);
    vm = std::fmin(vm, (700.0 / ci - 17.0) / 2.0);
    vm = std::fmin(vm, 700.0 / (8.0 * ci) - 34.0);
    c->rec_vmax = (ci > 0.0 && vm > 0.0) ? vm : 0.0;
  }
  c->near_f = P->f_lim - 0x1p-40 * std::fmax(1.0, std::fabs(P->f_lim));
  c->counter_max = P->counter_max;
  c->use_prior = P->use_prior != 0;
  c->use_Vc = P->use_Vc != 0;
  return RHMC_OK;
}

// Workgroup shape: W waves share one LDS copy of D; pick the largest W<=4
// whose LDS fits.
int pick_waves(const rhmc_ctx* ctx, int K, size_t* lds_bytes, int* W_out) {
  const size_t img = (size_t)ctx->rows * ctx->cols * sizeof(double);
  const size_t tab = table_doubles(K, ctx->rows, ctx->cols) * sizeof(double);
  for (int W = 4; W >= 1; W >>= 1) {
    const size_t need = img + W * tab;
    if (need <= (size_t)ctx->max_lds) {
      *lds_bytes = need;
      *W_out = W;
      return RHMC_OK;
    }
  }
  return fail(RHMC_ERR_UNSUPPORTED,
              "image + PSF tables exceed LDS (" + std::to_string(img + tab) + " B > " +
                  std::to_string(ctx->max_lds) + " B); large images are not built yet");
}

int check_common(rhmc_ctx* ctx, int64_t n_chains, int32_t K) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!ctx->d_D) return fail(RHMC_ERR_ARG, "no image uploaded");
  if (n_chains < 0) return fail(RHMC_ERR_ARG, "n_chains < 0");
  if (K < 1 || K > kMaxK) return fail(RHMC_ERR_ARG, "K must be in [1, 1024]");
  if (n_chains > ((int64_t)1 << 40)) return fail(RHMC_ERR_ARG, "n_chains too large");
  return RHMC_OK;
}

int ensure_scratch(rhmc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->scratch_bytes) return RHMC_OK;
  if (ctx->scratch) HIP_TRY(hipFree(ctx->scratch));
  ctx->scratch = nullptr;
  ctx->scratch_bytes = 0;
  if (hipMalloc(&ctx->scratch, bytes) != hipSuccess)
    return fail(RHMC_ERR_NOMEM, "hipMalloc scratch " + std::to_string(bytes) + " B failed");
  ctx->scratch_bytes = bytes;
  return RHMC_OK;
}

template <template <int> class Launcher, typename Args>
int dispatch_k(int K, dim3 grid, dim3 block, size_t lds, hipStream_t s, const Args& a) {
  if (K == 1) return Launcher<1>::go(grid, block, lds, s, a);
  if (K <= 2) return Launcher<2>::go(grid, block, lds, s, a);
  if (K <= 4) return Launcher<4>::go(grid, block, lds, s, a);
  if (K <= 8) return Launcher<8>::go(grid, block, lds, s, a);
  return Launcher<16>::go(grid, block, lds, s, a);
}

template <int MAXK>
struct LeapLaunch {
  static int go(dim3 grid, dim3 block, size_t lds, hipStream_t s, const LeapArgs& a) {
    hipLaunchKernelGGL(leapfrog_kernel<MAXK>, grid, block, lds, s, a);
    HIP_TRY(hipGetLastError());
    return RHMC_OK;
  }
};
template <int MAXK>
struct GradLaunch {
  static int go(dim3 grid, dim3 block, size_t lds, hipStream_t s, const GradArgs& a) {
    hipLaunchKernelGGL(gradient_kernel<MAXK>, grid, block, lds, s, a);
    HIP_TRY(hipGetLastError());
    return RHMC_OK;
  }
};
template <int MAXK>
struct EnergyLaunch {
  static int go(dim3 grid, dim3 block, size_t lds, hipStream_t s, const EnergyArgs& a) {
    hipLaunchKernelGGL(energy_kernel<MAXK>, grid, block, lds, s, a);
    HIP_TRY(hipGetLastError());
    return RHMC_OK;
  }
};



// Register-window single-star kernel (rhmc_tiledr.hpp).
template <int IMG, int WIN, typename DT, bool PROF>
int launch_tiledr_t(const rhmc_ctx* ctx, const LeapArgsK1& a, hipStream_t s) {
  using TL = TiledR<IMG, WIN, DT>;
  size_t lds = TL::lds_bytes();
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
  constexpr int W = 4;
  const int64_t waves = (a.n_chains + TL::CPW - 1) / TL::CPW;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  hipLaunchKernelGGL((leapfrog_k1_tiledr<IMG, WIN, DT, PROF>), grid, block, lds, s, a);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}
// Register-window kernel (rhmc_tiledr.hpp): the 28-pixel window when the PSF
// allows it (RHMC_KERNEL_REGWIN32 forces 32), the fp32 pixel cache when the
// image allows it exactly (RHMC_KERNEL_REGWIN_F64 forces fp64).  A library
// built with -DRHMC_PHASE_PROF (make prof, tools/phase_prof.py only) runs the
// phase-timing instantiation instead, which writes cycle counts over the state.
template <int IMG>
int launch_tiledr(const rhmc_ctx* ctx, LeapArgsK1 a, hipStream_t s) {
  const bool w28 = reg_window_ok(28, a.c.inv_two_sig2) && ctx->kernel != RHMC_KERNEL_REGWIN32;
  const bool f32 = ctx->img_f32 && ctx->kernel != RHMC_KERNEL_REGWIN_F64;
#ifdef RHMC_PHASE_PROF
  if (w28 && f32) {
    a.Df = ctx->d_Df;
    return launch_tiledr_t<IMG, 28, float, true>(ctx, a, s);
  }
#endif
  if (f32) {
    a.Df = ctx->d_Df;
    return w28 ? launch_tiledr_t<IMG, 28, float, false>(ctx, a, s)
               : launch_tiledr_t<IMG, 32, float, false>(ctx, a, s);
  }
  return w28 ? launch_tiledr_t<IMG, 28, double, false>(ctx, a, s)
             : launch_tiledr_t<IMG, 32, double, false>(ctx, a, s);
}

// Lane-group single-star kernel for large batches (rhmc_tiledl.hpp).
template <int IMG, typename DT, int LPC>
int launch_tiledl_t(const rhmc_ctx* ctx, const LeapArgsK1& a, hipStream_t s) {
  using TL = TiledL<IMG, 28, DT, LPC>;
  const size_t lds = TL::lds_bytes();
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
  constexpr int W = 4;
  const int64_t waves = (a.n_chains + TL::CPW - 1) / TL::CPW;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  hipLaunchKernelGGL((leapfrog_k1_tiledl<IMG, 28, DT, LPC>), grid, block, lds, s, a);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}
template <int IMG, int LPC>
int launch_tiledl_lpc(const rhmc_ctx* ctx, LeapArgsK1 a, bool f32, hipStream_t s) {
  if (f32) {
    a.Df = ctx->d_Df;
    return launch_tiledl_t<IMG, float, LPC>(ctx, a, s);
  }
  return launch_tiledl_t<IMG, double, LPC>(ctx, a, s);
}

// Lanes per chain of the lane-group kernel for a K = 1 batch of n chains, or 0
// for the register-window kernel.  RHMC_KERNEL_LANE1 / _LANE4 / _LANE1_F64
// force it, RHMC_KERNEL_REGWIN* turn it off.
// Measured (C2 geometry, 500 steps, chain-steps/s): 16384 chains tiledr
// 1.99e9 / LPC 4 2.25e9; 65536: 2.28e9 / LPC 1 3.06e9; 131072: 2.31e9 / 3.59e9.
constexpr int64_t kLaneChains1 = 65536;   // >= one 64-chain wave per SIMD
constexpr int64_t kLaneChains4 = 16384;   // >= one 16-chain wave per SIMD
int tiledl_lpc(int64_t n, int kern) {
  if (kern == RHMC_KERNEL_LANE1 || kern == RHMC_KERNEL_LANE1_F64) return 1;
  if (kern == RHMC_KERNEL_LANE4) return 4;
  if (kern == RHMC_KERNEL_REGWIN || kern == RHMC_KERNEL_REGWIN32 || kern == RHMC_KERNEL_REGWIN_F64)
    return 0;
  return n >= kLaneChains1 ? 1 : n >= kLaneChains4 ? 4 : 0;
}

template <int IMG>
int launch_tiledl(const rhmc_ctx* ctx, const LeapArgsK1& a, int lpc, hipStream_t s) {
  const bool f32 = ctx->img_f32 && ctx->kernel != RHMC_KERNEL_LANE1_F64;
  return lpc == 4 ? launch_tiledl_lpc<IMG, 4>(ctx, a, f32, s)
                  : launch_tiledl_lpc<IMG, 1>(ctx, a, f32, s);
}


// V (and optionally T) of n chains on device buffers, async on `s`.
template <int IMG>
int launch_energy_k1(const rhmc_ctx* ctx, EnergyK1Args k, hipStream_t s) {
  constexpr int W = 4;
  const int64_t waves = (k.n + 3) / 4;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  if (ctx->img_f32) {
    k.Df = ctx->d_Df;
    const size_t lds = TiledR<IMG, 28, float>::lds_bytes();
    if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((energy_k1_tiledr<IMG, float>), grid, block, lds, s, k);
  } else {
    const size_t lds = TiledR<IMG, 28, double>::lds_bytes();
    if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((energy_k1_tiledr<IMG, double>), grid, block, lds, s, k);
  }
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

int launch_energy(const rhmc_ctx* ctx, const Consts& c, const double* d_q, const double* d_p,
                  double* d_V, double* d_T, int64_t n, int K, int f_pos, hipStream_t s) {
  // one star on a 32/48/64-px image: the register-window energy kernel
  // (rhmc_mhk1.hpp); RHMC_KERNEL_GENERIC / _WINDOWED keep the per-wave kernels
  const int side = ctx->rows;
  if (K == 1 && !c.use_Vc && ctx->rows == ctx->cols && (side == 32 || side == 48 || side == 64) &&
      reg_window_ok(28, c.inv_two_sig2) && !per_wave_forced(ctx) &&
      ctx->kernel != RHMC_KERNEL_DENSE) {
    if (n == 0) return RHMC_OK;
    EnergyK1Args k;
    k.q = d_q;
    k.p = d_p;
    k.V = d_V;
    k.T = d_T;
    k.D = ctx->d_D;
    k.Df = nullptr;
    k.n = n;
    k.f_pos = f_pos & (RHMC_V_FLUX_WALL | RHMC_V_NO_POSCHECK);
    k.pad = 0;
    k.c = c;
    switch (side) {
      case 32: return launch_energy_k1<32>(ctx, k, s);
      case 48: return launch_energy_k1<48>(ctx, k, s);
      default: return launch_energy_k1<64>(ctx, k, s);
    }
  }
  EnergyArgs a;
  a.c = c;
  size_t lds;
  int W;
  int rc;
  const int path = dense_path(ctx, K, c);
  const bool win = path || use_windowed(ctx, K);
  if (win && !path && !window_exact(c)) return window_unsupported();
  if (win && !path && K >= kWinGlobalFromK) {  // global tables (WinGG)
    if ((rc = pick_waves_win(ctx, K, &lds, &W))) return rc;
  } else if (win && !path) {  // potential-only windowed tables (WinEG)
    W = 4;
    while (W > 1 && WinEG::lds_bytes(W, K) > (size_t)ctx->max_lds) W >>= 1;
    lds = WinEG::lds_bytes(W, K);
    if (lds > (size_t)ctx->max_lds)
      return fail(RHMC_ERR_UNSUPPORTED, "windowed energy tables exceed the device's LDS");
  } else if (win) {
    if ((rc = pick_waves_path(ctx, path, K, &lds, &W))) return rc;
  } else if ((rc = pick_waves(ctx, K, &lds, &W))) {
    return rc;
  }
  a.q = d_q;
  a.p = d_p;
  a.V = d_V;
  a.T = d_T;
  a.D = ctx->d_D;
  a.n_chains = n;
  a.K = K;
  a.f_pos = f_pos & (RHMC_V_FLUX_WALL | RHMC_V_NO_POSCHECK);
  a.g = make_geometry(ctx->rows, ctx->cols);
  TableLease lease;
  if ((rc = work_tables(ctx, path, K, n, s, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
  if (win) {
    auto go = [&](auto gt, auto st) {
      using G = typename decltype(gt)::type;
      hipLaunchKernelGGL((energy_win_kernel<G, decltype(st)::value>), grid, block, lds, s, a);
      HIP_TRY(hipGetLastError());
      return (int)RHMC_OK;
    };
    return path ? with_path(path, K, go) : with_energy_win(K, go);
  }
  return dispatch_k<EnergyLaunch>(K, grid, block, lds, s, a);
}


// Multi-star register-window kernel (rhmc_tiledrk.hpp): K in [2, 64], square
// image of side >= 32, PSF narrow enough for the 28-row window.
bool tiledrk_ok(const rhmc_ctx* ctx, int K, const Consts& c) {
  return K >= 1 && K <= 64 && ctx->rows == ctx->cols && ctx->rows >= 32 &&
         reg_window_ok(28, c.inv_two_sig2);
}

// Which multi-star kernel serves (K, image) by default: the register-window
// kernel wherever it applies (C3 with LDS factor tables: 18.0 ms per 100 steps
// against 20.3 for the full-image tiled kernel; C5: 3.2x the windowed kernel).
// RHMC_KERNEL_GENERIC / _WINDOWED force the one-wave-per-chain families.
bool use_tiledrk(const rhmc_ctx* ctx, int K, const Consts& c) {
  return !per_wave_forced(ctx) && tiledrk_ok(ctx, K, c);
}

template <typename DT, int SLOTS, bool TAB, int SOLVER = RHMC_SOLVER_IMPLICIT, int WS = 1>
int launch_kr_ws(const rhmc_ctx* ctx, const LeapArgsKR& a, int f_pos, hipStream_t s) {
  using TK = TiledRK<DT, SLOTS, TAB>;
  int W = 4;
  while (W > WS && TK::lds_bytes(W, a.K, a.side, WS) > (size_t)ctx->max_lds / 2) W >>= 1;
  const size_t lds = TK::lds_bytes(W, a.K, a.side, WS);
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "factor tables exceed LDS");
  const int64_t waves = (a.n_chains + TK::CPW - 1) / TK::CPW * WS;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  hipLaunchKernelGGL((leapfrog_kr<DT, SLOTS, TAB, SOLVER, WS>), grid, block, lds, s, a, f_pos);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

// Waves per chain pair for the implicit window-major kernel: the option, or
// the least of 1, 2, 4 that gives the launch eight waves per SIMD (four rounds
// of the kernel's two resident waves: finer rounds even out the waves' unequal
// neighbour work).  C5 sweep (profiles/r03_ws/, chain-steps/s, WS 1 / 2 / 4):
// 1024 chains 5.19e6 / 1.01e7 / 1.29e7, 2048 1.03e7 / 1.39e7 / 1.38e7,
// 4096 1.42e7 / 1.48e7 / 1.48e7, 8192 1.50e7 / 1.53e7 / 1.52e7,
// 16384 1.58e7 / 1.58e7 / 1.55e7.
int kr_window_split(const rhmc_ctx* ctx, int64_t n_chains) {
  if (ctx->window_split) return ctx->window_split;
  const int64_t pairs = (n_chains + 1) / 2, target = 32 * (int64_t)(ctx->n_cu > 0 ? ctx->n_cu : 256);
  int ws = 1;
  while (ws < 4 && pairs * ws < target) ws *= 2;
  return ws;
}

template <typename DT, int SLOTS, bool TAB, int SOLVER = RHMC_SOLVER_IMPLICIT>
int launch_kr_t(const rhmc_ctx* ctx, const LeapArgsKR& a, int f_pos, hipStream_t s) {
  if constexpr (SOLVER == RHMC_SOLVER_IMPLICIT && !TAB) {
    switch (kr_window_split(ctx, a.n_chains)) {
      case 2: return launch_kr_ws<DT, SLOTS, TAB, SOLVER, 2>(ctx, a, f_pos, s);
      case 4: return launch_kr_ws<DT, SLOTS, TAB, SOLVER, 4>(ctx, a, f_pos, s);
      default: break;
    }
  }
  return launch_kr_ws<DT, SLOTS, TAB, SOLVER, 1>(ctx, a, f_pos, s);
}

// Factor tables in LDS (TiledRK<..., TAB>) for images up to 64 px with K <= 16,
// where every window overlaps (nearly) every star; RHMC_KERNEL_MULTIWIN_NOTAB
// forces the exp path there.
bool kr_tables(const rhmc_ctx* ctx, int K) {
  return ctx->kernel != RHMC_KERNEL_MULTIWIN_NOTAB && ctx->rows <= 64 && K <= 16;
}

template <int SOLVER = RHMC_SOLVER_IMPLICIT>
int launch_kr(const rhmc_ctx* ctx, LeapArgsKR a, int f_pos, hipStream_t s) {
  const bool f32 = ctx->img_f32;
  if (f32) a.Df = ctx->d_Df;
  if (kr_tables(ctx, a.K))
    return f32 ? launch_kr_t<float, 1, true, SOLVER>(ctx, a, f_pos, s)
               : launch_kr_t<double, 1, true, SOLVER>(ctx, a, f_pos, s);
  if (a.K <= 32)
    return f32 ? launch_kr_t<float, 1, false, SOLVER>(ctx, a, f_pos, s)
               : launch_kr_t<double, 1, false, SOLVER>(ctx, a, f_pos, s);
  return f32 ? launch_kr_t<float, 2, false, SOLVER>(ctx, a, f_pos, s)
             : launch_kr_t<double, 2, false, SOLVER>(ctx, a, f_pos, s);
}

// Pixel-major multi-star kernel (rhmc_pixk.hpp): the default for 2 <= K <= 10
// on a 32/48-px fp32-exact image (C3: 1.23e8 chain-steps/s against 1.05e8 for
// the window-major kernel with LDS tables, measured A/B on one box).
// RHMC_KERNEL_MULTIWIN* force the window-major kernel, GENERIC / WINDOWED the
// per-wave ones.
bool use_pixk(const rhmc_ctx* ctx, int K, const Consts& c) {
  const int k = ctx->kernel;
  const bool want = !per_wave_forced(ctx) && k != RHMC_KERNEL_MULTIWIN &&
                    k != RHMC_KERNEL_MULTIWIN_NOTAB && k != RHMC_KERNEL_DENSE;
  return want && K >= 2 && K <= 10 && !c.use_Vc && ctx->img_f32 && ctx->rows == ctx->cols &&
         (ctx->rows == 32 || ctx->rows == 48);
}

template <int IMG, int SOLVER = RHMC_SOLVER_IMPLICIT, bool RAGGED = false>
int launch_pk(const rhmc_ctx* ctx, LeapArgsKR a, hipStream_t s, int f_pos = 0) {
  using PK = PixK<IMG, 10>;  // LDS layout does not depend on the columns per pass
  int W = 4;
  while (W > 1 && PK::lds_bytes(W) > (size_t)ctx->max_lds / 2) W >>= 1;
  const size_t lds = PK::lds_bytes(W);
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "pixk LDS");
  a.Df = ctx->d_Df;
  const int64_t waves = (a.n_chains + PK::CPW - 1) / PK::CPW;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  hipLaunchKernelGGL((leapfrog_pk<IMG, 10, SOLVER, RAGGED>), grid, block, lds, s, a, f_pos);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

template <int SOLVER>
int launch_pk_side(const rhmc_ctx* ctx, const LeapArgsKR& a, hipStream_t s, int f_pos) {
  return ctx->rows == 32 ? launch_pk<32, SOLVER>(ctx, a, s, f_pos)
                         : launch_pk<48, SOLVER>(ctx, a, s, f_pos);
}

int launch_leapfrog(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                    int64_t n_chains, int32_t K, int32_t n_steps, int32_t* d_it, int32_t* d_st,
                    hipStream_t s) {
  LeapArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  if (n_steps < 0) return fail(RHMC_ERR_ARG, "n_steps < 0");
  if (P->counter_max < 1) return fail(RHMC_ERR_ARG, "counter_max < 1");
  if (n_chains == 0) return RHMC_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const int side = ctx->rows;
  // one star: the register-window kernel (C1, C2) or, from 16 Ki chains, the
  // lane-group kernel (C4 shards); wider PSFs and other image sides take the
  // generic kernel below
  const bool k1 = K == 1 && !a.c.use_Vc && ctx->rows == ctx->cols && !per_wave_forced(ctx) &&
                  ctx->kernel != RHMC_KERNEL_DENSE;
  const bool img_ok = side == 32 || side == 48 || side == 64 || side == 96 || side == 128;
  if (k1 && img_ok && reg_window_ok(32, a.c.inv_two_sig2)) {
    LeapArgsK1 t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = d_it;
    t.status = d_st;
    t.D = ctx->d_D;
    t.n_chains = n_chains;
    t.n_steps = n_steps;
    t.rows = ctx->rows;
    t.cols = ctx->cols;
    t.pad = 0;
    t.Df = nullptr;
    t.c = a.c;
    const int lpc = tiledl_lpc(n_chains, ctx->kernel);
    if (lpc && side <= 64 && reg_window_ok(28, a.c.inv_two_sig2)) {
      switch (side) {
        case 32: return launch_tiledl<32>(ctx, t, lpc, s);
        case 48: return launch_tiledl<48>(ctx, t, lpc, s);
        default: return launch_tiledl<64>(ctx, t, lpc, s);
      }
    }
    switch (side) {
      case 32: return launch_tiledr<32>(ctx, t, s);
      case 48: return launch_tiledr<48>(ctx, t, s);
      case 64: return launch_tiledr<64>(ctx, t, s);
      case 96: return launch_tiledr<96>(ctx, t, s);
      default: return launch_tiledr<128>(ctx, t, s);
    }
  }
  const int path = dense_path(ctx, K, a.c);
  if (!path && (use_pixk(ctx, K, a.c) || use_tiledrk(ctx, K, a.c))) {
    LeapArgsKR t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = d_it;
    t.status = d_st;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n_chains;
    t.K = K;
    t.n_steps = n_steps;
    t.side = ctx->rows;
    t.pad = 0;
    t.c = a.c;
    t.dtv = nullptr;
    t.steps = nullptr;
    if (use_pixk(ctx, K, a.c)) return ctx->rows == 32 ? launch_pk<32>(ctx, t, s) : launch_pk<48>(ctx, t, s);
    return launch_kr(ctx, t, 0, s);
  }
  a.g = make_geometry(ctx->rows, ctx->cols);
  size_t lds;
  int W;
  if (path || use_windowed(ctx, K)) {
    if (!path && !window_exact(a.c)) return window_unsupported();
    a.q = d_q;
    a.p = d_p;
    a.fp_iters = d_it;
    a.status = d_st;
    a.D = ctx->d_D;
    a.n_chains = n_chains;
    a.K = K;
    a.n_steps = n_steps;
    if (int rc = pick_waves_path(ctx, path, K, &lds, &W)) return rc;
    TableLease lease;
    if ((rc = work_tables(ctx, path, K, n_chains, s, &a.g.work, &lease))) return rc;
    const dim3 grid((unsigned)((n_chains + W - 1) / W)), block(W * kWave);
    return with_path(path, K, [&](auto gt, auto st) {
      using G = typename decltype(gt)::type;
      hipLaunchKernelGGL((leapfrog_win_kernel<G, decltype(st)::value>), grid, block, lds, s, a);
      HIP_TRY(hipGetLastError());
      return (int)RHMC_OK;
    });
  }
  a.q = d_q;
  a.p = d_p;
  a.fp_iters = d_it;
  a.status = d_st;
  a.D = ctx->d_D;
  a.n_chains = n_chains;
  a.K = K;
  a.n_steps = n_steps;
  if ((rc = pick_waves(ctx, K, &lds, &W))) return rc;
  const dim3 grid((unsigned)((n_chains + W - 1) / W)), block(W * kWave);
  return dispatch_k<LeapLaunch>(K, grid, block, lds, s, a);
}

int launch_leapfrog(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                    int64_t n_chains, int32_t K, int32_t n_steps, int32_t* d_it, int32_t* d_st,
                    hipStream_t s);

// ---------------------------------------------------------------------------
// Ragged chain sets (rhmc.h: rhmc_leapfrog_ragged_device & co.; the
// reversible-jump driver).  Which star counts the automatic dispatch serves
// with a slotted one-wave-per-chain kernel — for both the step and the
// energy — where chains of different K can share a launch: 1 = the dense
// kernel (32/48-px images, from 11 stars), 2 = the windowed kernel, 3 = the
// pixel-major kernel (2-10 stars on 32/48-px fp32-exact images) with the
// LDS-image energy kernel; 0 = a kernel with a fixed K per launch (one-star,
// multi-star register-window).
int ragged_family(const rhmc_ctx* ctx, const Consts& c, int K) {
  if (K < 1 || K > kMaxK) return 0;
  if (dense_path(ctx, K, c)) return 1;
  if (K == 1) return 0;
  if (use_pixk(ctx, K, c))  // the energy of those K: the LDS-image kernel
    return !use_windowed(ctx, K) ? 3 : 0;
  if (use_tiledrk(ctx, K, c)) return 0;
  return use_windowed(ctx, K) && window_exact(c) ? 2 : 0;
}

// [K_min, K_max]: one family and one register-slot count (the launch's SLOTS
// and LDS follow K_max)
int ragged_check(const rhmc_ctx* ctx, const Consts& c, int K_min, int K_max, int64_t ld,
                 int* family) {
  if (K_min < 1 || K_max > kMaxK || K_min > K_max)
    return fail(RHMC_ERR_ARG, "ragged set: need 1 <= K_min <= K_max <= 1024");
  if (win_slots(K_min) != win_slots(K_max))
    return fail(RHMC_ERR_ARG, "ragged set: K_min and K_max need the same register slots "
                              "(1-64, 65-128, 129-256, 257-512, 513-1024 stars)");
  if (ld < 3 * (int64_t)K_max) return fail(RHMC_ERR_ARG, "ragged set: ld < 3 K_max");
  const int f = ragged_family(ctx, c, K_min);
  for (int K = K_min; K <= K_max; ++K)
    if (ragged_family(ctx, c, K) != f || f == 0)
      return fail(RHMC_ERR_UNSUPPORTED, "ragged set: K = " + std::to_string(K) +
                                            " is not served by a slotted kernel on this image "
                                            "(rhmc_ragged_ok)");
  *family = f;
  return RHMC_OK;
}

int launch_leapfrog_ragged(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                           int64_t ld, const int64_t* d_rows, const int32_t* d_K, int64_t n,
                           int K_min, int K_max, int32_t n_steps, hipStream_t s) {
  LeapArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  if (n_steps < 0) return fail(RHMC_ERR_ARG, "n_steps < 0");
  if (P->counter_max < 1) return fail(RHMC_ERR_ARG, "counter_max < 1");
  int fam;
  if ((rc = ragged_check(ctx, a.c, K_min, K_max, ld, &fam))) return rc;
  if (n == 0) return RHMC_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  if (fam == 3) {  // the pixel-major kernel, each chain its own row and K
    LeapArgsKR t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = nullptr;
    t.status = nullptr;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n;
    t.K = K_max;
    t.n_steps = n_steps;
    t.side = ctx->rows;
    t.pad = 0;
    t.c = a.c;
    t.dtv = nullptr;
    t.steps = nullptr;
    t.Kc = d_K;
    t.rows = d_rows;
    t.ld = ld;
    return ctx->rows == 32 ? launch_pk<32, RHMC_SOLVER_IMPLICIT, true>(ctx, t, s)
                           : launch_pk<48, RHMC_SOLVER_IMPLICIT, true>(ctx, t, s);
  }
  const int path = dense_path(ctx, K_max, a.c);
  a.g = make_geometry(ctx->rows, ctx->cols);
  a.q = d_q;
  a.p = d_p;
  a.fp_iters = nullptr;
  a.status = nullptr;
  a.D = ctx->d_D;
  a.n_chains = n;
  a.K = K_max;
  a.n_steps = n_steps;
  a.Kc = d_K;
  a.rows = d_rows;
  a.ld = ld;
  size_t lds;
  int W;
  if ((rc = pick_waves_path(ctx, path, K_max, &lds, &W))) return rc;
  TableLease lease;
  if ((rc = work_tables(ctx, path, K_max, n, s, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
  return with_path(path, K_max, [&](auto gt, auto st) {
    using G = typename decltype(gt)::type;
    hipLaunchKernelGGL((leapfrog_win_kernel<G, decltype(st)::value>), grid, block, lds, s, a);
    HIP_TRY(hipGetLastError());
    return (int)RHMC_OK;
  });
}

int launch_energy_ragged(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int64_t ld,
                         const int64_t* d_rows, const int32_t* d_K, int64_t n, int K_min,
                         int K_max, int f_pos, double* d_V, hipStream_t s) {
  EnergyArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  int fam;
  if ((rc = ragged_check(ctx, a.c, K_min, K_max, ld, &fam))) return rc;
  if (n == 0) return RHMC_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const int path = dense_path(ctx, K_max, a.c);
  size_t lds;
  int W;
  if (fam == 3) {  // the LDS-image kernel, each chain its own row and K
    if ((rc = pick_waves(ctx, K_max, &lds, &W))) return rc;
    a.q = d_q;
    a.p = nullptr;
    a.V = d_V;
    a.T = nullptr;
    a.D = ctx->d_D;
    a.n_chains = n;
    a.K = K_max;
    a.f_pos = f_pos & (RHMC_V_FLUX_WALL | RHMC_V_NO_POSCHECK);
    a.g = make_geometry(ctx->rows, ctx->cols);
    a.Kc = d_K;
    a.rows = d_rows;
    a.ld = ld;
    const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
    return dispatch_k<EnergyLaunch>(K_max, grid, block, lds, s, a);
  }
  if (path || K_max >= kWinGlobalFromK) {
    if ((rc = pick_waves_path(ctx, path, K_max, &lds, &W))) return rc;
  } else {  // potential-only windowed tables, as launch_energy
    W = 4;
    while (W > 1 && WinEG::lds_bytes(W, K_max) > (size_t)ctx->max_lds) W >>= 1;
    lds = WinEG::lds_bytes(W, K_max);
    if (lds > (size_t)ctx->max_lds)
      return fail(RHMC_ERR_UNSUPPORTED, "windowed energy tables exceed the device's LDS");
  }
  a.q = d_q;
  a.p = nullptr;
  a.V = d_V;
  a.T = nullptr;
  a.D = ctx->d_D;
  a.n_chains = n;
  a.K = K_max;
  a.f_pos = f_pos & (RHMC_V_FLUX_WALL | RHMC_V_NO_POSCHECK);
  a.g = make_geometry(ctx->rows, ctx->cols);
  a.Kc = d_K;
  a.rows = d_rows;
  a.ld = ld;
  TableLease lease;
  if ((rc = work_tables(ctx, path, K_max, n, s, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
  auto go = [&](auto gt, auto st) {
    using G = typename decltype(gt)::type;
    hipLaunchKernelGGL((energy_win_kernel<G, decltype(st)::value>), grid, block, lds, s, a);
    HIP_TRY(hipGetLastError());
    return (int)RHMC_OK;
  };
  return path ? with_path(path, K_max, go) : with_energy_win(K_max, go);
}

// One star where launch_leapfrog takes the register-window kernel (28-px
// window, 32/48/64-px image, fewer chains than the lane-group threshold): the
// whole MH loop in one launch (rhmc_mhk1.hpp).  RHMC_OPT_MH_FUSED = 0, or a
// forced kernel other than REGWIN, keeps the four-kernel loop below.
bool mh_k1_fused(const rhmc_ctx* ctx, const Consts& c, int64_t n) {
  if (!ctx->mh_fused) return false;
  if (ctx->kernel != RHMC_KERNEL_AUTO && ctx->kernel != RHMC_KERNEL_REGWIN) return false;
  const int side = ctx->rows;
  return !c.use_Vc && ctx->rows == ctx->cols && (side == 32 || side == 48 || side == 64) &&
         reg_window_ok(28, c.inv_two_sig2) && tiledl_lpc(n, ctx->kernel) == 0;
}

template <int IMG>
int launch_mh_k1(const rhmc_ctx* ctx, MhK1Args k, hipStream_t s) {
  const size_t lds16 = TiledR<IMG, 28, float>::lds_bytes();
  const size_t lds64 = TiledR<IMG, 28, double>::lds_bytes();
  constexpr int W = 4;
  const int64_t waves = (k.n + 3) / 4;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  if (ctx->img_f32) {
    k.Df = ctx->d_Df;
    if (lds16 > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((mh_k1_tiledr<IMG, 28, float>), grid, block, lds16, s, k);
  } else {
    if (lds64 > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((mh_k1_tiledr<IMG, 28, double>), grid, block, lds64, s, k);
  }
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

// 2 <= K <= 10 stars where launch_leapfrog takes the pixel-major kernel: one
// launch per MH iteration instead of four (rhmc_mhpk.hpp).  RHMC_OPT_MH_FUSED
// = 0, or a forced kernel other than PIXMAJOR, keeps the four-kernel loop.
bool mh_pk_fused(const rhmc_ctx* ctx, const Consts& c, int K) {
  if (!ctx->mh_fused) return false;
  if (ctx->kernel != RHMC_KERNEL_AUTO && ctx->kernel != RHMC_KERNEL_PIXMAJOR) return false;
  return use_pixk(ctx, K, c);
}

// The run's parameters at MH iteration l: multi_gym.run_RHMC's schedules
// (sampler_RHMC.py:1010-1016) set g_ff2 = schedule_g_ff2[l] and beta =
// schedule_beta[l] while l < the schedule's size and keep the last value
// after it; no schedule keeps P's value.
rhmc_params sched_params(const rhmc_params& P, const rhmc_mh_schedule* sc, int l) {
  rhmc_params q = P;
  if (sc && sc->g_ff2 && sc->n_g_ff2 > 0) q.g_ff2 = sc->g_ff2[l < sc->n_g_ff2 ? l : sc->n_g_ff2 - 1];
  if (sc && sc->beta && sc->n_beta > 0) q.beta = sc->beta[l < sc->n_beta ? l : sc->n_beta - 1];
  return q;
}

bool sched_active(const rhmc_mh_schedule* sc) {
  return sc && ((sc->g_ff2 && sc->n_g_ff2 > 0) || (sc->beta && sc->n_beta > 0));
}

// V(q) once, then one mh_pk_iter launch per iteration (rhmc_mhpk.hpp); V
// [n] is the carried V(q) (device scratch).  A schedule changes only g_ff2
// and beta, which this kernel's V does not read (no repulsion here), so the
// carried V stays exact; each launch gets its iteration's constants.
template <int IMG>
int launch_mh_pk(const rhmc_ctx* ctx, MhKArgs k, double* V, hipStream_t s,
                 const rhmc_params* P, const rhmc_mh_schedule* sc) {
  using MP = MhPK<IMG, 10>;
  int W = 4;
  while (W > 1 && MP::lds_bytes(W) > (size_t)ctx->max_lds / 2) W >>= 1;
  const size_t lds = MP::lds_bytes(W);
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "mh_pk LDS");
  k.Df = ctx->d_Df;
  const int64_t waves = (k.n + MP::PK::CPW - 1) / MP::PK::CPW;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  hipLaunchKernelGGL((mh_pk_v0<IMG, 10>), grid, block, lds, s, k, V);
  HIP_TRY(hipGetLastError());
  for (int it = 0; it < k.n_iter; ++it) {
    if (sched_active(sc)) {
      const rhmc_params Pl = sched_params(*P, sc, it);
      int rc = make_consts(&Pl, &k.c);
      if (rc) return rc;
    }
    hipLaunchKernelGGL((mh_pk_iter<IMG, 10>), grid, block, lds, s, k, it, V);
    HIP_TRY(hipGetLastError());
  }
  return RHMC_OK;
}

// The MH outer loop on device buffers (sampler_RHMC.py:1018-1083): per
// iteration begin -> n_steps fused leapfrog -> V(q') -> accept, all queued on
// `s` with no host synchronisation.  `rec` holds device pointers (nullable);
// `sc` (nullable, host arrays) schedules g_ff2 / beta per iteration
// (sampler_RHMC.py:1010-1016, sched_params).
int run_mh(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, int64_t n, int32_t K,
           int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* d_z, const double* d_u,
           uint64_t seed, const rhmc_mh_record* rec, hipStream_t s,
           const rhmc_mh_schedule* sc = nullptr) {
  Consts c;
  int rc = make_consts(P, &c);
  if (rc) return rc;
  if (n_iter < 0 || n_steps < 0) return fail(RHMC_ERR_ARG, "n_iter/n_steps < 0");
  if (sc && (sc->n_g_ff2 < 0 || sc->n_beta < 0 || (sc->n_g_ff2 > 0 && !sc->g_ff2) ||
             (sc->n_beta > 0 && !sc->beta)))
    return fail(RHMC_ERR_ARG, "schedule: negative size or NULL array with a nonzero size");
  const bool sched = sched_active(sc);
  if (sched)  // every iteration's parameters must be valid, not only the first's
    for (int it = 0; it < n_iter; ++it) {
      const rhmc_params Pl = sched_params(*P, sc, it);
      Consts cl;
      if ((rc = make_consts(&Pl, &cl))) return rc;
    }
  if (n == 0 || n_iter == 0) return RHMC_OK;
  if (K == 1 && mh_k1_fused(ctx, c, n)) {
    MhK1Args k;
    k.q = d_q;
    k.D = ctx->d_D;
    k.Df = nullptr;
    k.z = d_z;
    k.u = d_u;
    k.q_chain = rec ? rec->q_chain : nullptr;
    k.E_chain = rec ? rec->E_chain : nullptr;
    k.V_chain = rec ? rec->V_chain : nullptr;
    k.T_chain = rec ? rec->T_chain : nullptr;
    k.accept = rec ? rec->accept : nullptr;
    k.n = n;
    k.n_iter = n_iter;
    k.n_steps = n_steps;
    k.f_pos = f_pos != 0 ? RHMC_V_FLUX_WALL : 0;
    k.it0 = 0;
    k.seed = seed;
    k.c = c;
    auto launch = [&]() {
      switch (ctx->rows) {
        case 32: return launch_mh_k1<32>(ctx, k, s);
        case 48: return launch_mh_k1<48>(ctx, k, s);
        default: return launch_mh_k1<64>(ctx, k, s);
      }
    };
    if (!sched) return launch();
    // scheduled: one launch per iteration with its own constants (V(q) is
    // re-evaluated at each launch's start: the same operations, the same value)
    for (int it = 0; it < n_iter; ++it) {
      const rhmc_params Pl = sched_params(*P, sc, it);
      if ((rc = make_consts(&Pl, &k.c))) return rc;
      k.n_iter = 1;
      k.it0 = it;
      if ((rc = launch())) return rc;
    }
    return RHMC_OK;
  }
  if (K >= 2 && mh_pk_fused(ctx, c, K)) {
    MhKArgs k;
    k.q = d_q;
    k.Df = nullptr;
    k.z = d_z;
    k.u = d_u;
    k.q_chain = rec ? rec->q_chain : nullptr;
    k.E_chain = rec ? rec->E_chain : nullptr;
    k.V_chain = rec ? rec->V_chain : nullptr;
    k.T_chain = rec ? rec->T_chain : nullptr;
    k.accept = rec ? rec->accept : nullptr;
    k.n = n;
    k.K = K;
    k.n_iter = n_iter;
    k.n_steps = n_steps;
    k.f_pos = f_pos != 0 ? RHMC_V_FLUX_WALL : 0;
    k.seed = seed;
    k.c = c;
    const size_t need = (size_t)n * sizeof(double) + 256;
    if (need > ctx->mh_scratch_bytes) {
      if (ctx->mh_scratch) HIP_TRY(hipFree(ctx->mh_scratch));
      ctx->mh_scratch = nullptr;
      ctx->mh_scratch_bytes = 0;
      if (hipMalloc(&ctx->mh_scratch, need) != hipSuccess)
        return fail(RHMC_ERR_NOMEM, "hipMalloc MH scratch failed");
      ctx->mh_scratch_bytes = need;
    }
    double* V = (double*)ctx->mh_scratch;
    return ctx->rows == 32 ? launch_mh_pk<32>(ctx, k, V, s, P, sc)
                           : launch_mh_pk<48>(ctx, k, V, s, P, sc);
  }
  const size_t sb = (size_t)n * 3 * K * sizeof(double), eb = (size_t)n * sizeof(double);
  const size_t need = 2 * sb + 3 * eb + 256;
  if (need > ctx->mh_scratch_bytes) {
    if (ctx->mh_scratch) HIP_TRY(hipFree(ctx->mh_scratch));
    ctx->mh_scratch = nullptr;
    ctx->mh_scratch_bytes = 0;
    if (hipMalloc(&ctx->mh_scratch, need) != hipSuccess)
      return fail(RHMC_ERR_NOMEM, "hipMalloc MH scratch failed");
    ctx->mh_scratch_bytes = need;
  }
  char* b = (char*)ctx->mh_scratch;
  MhArgs m;
  m.q = d_q;
  m.q_prop = (double*)b;
  m.p = (double*)(b + sb);
  m.V_cur = (double*)(b + 2 * sb);
  m.V_prop = (double*)(b + 2 * sb + eb);
  m.E0 = (double*)(b + 2 * sb + 2 * eb);
  m.z = d_z;
  m.u = d_u;
  m.q_chain = rec ? rec->q_chain : nullptr;
  m.E_chain = rec ? rec->E_chain : nullptr;
  m.V_chain = rec ? rec->V_chain : nullptr;
  m.T_chain = rec ? rec->T_chain : nullptr;
  m.accept = rec ? rec->accept : nullptr;
  m.n = n;
  m.K = K;
  m.seed = seed;
  m.c = c;
  f_pos = f_pos != 0 ? RHMC_V_FLUX_WALL : 0;
  if ((rc = launch_energy(ctx, c, d_q, nullptr, m.V_cur, nullptr, n, K, f_pos, s))) return rc;
  // V reads beta through the repulsion term: a beta schedule re-evaluates
  // V(q) at each iteration's start, like the reference's V_initial (:1025)
  const bool v_sched = sched && c.use_Vc && sc->beta && sc->n_beta > 0;
  // begin / end: one thread per chain for few stars, one wave per chain
  // (lanes over the coordinates) from 8 stars
  const bool wave_mh = K >= 8;
  const dim3 grid((unsigned)(wave_mh ? (n + 3) / 4 : (n + 255) / 256)), block(256);
  for (int it = 0; it < n_iter; ++it) {
    m.iter = it;
    const rhmc_params Pl = sched ? sched_params(*P, sc, it) : *P;
    if (sched) {
      if ((rc = make_consts(&Pl, &m.c))) return rc;
      if (v_sched &&
          (rc = launch_energy(ctx, m.c, d_q, nullptr, m.V_cur, nullptr, n, K, f_pos, s)))
        return rc;
    }
    if (wave_mh)
      hipLaunchKernelGGL(mh_begin_wave_kernel, grid, block, 0, s, m);
    else
      hipLaunchKernelGGL(mh_begin_kernel, grid, block, 0, s, m);
    HIP_TRY(hipGetLastError());
    if ((rc = launch_leapfrog(ctx, &Pl, m.q_prop, m.p, n, K, n_steps, nullptr, nullptr, s)))
      return rc;
    if ((rc = launch_energy(ctx, m.c, m.q_prop, nullptr, m.V_prop, nullptr, n, K, f_pos, s)))
      return rc;
    if (wave_mh)
      hipLaunchKernelGGL(mh_end_wave_kernel, grid, block, 0, s, m);
    else
      hipLaunchKernelGGL(mh_end_kernel, grid, block, 0, s, m);
    HIP_TRY(hipGetLastError());
  }
  return RHMC_OK;
}

// Explicit integrators, one star, register-window gradient (rhmc_tiledr.hpp):
// 28-pixel window, fp32 pixel cache when the image is exact in fp32.
template <int IMG, typename DT>
int launch_integrate_tiledr_t(const rhmc_ctx* ctx, const LeapArgsK1& a, int32_t solver,
                              int f_pos, hipStream_t s) {
  using TL = TiledR<IMG, 28, DT>;
  const size_t lds = TL::lds_bytes();
  if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
  constexpr int W = 4;
  const int64_t waves = (a.n_chains + TL::CPW - 1) / TL::CPW;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  if (solver == RHMC_SOLVER_HMC)
    hipLaunchKernelGGL((integrate_k1_tiledr<IMG, 28, DT, RHMC_SOLVER_HMC>), grid, block, lds, s,
                       a, f_pos);
  else if (solver == RHMC_SOLVER_RHMC_NAIVE)
    hipLaunchKernelGGL((integrate_k1_tiledr<IMG, 28, DT, RHMC_SOLVER_RHMC_NAIVE>), grid, block,
                       lds, s, a, f_pos);
  else
    hipLaunchKernelGGL((integrate_k1_tiledr<IMG, 28, DT, RHMC_SOLVER_RHMC_LEAPFROG>), grid,
                       block, lds, s, a, f_pos);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}
template <int IMG>
int launch_integrate_tiledr(const rhmc_ctx* ctx, LeapArgsK1 a, int32_t solver, int f_pos,
                            hipStream_t s) {
  if (ctx->img_f32) {
    a.Df = ctx->d_Df;
    return launch_integrate_tiledr_t<IMG, float>(ctx, a, solver, f_pos, s);
  }
  return launch_integrate_tiledr_t<IMG, double>(ctx, a, solver, f_pos, s);
}

int launch_integrate(rhmc_ctx* ctx, const rhmc_params* P, int32_t solver, double* d_q,
                     double* d_p, int64_t n, int32_t K, int32_t n_steps, int32_t f_pos,
                     int32_t* d_st, hipStream_t s) {
  if (solver == RHMC_SOLVER_IMPLICIT)
    return launch_leapfrog(ctx, P, d_q, d_p, n, K, n_steps, nullptr, d_st, s);
  if (solver < RHMC_SOLVER_HMC || solver > RHMC_SOLVER_RHMC_LEAPFROG)
    return fail(RHMC_ERR_ARG, "unknown solver");
  LeapArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  if (n_steps < 0) return fail(RHMC_ERR_ARG, "n_steps < 0");
  if (n == 0) return RHMC_OK;
  // one star on a 32/48/64-px image: register-window kernel (RHMC_KERNEL_GENERIC
  // / _WINDOWED keep the windowed one)
  const int side = ctx->rows;
  if (K == 1 && !a.c.use_Vc && ctx->rows == ctx->cols && !per_wave_forced(ctx) &&
      ctx->kernel != RHMC_KERNEL_DENSE && (side == 32 || side == 48 || side == 64) &&
      reg_window_ok(28, a.c.inv_two_sig2)) {
    LeapArgsK1 t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = nullptr;
    t.status = d_st;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n;
    t.n_steps = n_steps;
    t.rows = ctx->rows;
    t.cols = ctx->cols;
    t.pad = 0;
    t.c = a.c;
    HIP_TRY(hipSetDevice(ctx->device));
    const int fp = f_pos != 0;
    switch (side) {
      case 32: return launch_integrate_tiledr<32>(ctx, t, solver, fp, s);
      case 48: return launch_integrate_tiledr<48>(ctx, t, solver, fp, s);
      default: return launch_integrate_tiledr<64>(ctx, t, solver, fp, s);
    }
  }
  // many stars: the pixel-major kernel (full image, any PSF width) or the
  // multi-star register-window kernel (rhmc_tiledrk.hpp, 28-px windows);
  // many stars on a small image: the dense kernel (below)
  const int path = dense_path(ctx, K, a.c);
  if (!path && (use_pixk(ctx, K, a.c) || use_tiledrk(ctx, K, a.c))) {
    LeapArgsKR t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = nullptr;
    t.status = d_st;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n;
    t.K = K;
    t.n_steps = n_steps;
    t.side = ctx->rows;
    t.pad = 0;
    t.c = a.c;
    t.dtv = nullptr;
    t.steps = nullptr;
    HIP_TRY(hipSetDevice(ctx->device));
    const int fp = f_pos != 0;
    if (use_pixk(ctx, K, a.c)) {
      if (solver == RHMC_SOLVER_HMC) return launch_pk_side<RHMC_SOLVER_HMC>(ctx, t, s, fp);
      if (solver == RHMC_SOLVER_RHMC_NAIVE)
        return launch_pk_side<RHMC_SOLVER_RHMC_NAIVE>(ctx, t, s, fp);
      return launch_pk_side<RHMC_SOLVER_RHMC_LEAPFROG>(ctx, t, s, fp);
    }
    if (solver == RHMC_SOLVER_HMC) return launch_kr<RHMC_SOLVER_HMC>(ctx, t, fp, s);
    if (solver == RHMC_SOLVER_RHMC_NAIVE) return launch_kr<RHMC_SOLVER_RHMC_NAIVE>(ctx, t, fp, s);
    return launch_kr<RHMC_SOLVER_RHMC_LEAPFROG>(ctx, t, fp, s);
  }
  if (!path && !window_exact(a.c)) return window_unsupported();  // integrate_win_kernel
  a.q = d_q;
  a.p = d_p;
  a.fp_iters = nullptr;
  a.status = d_st;
  a.D = ctx->d_D;
  a.n_chains = n;
  a.K = K;
  a.n_steps = n_steps;
  a.g = make_geometry(ctx->rows, ctx->cols);
  size_t lds;
  int W;
  if (int rc = pick_waves_path(ctx, path, K, &lds, &W)) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  TableLease lease;
  if ((rc = work_tables(ctx, path, K, n, s, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
  const int fp = f_pos != 0;
  return with_path(path, K, [&](auto gt, auto st) {
    launch_integrate_win<typename decltype(gt)::type, decltype(st)::value>(solver, grid, block,
                                                                          lds, s, a, fp);
    HIP_TRY(hipGetLastError());
    return (int)RHMC_OK;
  });
}

template <int IMG>
int launch_hmc_random_k1(const rhmc_ctx* ctx, LeapArgsK1 t, const double* d_dt,
                         const int32_t* d_steps, hipStream_t s) {
  constexpr int W = 4;
  const int64_t waves = (t.n_chains + 3) / 4;
  const dim3 grid((unsigned)((waves + W - 1) / W)), block(W * kWave);
  if (ctx->img_f32) {
    t.Df = ctx->d_Df;
    const size_t lds = TiledR<IMG, 28, float>::lds_bytes();
    if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((hmc_random_k1_tiledr<IMG, float>), grid, block, lds, s, t, d_dt, d_steps);
  } else {
    const size_t lds = TiledR<IMG, 28, double>::lds_bytes();
    if (lds > (size_t)ctx->max_lds) return fail(RHMC_ERR_UNSUPPORTED, "image too large for LDS");
    hipLaunchKernelGGL((hmc_random_k1_tiledr<IMG, double>), grid, block, lds, s, t, d_dt, d_steps);
  }
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

int launch_hmc_random(rhmc_ctx* ctx, const rhmc_params* P, const double* d_dt, double* d_q,
                      double* d_p, const int32_t* d_steps, int64_t n, int32_t K, int32_t* d_st,
                      hipStream_t s) {
  LeapArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  if (n == 0) return RHMC_OK;
  if (!d_dt || !d_steps) return fail(RHMC_ERR_ARG, "dt/steps is NULL");
  // one star on a 32/48/64-px image: register-window kernel (RHMC_KERNEL_GENERIC
  // / _WINDOWED keep the windowed one)
  const int side = ctx->rows;
  if (K == 1 && !a.c.use_Vc && ctx->rows == ctx->cols && (side == 32 || side == 48 || side == 64) &&
      reg_window_ok(28, a.c.inv_two_sig2) && !per_wave_forced(ctx) &&
      ctx->kernel != RHMC_KERNEL_DENSE) {
    LeapArgsK1 t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = nullptr;
    t.status = d_st;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n;
    t.n_steps = 0;
    t.rows = ctx->rows;
    t.cols = ctx->cols;
    t.pad = 0;
    t.c = a.c;
    HIP_TRY(hipSetDevice(ctx->device));
    switch (side) {
      case 32: return launch_hmc_random_k1<32>(ctx, t, d_dt, d_steps, s);
      case 48: return launch_hmc_random_k1<48>(ctx, t, d_dt, d_steps, s);
      default: return launch_hmc_random_k1<64>(ctx, t, d_dt, d_steps, s);
    }
  }
  // many stars: the pixel-major kernel (full image, any PSF width) or the
  // multi-star register-window kernel (rhmc_tiledrk.hpp); RHMC_KERNEL_MULTIWIN
  // forces the latter, GENERIC / WINDOWED the windowed kernel below; many
  // stars on a small image: the dense kernel (below)
  const int path = dense_path(ctx, K, a.c);
  if (!path && (use_pixk(ctx, K, a.c) || use_tiledrk(ctx, K, a.c))) {
    LeapArgsKR t;
    t.q = d_q;
    t.p = d_p;
    t.fp_iters = nullptr;
    t.status = d_st;
    t.D = ctx->d_D;
    t.Df = nullptr;
    t.n_chains = n;
    t.K = K;
    t.n_steps = 0;
    t.side = ctx->rows;
    t.pad = 0;
    t.c = a.c;
    t.dtv = d_dt;
    t.steps = d_steps;
    HIP_TRY(hipSetDevice(ctx->device));
    if (use_pixk(ctx, K, a.c)) return launch_pk_side<kSolverHmcRandom>(ctx, t, s, 0);
    return launch_kr<kSolverHmcRandom>(ctx, t, 0, s);
  }
  if (!path && !window_exact(a.c)) return window_unsupported();  // windowed gradient
  a.q = d_q;
  a.p = d_p;
  a.fp_iters = nullptr;
  a.status = d_st;
  a.D = ctx->d_D;
  a.n_chains = n;
  a.K = K;
  a.n_steps = 0;
  a.g = make_geometry(ctx->rows, ctx->cols);
  size_t lds;
  int W;
  if (int rc = pick_waves_path(ctx, path, K, &lds, &W)) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  TableLease lease;
  if ((rc = work_tables(ctx, path, K, n, s, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n + W - 1) / W)), block(W * kWave);
  return with_path(path, K, [&](auto gt, auto st) {
    using G = typename decltype(gt)::type;
    hipLaunchKernelGGL((hmc_random_win_kernel<G, decltype(st)::value>), grid, block, lds, s, a,
                       d_dt, d_steps);
    HIP_TRY(hipGetLastError());
    return (int)RHMC_OK;
  });
}

// Model image / Poisson realisations (rhmc_datagen.hpp) into d_out
// [max(n_real,1)][rows][cols].
int launch_gen_image(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int32_t K,
                     int32_t rows, int32_t cols, int32_t n_real, uint64_t seed, double* d_out,
                     hipStream_t s) {
  DataArgs a;
  int rc = make_consts(P, &a.c);
  if (rc) return rc;
  if (K < 0 || K > (1 << 20)) return fail(RHMC_ERR_ARG, "K must be in [0, 2^20]");
  if (rows < 1 || cols < 1) return fail(RHMC_ERR_ARG, "rows/cols must be >= 1");
  if (n_real < 0) return fail(RHMC_ERR_ARG, "n_real < 0");
  if (K > 0 && !d_q) return fail(RHMC_ERR_ARG, "q is NULL");
  if (!d_out) return fail(RHMC_ERR_ARG, "out is NULL");
  const int64_t npix = (int64_t)rows * cols;
  const int64_t total = npix * (n_real > 0 ? n_real : 1);
  if (total > ((int64_t)1 << 36)) return fail(RHMC_ERR_ARG, "rows*cols*n_real too large");
  a.q = d_q;
  a.out = d_out;
  a.K = K;
  a.rows = rows;
  a.cols = cols;
  a.poisson = n_real > 0;
  a.n_real = n_real;
  a.seed = seed;
  HIP_TRY(hipSetDevice(ctx->device));
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  hipLaunchKernelGGL(datagen_kernel, grid, block, 0, s, a);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

}  // namespace

namespace {

// fp32 copy of the image and whether it is exact (every pixel == (float)pixel,
// NaN counts as inexact): the register-window kernel caches window pixels in
// fp32 when it is (rhmc_tiledr.hpp).
__global__ void image_f32_kernel(const double* __restrict__ D, float* __restrict__ Df,
                                 int64_t n, int* __restrict__ inexact) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double v = D[i];
    const float f = (float)v;
    Df[i] = f;
    if (!((double)f == v)) atomicOr(inexact, 1);
  }
}

// Called with the new image already enqueued on ctx->stream; synchronises.
int refresh_image_f32(rhmc_ctx* ctx) {
  const int64_t n = (int64_t)ctx->rows * ctx->cols;
  if (ctx->d_Df) HIP_TRY(hipFree(ctx->d_Df));
  ctx->d_Df = nullptr;
  ctx->img_f32 = false;
  if (hipMalloc(&ctx->d_Df, (size_t)n * sizeof(float)) != hipSuccess)
    return fail(RHMC_ERR_NOMEM, "hipMalloc fp32 image failed");
  if (!ctx->d_flag && hipMalloc(&ctx->d_flag, sizeof(int)) != hipSuccess)
    return fail(RHMC_ERR_NOMEM, "hipMalloc flag failed");
  HIP_TRY(hipMemsetAsync(ctx->d_flag, 0, sizeof(int), ctx->stream));
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(image_f32_kernel, dim3(blocks), dim3(256), 0, ctx->stream, ctx->d_D,
                     ctx->d_Df, n, ctx->d_flag);
  HIP_TRY(hipGetLastError());
  int inexact = 1;
  HIP_TRY(hipMemcpyAsync(&inexact, ctx->d_flag, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->img_f32 = inexact == 0;
  return RHMC_OK;
}

}  // namespace

extern "C" {

int rhmc_abi_version(void) { return RHMC_ABI_VERSION; }

const char* rhmc_last_error(void) { return g_err.c_str(); }

int rhmc_device_count(int* n) {
  if (!n) return fail(RHMC_ERR_ARG, "n is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  *n = (e == hipSuccess) ? c : 0;
  return RHMC_OK;
}

int rhmc_ctx_set_image(rhmc_ctx* ctx, const double* D, int32_t rows, int32_t cols) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!D) return fail(RHMC_ERR_ARG, "D is NULL");
  if (rows < 1 || cols < 1) return fail(RHMC_ERR_ARG, "rows/cols must be >= 1");
  if (rows != cols)
    return fail(RHMC_ERR_ARG, "rows must equal cols (reference gauss_PSF is square-only)");
  if ((int64_t)rows * cols > (1 << 26)) return fail(RHMC_ERR_ARG, "image too large");
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t bytes = (size_t)rows * cols * sizeof(double);
  if (ctx->d_D && (ctx->rows * ctx->cols != rows * cols)) {
    HIP_TRY(hipFree(ctx->d_D));
    ctx->d_D = nullptr;
  }
  if (!ctx->d_D && hipMalloc(&ctx->d_D, bytes) != hipSuccess)
    return fail(RHMC_ERR_NOMEM, "hipMalloc image failed");
  HIP_TRY(hipMemcpyAsync(ctx->d_D, D, bytes, hipMemcpyHostToDevice, ctx->stream));
  ctx->rows = rows;
  ctx->cols = cols;
  int rc = refresh_image_f32(ctx);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_ctx_create(int device, const double* D, int32_t rows, int32_t cols, rhmc_ctx** out) {
  if (!out) return fail(RHMC_ERR_ARG, "out is NULL");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RHMC_ERR_HIP, "no HIP device");
  if (device < 0 || device >= n) return fail(RHMC_ERR_ARG, "device out of range");
  HIP_TRY(hipSetDevice(device));
  rhmc_ctx* ctx = new rhmc_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
    delete ctx;
    return fail(RHMC_ERR_HIP, "hipGetDeviceProperties failed");
  }
  ctx->max_lds = (int)prop.sharedMemPerBlock;
  ctx->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return fail(RHMC_ERR_HIP, "hipStreamCreate failed");
  }
  int rc = D ? rhmc_ctx_set_image(ctx, D, rows, cols) : RHMC_OK;  // NULL: no image yet
  if (rc) {
    std::string keep = g_err;
    rhmc_ctx_destroy(ctx);
    g_err = keep;
    return rc;
  }
  *out = ctx;
  return RHMC_OK;
}

int rhmc_ctx_set_option(rhmc_ctx* ctx, int32_t option, int32_t value) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  switch (option) {
    case RHMC_OPT_KERNEL:
      if (value < RHMC_KERNEL_AUTO || value > RHMC_KERNEL_DENSE)
        return fail(RHMC_ERR_ARG, "unknown RHMC_KERNEL_* value " + std::to_string(value));
      ctx->kernel = value;
      return RHMC_OK;
    case RHMC_OPT_MH_FUSED:
      if (value != 0 && value != 1) return fail(RHMC_ERR_ARG, "RHMC_OPT_MH_FUSED must be 0 or 1");
      ctx->mh_fused = value;
      return RHMC_OK;
    case RHMC_OPT_WINDOW_SPLIT:
      if (value != 0 && value != 1 && value != 2 && value != 4)
        return fail(RHMC_ERR_ARG, "RHMC_OPT_WINDOW_SPLIT must be 0, 1, 2 or 4");
      ctx->window_split = value;
      return RHMC_OK;
    case RHMC_OPT_TABLES:
      if (value < RHMC_TABLES_STREAM || value > RHMC_TABLES_POOL_BARRIER)
        return fail(RHMC_ERR_ARG, "RHMC_OPT_TABLES must be 0 ... 6");
#ifndef RHMC_TABLE_DIAG
      // the stream-ordered pool modes reproduce a runtime defect (DESIGN.md
      // section 4a: reused blocks are zeroed under a running launch); only
      // diagnostic builds take them
      if (value > RHMC_TABLES_STREAM_POISON)
        return fail(RHMC_ERR_UNSUPPORTED,
                    "RHMC_OPT_TABLES pool modes exist only in -DRHMC_TABLE_DIAG builds");
#endif
      ctx->table_mode = value;
      return RHMC_OK;
    default:
      return fail(RHMC_ERR_ARG, "unknown option " + std::to_string(option));
  }
}

int rhmc_ctx_get_option(rhmc_ctx* ctx, int32_t option, int32_t* value) {
  if (!ctx || !value) return fail(RHMC_ERR_ARG, "NULL argument");
  switch (option) {
    case RHMC_OPT_KERNEL: *value = ctx->kernel; return RHMC_OK;
    case RHMC_OPT_MH_FUSED: *value = ctx->mh_fused; return RHMC_OK;
    case RHMC_OPT_WINDOW_SPLIT: *value = ctx->window_split; return RHMC_OK;
    case RHMC_OPT_TABLES: *value = ctx->table_mode; return RHMC_OK;
    default: return fail(RHMC_ERR_ARG, "unknown option " + std::to_string(option));
  }
}

int rhmc_ctx_image_device(rhmc_ctx* ctx, const double** d_image) {
  if (!ctx || !d_image) return fail(RHMC_ERR_ARG, "NULL argument");
  *d_image = ctx->d_D;
  return RHMC_OK;
}

void rhmc_ctx_destroy(rhmc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->d_D) (void)hipFree(ctx->d_D);
  if (ctx->d_Df) (void)hipFree(ctx->d_Df);
  if (ctx->d_flag) (void)hipFree(ctx->d_flag);
  if (ctx->scratch) (void)hipFree(ctx->scratch);
  if (ctx->mh_scratch) (void)hipFree(ctx->mh_scratch);
  if (!ctx->tabs.empty() || !ctx->kept.empty())
    (void)hipDeviceSynchronize();   // tables may serve user streams
  for (auto& t : ctx->tabs)
    if (t.buf) t.buf->synced = true;  // user streams may be gone: no per-stream sync
  for (auto& b : ctx->kept) b->s = nullptr;  // pool frees after the device sync above
  ctx->tabs.clear();
  ctx->kept.clear();
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int rhmc_ctx_synchronize(rhmc_ctx* ctx) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_leapfrog_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                         int64_t n_chains, int32_t K, int32_t n_steps, int32_t* d_fp_iters,
                         int32_t* d_status, void* stream) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains > 0 && (!d_q || !d_p)) return fail(RHMC_ERR_ARG, "q/p is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_leapfrog(ctx, P, d_q, d_p, n_chains, K, n_steps, d_fp_iters, d_status, s);
}

int rhmc_ragged_ok(rhmc_ctx* ctx, const rhmc_params* P, int32_t K, int32_t* ok) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!ok) return fail(RHMC_ERR_ARG, "ok is NULL");
  if (!ctx->d_D) return fail(RHMC_ERR_ARG, "no image uploaded");
  Consts c;
  if (int rc = make_consts(P, &c)) return rc;
  *ok = ragged_family(ctx, c, K) != 0 ? 1 : 0;
  return RHMC_OK;
}

int rhmc_leapfrog_ragged_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, double* d_p,
                                int64_t ld, const int64_t* d_rows, const int32_t* d_K,
                                int64_t n, int32_t K_min, int32_t K_max, int32_t n_steps,
                                void* stream) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!ctx->d_D) return fail(RHMC_ERR_ARG, "no image uploaded");
  if (n < 0 || n > ((int64_t)1 << 40)) return fail(RHMC_ERR_ARG, "bad n");
  if (n > 0 && (!d_q || !d_p || !d_K)) return fail(RHMC_ERR_ARG, "q, p or K is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_leapfrog_ragged(ctx, P, d_q, d_p, ld, d_rows, d_K, n, K_min, K_max, n_steps, s);
}

int rhmc_energy_ragged_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int64_t ld,
                              const int64_t* d_rows, const int32_t* d_K, int64_t n,
                              int32_t K_min, int32_t K_max, int32_t f_pos, double* d_V,
                              void* stream) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!ctx->d_D) return fail(RHMC_ERR_ARG, "no image uploaded");
  if (n < 0 || n > ((int64_t)1 << 40)) return fail(RHMC_ERR_ARG, "bad n");
  if (n > 0 && (!d_q || !d_K || !d_V)) return fail(RHMC_ERR_ARG, "q, K or V is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_energy_ragged(ctx, P, d_q, ld, d_rows, d_K, n, K_min, K_max, f_pos, d_V, s);
}

int rhmc_rows_copy_device(rhmc_ctx* ctx, const double* d_src, int64_t ld_src,
                          const int64_t* d_src_rows, double* d_dst, int64_t ld_dst,
                          const int64_t* d_dst_rows, int64_t n, int32_t width, void* stream) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (n < 0 || width < 0 || ld_src < width || ld_dst < width)
    return fail(RHMC_ERR_ARG, "rows copy: need n, width >= 0 and ld_src, ld_dst >= width");
  if (n == 0 || width == 0) return RHMC_OK;
  if (!d_src || !d_dst) return fail(RHMC_ERR_ARG, "rows copy: src or dst is NULL");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  RowsCopyArgs a{d_src, d_dst, d_src_rows, d_dst_rows, ld_src, ld_dst, n, width};
  const int64_t total = n * (int64_t)width;
  hipLaunchKernelGGL(rows_copy_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

int rhmc_kinetic_rows_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, double* d_p,
                             int64_t ld, const int32_t* d_K, const double* d_z,
                             const int64_t* d_zoff, int64_t n, double* d_T, void* stream) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!P) return fail(RHMC_ERR_ARG, "params is NULL");
  if (n < 0 || ld < 3 || n > INT32_MAX) return fail(RHMC_ERR_ARG, "kinetic: bad n or ld");
  if (n == 0) return RHMC_OK;
  if (!d_q || !d_p || !d_K || !d_T || (d_z && !d_zoff))
    return fail(RHMC_ERR_ARG, "kinetic: q, p, K, T (or zoff with z) is NULL");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  KineticArgs a;
  a.q = d_q;
  a.p = d_p;
  a.z = d_z;
  a.zoff = d_zoff;
  a.K = d_K;
  a.T = d_T;
  a.ld = ld;
  a.n = n;
  a.g_ff2 = P->g_ff2;
  a.g_ff = P->g_ff;
  a.g_xx = P->g_xx;
  a.g0 = P->g0;
  a.g1 = P->g1;
  a.g2 = P->g2;
  a.B = P->B_count;
  a.f_low = P->f_low;
  if (ld <= 768)  // up to 256 stars: four chains per block
    hipLaunchKernelGGL((kinetic_rows_kernel<4, 768, 3>), dim3((unsigned)((n + 3) / 4)), dim3(256),
                       0, s, a);
  else  // up to 1024 stars: one chain per block (48 KB of LDS)
    hipLaunchKernelGGL((kinetic_rows_kernel<1, 3072, 5>), dim3((unsigned)n), dim3(64), 0, s, a);
  HIP_TRY(hipGetLastError());
  return RHMC_OK;
}

int rhmc_leapfrog(rhmc_ctx* ctx, const rhmc_params* P, double* q, double* p, int64_t n_chains,
                  int32_t K, int32_t n_steps, int32_t* fp_iters, int32_t* status) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0) return RHMC_OK;
  if (!q || !p) return fail(RHMC_ERR_ARG, "q/p is NULL");
  const size_t sb = (size_t)n_chains * 3 * K * sizeof(double);
  const size_t ib = (size_t)n_chains * 2 * sizeof(int32_t);
  const size_t tb = (size_t)n_chains * sizeof(int32_t);
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, 2 * sb + ib + tb + 256))) return rc;
  char* base = (char*)ctx->scratch;
  double* dq = (double*)base;
  double* dp = (double*)(base + sb);
  int32_t* dit = (int32_t*)(base + 2 * sb);
  int32_t* dst = (int32_t*)(base + 2 * sb + ib);
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dp, p, sb, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = launch_leapfrog(ctx, P, dq, dp, n_chains, K, n_steps, dit, dst, ctx->stream)))
    return rc;
  HIP_TRY(hipMemcpyAsync(q, dq, sb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(p, dp, sb, hipMemcpyDeviceToHost, ctx->stream));
  if (fp_iters) HIP_TRY(hipMemcpyAsync(fp_iters, dit, ib, hipMemcpyDeviceToHost, ctx->stream));
  if (status) HIP_TRY(hipMemcpyAsync(status, dst, tb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_gradient(rhmc_ctx* ctx, const rhmc_params* P, const double* q, double* grad,
                  int64_t n_chains, int32_t K, int32_t kind) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (kind != 0 && kind != 1) return fail(RHMC_ERR_ARG, "kind must be 0 (dVdq) or 1 (dphidq)");
  if (n_chains == 0) return RHMC_OK;
  if (!q || !grad) return fail(RHMC_ERR_ARG, "q/grad is NULL");
  GradArgs a;
  if ((rc = make_consts(P, &a.c))) return rc;
  size_t lds;
  int W;
  const int path = dense_path(ctx, K, a.c);
  const bool win = path || use_windowed(ctx, K);
  if (win && !path && !window_exact(a.c)) return window_unsupported();
  if (win) {
    if ((rc = pick_waves_path(ctx, path, K, &lds, &W))) return rc;
  } else if ((rc = pick_waves(ctx, K, &lds, &W))) {
    return rc;
  }
  const size_t sb = (size_t)n_chains * 3 * K * sizeof(double);
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, 2 * sb + 256))) return rc;
  double* dq = (double*)ctx->scratch;
  double* dg = (double*)((char*)ctx->scratch + sb);
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  a.q = dq;
  a.grad = dg;
  a.D = ctx->d_D;
  a.n_chains = n_chains;
  a.K = K;
  a.with_metric = kind;
  a.g = make_geometry(ctx->rows, ctx->cols);
  TableLease lease;
  if ((rc = work_tables(ctx, path, K, n_chains, ctx->stream, &a.g.work, &lease))) return rc;
  const dim3 grid((unsigned)((n_chains + W - 1) / W)), block(W * kWave);
  if (win) {
    rc = with_path(path, K, [&](auto gt, auto st) {
      using G = typename decltype(gt)::type;
      hipLaunchKernelGGL((gradient_win_kernel<G, decltype(st)::value>), grid, block, lds,
                         ctx->stream, a);
      HIP_TRY(hipGetLastError());
      return (int)RHMC_OK;
    });
    if (rc) return rc;
  } else if ((rc = dispatch_k<GradLaunch>(K, grid, block, lds, ctx->stream, a))) {
    return rc;
  }
  HIP_TRY(hipMemcpyAsync(grad, dg, sb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_energy_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, const double* d_p,
                       double* d_V, double* d_T, int64_t n_chains, int32_t K, int32_t f_pos,
                       void* stream) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0) return RHMC_OK;
  if (!d_q) return fail(RHMC_ERR_ARG, "q is NULL");
  if (d_T && !d_p) return fail(RHMC_ERR_ARG, "T requested but p is NULL");
  Consts c;
  if ((rc = make_consts(P, &c))) return rc;
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_energy(ctx, c, d_q, d_T ? d_p : nullptr, d_V, d_T, n_chains, K, f_pos, s);
}

int rhmc_energy(rhmc_ctx* ctx, const rhmc_params* P, const double* q, const double* p, double* V,
                double* T, int64_t n_chains, int32_t K, int32_t f_pos) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0) return RHMC_OK;
  if (!q) return fail(RHMC_ERR_ARG, "q is NULL");
  if (T && !p) return fail(RHMC_ERR_ARG, "T requested but p is NULL");
  Consts c;
  if ((rc = make_consts(P, &c))) return rc;
  const size_t sb = (size_t)n_chains * 3 * K * sizeof(double);
  const size_t eb = (size_t)n_chains * sizeof(double);
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, 2 * sb + 2 * eb + 256))) return rc;
  char* base = (char*)ctx->scratch;
  double* dq = (double*)base;
  double* dp = (double*)(base + sb);
  double* dV = (double*)(base + 2 * sb);
  double* dT = (double*)(base + 2 * sb + eb);
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  if (T) HIP_TRY(hipMemcpyAsync(dp, p, sb, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = launch_energy(ctx, c, dq, T ? dp : nullptr, V ? dV : nullptr, T ? dT : nullptr,
                          n_chains, K, f_pos, ctx->stream)))
    return rc;
  if (V) HIP_TRY(hipMemcpyAsync(V, dV, eb, hipMemcpyDeviceToHost, ctx->stream));
  if (T) HIP_TRY(hipMemcpyAsync(T, dT, eb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_mh_scheduled_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q,
                             int64_t n_chains, int32_t K, int32_t n_iter, int32_t n_steps,
                             int32_t f_pos, const double* d_z, const double* d_u, uint64_t seed,
                             const rhmc_mh_record* rec, const rhmc_mh_schedule* sched,
                             void* stream) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains > 0 && !d_q) return fail(RHMC_ERR_ARG, "q is NULL");
  HIP_TRY(hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return run_mh(ctx, P, d_q, n_chains, K, n_iter, n_steps, f_pos, d_z, d_u, seed, rec, s, sched);
}

int rhmc_mh_device(rhmc_ctx* ctx, const rhmc_params* P, double* d_q, int64_t n_chains,
                   int32_t K, int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* d_z,
                   const double* d_u, uint64_t seed, const rhmc_mh_record* rec, void* stream) {
  return rhmc_mh_scheduled_device(ctx, P, d_q, n_chains, K, n_iter, n_steps, f_pos, d_z, d_u,
                                  seed, rec, nullptr, stream);
}

int rhmc_mh(rhmc_ctx* ctx, const rhmc_params* P, double* q, int64_t n_chains, int32_t K,
            int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* z, const double* u,
            uint64_t seed, const rhmc_mh_record* rec) {
  return rhmc_mh_scheduled(ctx, P, q, n_chains, K, n_iter, n_steps, f_pos, z, u, seed, rec,
                           nullptr);
}

int rhmc_mh_scheduled(rhmc_ctx* ctx, const rhmc_params* P, double* q, int64_t n_chains,
                      int32_t K, int32_t n_iter, int32_t n_steps, int32_t f_pos, const double* z,
                      const double* u, uint64_t seed, const rhmc_mh_record* rec,
                      const rhmc_mh_schedule* sched) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0 || n_iter == 0) return RHMC_OK;
  if (!q) return fail(RHMC_ERR_ARG, "q is NULL");
  if (n_iter < 0) return fail(RHMC_ERR_ARG, "n_iter < 0");
  const size_t d = (size_t)3 * K;
  const size_t sb = (size_t)n_chains * d * sizeof(double);
  const size_t zb = z ? (size_t)n_iter * sb : 0;
  const size_t ub = u ? (size_t)n_iter * n_chains * sizeof(double) : 0;
  const size_t qcb = (rec && rec->q_chain) ? (size_t)n_iter * sb : 0;
  const size_t eb = (size_t)n_iter * n_chains * sizeof(double);
  const size_t ab = (size_t)n_iter * n_chains * sizeof(int32_t);
  size_t off[8], tot = 0;
  const size_t parts[8] = {sb, zb, ub, qcb, (rec && rec->E_chain) ? eb : 0,
                           (rec && rec->V_chain) ? eb : 0, (rec && rec->T_chain) ? eb : 0,
                           (rec && rec->accept) ? ab : 0};
  for (int i = 0; i < 8; ++i) {
    off[i] = tot;
    tot += (parts[i] + 255) & ~(size_t)255;
  }
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, tot + 256))) return rc;
  char* b = (char*)ctx->scratch;
  double* dq = (double*)(b + off[0]);
  const double* dz = z ? (const double*)(b + off[1]) : nullptr;
  const double* du = u ? (const double*)(b + off[2]) : nullptr;
  rhmc_mh_record drec{qcb ? (double*)(b + off[3]) : nullptr,
                      parts[4] ? (double*)(b + off[4]) : nullptr,
                      parts[5] ? (double*)(b + off[5]) : nullptr,
                      parts[6] ? (double*)(b + off[6]) : nullptr,
                      parts[7] ? (int32_t*)(b + off[7]) : nullptr};
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  if (z) HIP_TRY(hipMemcpyAsync((void*)dz, z, zb, hipMemcpyHostToDevice, ctx->stream));
  if (u) HIP_TRY(hipMemcpyAsync((void*)du, u, ub, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = run_mh(ctx, P, dq, n_chains, K, n_iter, n_steps, f_pos, dz, du, seed, &drec,
                   ctx->stream, sched)))
    return rc;
  HIP_TRY(hipMemcpyAsync(q, dq, sb, hipMemcpyDeviceToHost, ctx->stream));
  if (rec) {
    if (rec->q_chain) HIP_TRY(hipMemcpyAsync(rec->q_chain, drec.q_chain, qcb, hipMemcpyDeviceToHost, ctx->stream));
    if (rec->E_chain) HIP_TRY(hipMemcpyAsync(rec->E_chain, drec.E_chain, eb, hipMemcpyDeviceToHost, ctx->stream));
    if (rec->V_chain) HIP_TRY(hipMemcpyAsync(rec->V_chain, drec.V_chain, eb, hipMemcpyDeviceToHost, ctx->stream));
    if (rec->T_chain) HIP_TRY(hipMemcpyAsync(rec->T_chain, drec.T_chain, eb, hipMemcpyDeviceToHost, ctx->stream));
    if (rec->accept) HIP_TRY(hipMemcpyAsync(rec->accept, drec.accept, ab, hipMemcpyDeviceToHost, ctx->stream));
  }
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_integrate_device(rhmc_ctx* ctx, const rhmc_params* P, int32_t solver, double* d_q,
                          double* d_p, int64_t n_chains, int32_t K, int32_t n_steps,
                          int32_t f_pos, int32_t* d_status, void* stream) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains > 0 && (!d_q || !d_p)) return fail(RHMC_ERR_ARG, "q/p is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_integrate(ctx, P, solver, d_q, d_p, n_chains, K, n_steps, f_pos, d_status, s);
}

int rhmc_integrate(rhmc_ctx* ctx, const rhmc_params* P, int32_t solver, double* q, double* p,
                   int64_t n_chains, int32_t K, int32_t n_steps, int32_t f_pos,
                   int32_t* status) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0) return RHMC_OK;
  if (!q || !p) return fail(RHMC_ERR_ARG, "q/p is NULL");
  const size_t sb = (size_t)n_chains * 3 * K * sizeof(double);
  const size_t tb = (size_t)n_chains * sizeof(int32_t);
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, 2 * sb + tb + 256))) return rc;
  char* base = (char*)ctx->scratch;
  double* dq = (double*)base;
  double* dp = (double*)(base + sb);
  int32_t* dst = (int32_t*)(base + 2 * sb);
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dp, p, sb, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = launch_integrate(ctx, P, solver, dq, dp, n_chains, K, n_steps, f_pos, dst,
                             ctx->stream)))
    return rc;
  HIP_TRY(hipMemcpyAsync(q, dq, sb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(p, dp, sb, hipMemcpyDeviceToHost, ctx->stream));
  if (status) HIP_TRY(hipMemcpyAsync(status, dst, tb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_hmc_random_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_dt,
                           double* d_q, double* d_p, const int32_t* d_steps, int64_t n_chains,
                           int32_t K, int32_t* d_status, void* stream) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains > 0 && (!d_q || !d_p)) return fail(RHMC_ERR_ARG, "q/p is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_hmc_random(ctx, P, d_dt, d_q, d_p, d_steps, n_chains, K, d_status, s);
}

int rhmc_hmc_random(rhmc_ctx* ctx, const rhmc_params* P, const double* dt, double* q, double* p,
                    const int32_t* steps, int64_t n_chains, int32_t K, int32_t* status) {
  int rc = check_common(ctx, n_chains, K);
  if (rc) return rc;
  if (n_chains == 0) return RHMC_OK;
  if (!q || !p || !dt || !steps) return fail(RHMC_ERR_ARG, "q/p/dt/steps is NULL");
  for (int64_t i = 0; i < n_chains; ++i)
    if (steps[i] < 1) return fail(RHMC_ERR_ARG, "steps[i] must be >= 1");
  const size_t sb = (size_t)n_chains * 3 * K * sizeof(double);
  const size_t tb = (size_t)n_chains * sizeof(int32_t);
  const size_t db = (size_t)3 * K * sizeof(double);
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  HIP_TRY(hipSetDevice(ctx->device));
  if ((rc = ensure_scratch(ctx, 2 * up(sb) + 2 * up(tb) + up(db)))) return rc;
  char* base = (char*)ctx->scratch;
  double* dq = (double*)base;
  double* dp = (double*)(base + up(sb));
  int32_t* dst = (int32_t*)(base + 2 * up(sb));
  int32_t* dsteps = (int32_t*)(base + 2 * up(sb) + up(tb));
  double* ddt = (double*)(base + 2 * up(sb) + 2 * up(tb));
  HIP_TRY(hipMemcpyAsync(dq, q, sb, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dp, p, sb, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(dsteps, steps, tb, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(ddt, dt, db, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = launch_hmc_random(ctx, P, ddt, dq, dp, dsteps, n_chains, K, dst, ctx->stream)))
    return rc;
  HIP_TRY(hipMemcpyAsync(q, dq, sb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipMemcpyAsync(p, dp, sb, hipMemcpyDeviceToHost, ctx->stream));
  if (status) HIP_TRY(hipMemcpyAsync(status, dst, tb, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

int rhmc_gen_image_device(rhmc_ctx* ctx, const rhmc_params* P, const double* d_q, int32_t K,
                          int32_t rows, int32_t cols, int32_t n_real, uint64_t seed,
                          double* d_out, void* stream) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  return launch_gen_image(ctx, P, d_q, K, rows, cols, n_real, seed, d_out, s);
}

int rhmc_gen_image(rhmc_ctx* ctx, const rhmc_params* P, const double* q, int32_t K, int32_t rows,
                   int32_t cols, int32_t n_real, uint64_t seed, double* out, int32_t install) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  if (!out && !install) return fail(RHMC_ERR_ARG, "out is NULL and install == 0");
  if (K < 0 || K > (1 << 20)) return fail(RHMC_ERR_ARG, "K must be in [0, 2^20]");
  if (K > 0 && !q) return fail(RHMC_ERR_ARG, "q is NULL");
  if (rows < 1 || cols < 1) return fail(RHMC_ERR_ARG, "rows/cols must be >= 1");
  if (n_real < 0) return fail(RHMC_ERR_ARG, "n_real < 0");
  if (install && rows != cols)
    return fail(RHMC_ERR_ARG, "rows must equal cols to install the image");
  if (install && (int64_t)rows * cols > (1 << 26)) return fail(RHMC_ERR_ARG, "image too large");
  const int64_t npix = (int64_t)rows * cols;
  const int64_t nimg = n_real > 0 ? n_real : 1;
  if (npix * nimg > ((int64_t)1 << 36)) return fail(RHMC_ERR_ARG, "rows*cols*n_real too large");
  const size_t qb = ((size_t)3 * K * sizeof(double) + 255) & ~(size_t)255;
  const size_t ob = (size_t)(npix * nimg) * sizeof(double);
  HIP_TRY(hipSetDevice(ctx->device));
  int rc = ensure_scratch(ctx, qb + ob + 256);
  if (rc) return rc;
  double* dq = (double*)ctx->scratch;
  double* dout = (double*)((char*)ctx->scratch + qb);
  if (K > 0)
    HIP_TRY(hipMemcpyAsync(dq, q, (size_t)3 * K * sizeof(double), hipMemcpyHostToDevice,
                           ctx->stream));
  if ((rc = launch_gen_image(ctx, P, dq, K, rows, cols, n_real, seed, dout, ctx->stream)))
    return rc;
  if (install) {  // image 0 becomes the context's data image (stays on the device)
    const size_t bytes = (size_t)npix * sizeof(double);
    if (ctx->d_D && (int64_t)ctx->rows * ctx->cols != npix) {
      HIP_TRY(hipStreamSynchronize(ctx->stream));
      HIP_TRY(hipFree(ctx->d_D));
      ctx->d_D = nullptr;
    }
    if (!ctx->d_D && hipMalloc(&ctx->d_D, bytes) != hipSuccess)
      return fail(RHMC_ERR_NOMEM, "hipMalloc image failed");
    HIP_TRY(hipMemcpyAsync(ctx->d_D, dout, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    ctx->rows = rows;
    ctx->cols = cols;
    if ((rc = refresh_image_f32(ctx))) return rc;
  }
  if (out) HIP_TRY(hipMemcpyAsync(out, dout, ob, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return RHMC_OK;
}

#ifdef RHMC_TABLE_CANARY
// Diagnostic builds only (not declared in rhmc.h): the table-region conflicts
// seen since the last call (rhmc_windowed.hpp canary_leave: calls that saw a
// bump, gradients / potentials that saw one, gradient / potential bumps
// seen); resets them.
int rhmc_debug_table_conflicts(int64_t* out5) {
  unsigned long long h[6] = {0, 0, 0, 0, 0, 0};
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_tab_conflicts), sizeof(h)));
  const unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_tab_conflicts), z, sizeof(z)));
  for (int i = 0; i < 5; ++i) out5[i] = (int64_t)h[i];
  return RHMC_OK;
}
// The first 8 foreign header values a canary saw (raw 64-bit), [0] = how many.
int rhmc_debug_table_seen(uint64_t* out9) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out9, HIP_SYMBOL(g_tab_seen), 9 * sizeof(uint64_t)));
  return RHMC_OK;
}
#endif
}  // extern "C"
#endif  // RHMC_KERNELS_ONLY
