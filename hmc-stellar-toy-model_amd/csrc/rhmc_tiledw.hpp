// rhmc_tiledw.hpp — single-star leapfrog on a 32 x 32 pixel window per chain,
// 64/LPC chains per wave64 (LPC = 32 or 16 lanes per chain).
//
// Every pixel of the reference's dphidq sum (sampler_RHMC.py:365-425) carries
// a factor PSF_ij; a pixel centre >= 15.5 px from the star has
// PSF/peak = exp(-15.5^2 / (2 sigma^2)) <= 2^-70 whenever sigma <= 1.574 px
// (the reference's PSF: sigma = 3.5/2.354 = 1.487 px, 2.4e-24), so its term is
// below 1e-20 of the peak pixel's and far below one rounding of the fp64 sums
// — dropping it does not change the computed gradient beyond the summation's
// own rounding.  The window rows are win_base(x) = floor(x) - 16 .. + 31
// (clamped into the image), likewise the columns, so a 48 x 48 step touches
// 1024 pixels instead of 2304; launch_leapfrog uses this kernel only when the
// bound above holds (window_exact), else the full-image tiled kernels.
//
// Layout: D row-major in LDS with pitch P = IMG + 1 (P % 4 == 1).  Lane (a, b)
// of a chain's group (a = m / GC in 0..3, b = m % GC, GC = LPC/4) owns window
// rows 8a .. 8a+7 and the strided window columns b, b+GC, b+2GC, ...; the
// addresses of one read are then (8a P + b) mod 32 distinct doubles within a
// group — conflict-free — while the row/column product structure that
// separability needs is kept.
#pragma once
#include "rhmc_exp.hpp"
#include "rhmc_k1step.hpp"
#include "rhmc_tiled.hpp"
#include "rhmc_tiled2.hpp"
#include "rhmc_wave.hpp"
#include "rhmc_windowed.hpp"

namespace rhmc {

template <int IMG, int LPC>
struct TiledW {
  static_assert(LPC == 16 || LPC == 32, "LPC in {16, 32}");
  static constexpr int CPW = kWave / LPC;  // chains per wave
  static constexpr int GC = LPC / 4;       // lane grid columns (4 lane rows)
  static constexpr int P = IMG + 1;        // LDS row pitch
  static constexpr int TR = 8;             // window rows per lane
  static constexpr int TC = kWin / GC;     // window columns per lane (stride GC)
  static constexpr int NE = 2 * kWin / LPC;  // factor entries per lane
  static constexpr int TAB = CPW * 128;    // per wave: 64 (value, offset) pairs per chain
  static_assert(IMG >= kWin && IMG % 4 == 0, "window inside the image, P % 4 == 1");

  // LDS: D [IMG][P], the exp table, per-wave factor tables.
  static constexpr int EXP_OFF = IMG * P;
  static constexpr int TAB_OFF = IMG * P + kExpTab;
  static __host__ __device__ constexpr size_t lds_doubles(int waves) {
    return (size_t)TAB_OFF + (size_t)waves * TAB;
  }
  static __device__ __forceinline__ int origin(double v) {
    const int o = win_base(v);
    return o < 0 ? 0 : (o > IMG - kWin ? IMG - kWin : o);
  }

  static __device__ __forceinline__ double group_sum(double v) {
    v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_move<0x141>(v);  // row_half_mirror
    v += dpp_move<0x140>(v);  // row_mirror: 16-lane sums
    if constexpr (LPC == 32) v = swap_add<false>(v);  // v_permlane16_swap
    return v;
  }

  // Pixel part of the group's chain's dphidq (every lane of the group gets
  // it); the metric and prior terms are added by k1_steps.
  static __device__ __forceinline__ void gradient(const double* __restrict__ sD, double* tab,
                                                  double f, double x, double y, const Consts& c,
                                                  const LeanConsts& lc, double& gf, double& gx,
                                                  double& gy) {
    const int lane = lane_id();
    const int h = lane / LPC, m = lane % LPC;
    const int a = m / GC, b = m % GC;
    const int r0 = origin(x), c0 = origin(y);
    double* t = tab + h * 128;  // rows [32][2], cols [32][2]
#pragma unroll
    for (int n = 0; n < kWin / LPC; ++n) {
      const int e = n * LPC + m;
      const double vr = ((r0 + e) + 0.5) - x;
      t[2 * e] = exp_neg(-(vr * vr) * lc.inv_two_sig2, sD + EXP_OFF);
      t[2 * e + 1] = ((double)(r0 + e) - x) + 0.5;
      const double vc = ((c0 + e) + 0.5) - y;
      t[64 + 2 * e] = exp_neg(-(vc * vc) * lc.inv_two_sig2, sD + EXP_OFF) * lc.inv_norm;
      t[64 + 2 * e + 1] = ((double)(c0 + e) - y) + 0.5;
    }
    wave_lds_sync();
    double ex[TR], dx[TR], ey[TC], dy[TC];
#pragma unroll
    for (int k = 0; k < TR; ++k) {
      ex[k] = t[2 * (8 * a + k)];
      dx[k] = t[2 * (8 * a + k) + 1];
    }
#pragma unroll
    for (int k = 0; k < TC; ++k) {
      ey[k] = t[64 + 2 * (b + GC * k)];
      dy[k] = t[64 + 2 * (b + GC * k) + 1];
    }
    wave_lds_sync();

    // s_ij = D_ij / Lambda_ij - 1 and separable sums (see rhmc_tiled2.hpp).
    const double* sDl = sD + (r0 + 8 * a) * P + c0 + b;
    double fex[TR], R[TR], C[TC];
#pragma unroll
    for (int k = 0; k < TR; ++k) fex[k] = f * ex[k];
#pragma unroll
    for (int pp = 0; pp < TR * TC; pp += 2) {  // row-major pairs (i, j), (i, j + 1)
      const int i1 = pp / TC, j1 = pp % TC, i2 = (pp + 1) / TC, j2 = (pp + 1) % TC;
      const double d1 = sDl[i1 * P + GC * j1], d2 = sDl[i2 * P + GC * j2];
      const double l1 = fma(fex[i1], ey[j1], c.B), l2 = fma(fex[i2], ey[j2], c.B);  // :373-376
      const double L = l1 * l2;
      double r = __builtin_amdgcn_rcp(L);
      r = fma(r, fma(-L, r, 1.0), r);
      const double s1 = fma(d1, l2 * r, -1.0), s2 = fma(d2, l1 * r, -1.0);  // D/Lambda - 1 (:379)
      R[i1] = (j1 == 0) ? ey[j1] * s1 : fma(ey[j1], s1, R[i1]);
      C[j1] = (i1 == 0) ? ex[i1] * s1 : fma(ex[i1], s1, C[j1]);
      R[i2] = fma(ey[j2], s2, R[i2]);
      C[j2] = (i2 == 0) ? ex[i2] * s2 : fma(ex[i2], s2, C[j2]);
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int k = 0; k < TR; ++k) {
      const double tt = ex[k] * R[k];
      a0 += tt;
      a1 = fma(tt, dx[k], a1);
    }
#pragma unroll
    for (int k = 0; k < TC; ++k) a2 = fma(ey[k] * C[k], dy[k], a2);
    const double s0 = group_sum(a0);
    const double s1 = group_sum(a1);
    const double s2 = group_sum(a2);
    gf = -s0;                                          // :404
    gx = -s1 * f * lc.inv_var;                         // :405
    gy = -s2 * f * lc.inv_var;                         // :406
  }
};

// PROF (tools only): fp_iters[c] = (gradient, rest) cycles per step.
template <int IMG, int LPC, bool PROF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
leapfrog_k1_tiledw(LeapArgsK1 a) {
  using TL = TiledW<IMG, LPC>;
  extern __shared__ double lds[];
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    lds[r * TL::P + cc] = a.D[e];
  }
  exp_tab_fill(lds + TL::EXP_OFF);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / LPC;
  const int64_t chain = TL::CPW * wave + h;
  const bool real = chain < a.n_chains;            // ragged tail: mirror the wave's first chain
  const int64_t base = (real ? chain : TL::CPW * wave) * 3;
  double* tab = lds + TL::TAB_OFF + (threadIdx.x / kWave) * TL::TAB;

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const LeanConsts lc = lean_consts(c);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  long long prof[4] = {0, 0, 0, 0};
  k1_steps<PROF>(f, x, y, pf, px, py, a.n_steps, (double)(IMG - 1), c, lc,
                 [&](double f_, double x_, double y_, double& gf, double& gx, double& gy) {
                   TL::gradient(lds, tab, f_, x_, y_, c, lc, gf, gx, gy);
                 },
                 it_p, it_q, st, prof);
  if constexpr (PROF) {
    const int ns = a.n_steps > 0 ? a.n_steps : 1;
    it_p = (int)(prof[0] / ns);
    it_q = (int)((prof[1] + prof[2] + prof[3]) / ns);
  }

  if ((lane % LPC) == 0 && real) {
    if (!(isfinite(f) && isfinite(x) && isfinite(y) && isfinite(pf) && isfinite(px) &&
          isfinite(py)))
      st |= RHMC_STATUS_NONFINITE;
    a.q[base] = f;
    a.q[base + 1] = x;
    a.q[base + 2] = y;
    a.p[base] = pf;
    a.p[base + 1] = px;
    a.p[base + 2] = py;
    if (a.status) a.status[chain] = (int32_t)st;
    if (a.fp_iters) {
      a.fp_iters[2 * chain] = it_p;
      a.fp_iters[2 * chain + 1] = it_q;
    }
  }
}

}  // namespace rhmc
