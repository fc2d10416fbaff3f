// rhmc_pixk.hpp — multi-star leapfrog, PIXEL-MAJOR gradient for small images
// with a few stars (C3: 48x48, K = 10), where every star's window covers most
// of the image and the window-major kernel (rhmc_tiledrk.hpp) evaluates Lambda
// about 3.9 times per pixel.  Here Lambda is evaluated once per image pixel,
// as the reference does (sampler_RHMC.py:373-376, full image), and the three
// per-star sums of dphidq (:404-406) come out of separable accumulations:
//   s0_k = sum_j ey_k(j) sum_i ex_k(i) s_ij
//   s1_k = sum_j ey_k(j) sum_i (i + 1/2 - x_k) ex_k(i) s_ij
//   s2_k = sum_j (j + 1/2 - y_k) ey_k(j) sum_i ex_k(i) s_ij,  s = D/Lambda - 1.
// 32 lanes per chain (two chains per wave64): lane m = 16 rh + cg owns image
// columns cg, cg + 16, ... and rows rh IMG/2 .. rh IMG/2 + IMG/2 - 1.  Row
// factors ex_k(i), (i + 1/2 - x_k) ex_k(i) sit in a per-chain LDS table
// [IMG][KMAX][2] (rebuilt per gradient, read by 16 lanes at a time); the
// column factors of the lane's current column are in registers (f ey for
// Lambda, ey for the sums).  The step loop is km_steps (rhmc_tiledrk.hpp).
#pragma once
#include "rhmc_tiledrk.hpp"

namespace rhmc {

template <int IMG, int KMAX>
struct PixK {
  static constexpr int LPC = 32;           // lanes per chain
  static constexpr int CPW = kWave / LPC;  // chains per wave
  static constexpr int NC = IMG / 16;      // columns per lane
  static constexpr int NR = IMG / 2;       // rows per lane
  static_assert(IMG % 32 == 0 || IMG == 48, "image side");
  static constexpr size_t row_tab_doubles() { return (size_t)IMG * KMAX * 2; }
  // LDS: exp table, star tables (32 per chain), row tables, image (fp32 [IMG][IMG]).
  static __host__ __device__ constexpr size_t lds_bytes(int waves) {
    return kExpTab * sizeof(double) + (size_t)waves * CPW * LPC * sizeof(KRStar) +
           (size_t)waves * CPW * row_tab_doubles() * sizeof(double) +
           (size_t)IMG * IMG * sizeof(float);
  }

  // Pixel part of dphidq (:365-425 without metric / prior): lane m < K gets
  // star m's; the star table `tab` holds the chain's (f, x, y).
  static __device__ __forceinline__ void gradient(const double* __restrict__ etab,
                                                  const float* __restrict__ simg,
                                                  const KRStar* tab, double* rtab, int K,
                                                  const Consts& c, const LeanConsts& lc,
                                                  double& gf, double& gx, double& gy) {
    const int m = lane_id() & (LPC - 1);
    const int cg = m & 15, rh = m >> 4;
    wave_lds_sync();  // the previous gradient's table reads are done
    for (int e = m; e < IMG * KMAX; e += LPC) {
      const int i = e / KMAX, k = e - (e / KMAX) * KMAX;
      double ex = 0.0, dex = 0.0;
      if (k < K) {
        const double v = ((double)i + 0.5) - tab[k].x;
        ex = exp_neg(-(v * v) * lc.inv_two_sig2, etab);
        dex = v * ex;
      }
      rtab[2 * e] = ex;
      rtab[2 * e + 1] = dex;
    }
    wave_lds_sync();
    double A0[KMAX], A1[KMAX], A2[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) A0[k] = A1[k] = A2[k] = 0.0;
#pragma unroll 1
    for (int ci = 0; ci < NC; ++ci) {
      const int j = cg + 16 * ci;
      // column factors: f ey for Lambda here, ey again at the column's end
      // (recomputed rather than held: registers)
      auto col_factor = [&](int k) {
        const double v = ((double)j + 0.5) - tab[k].y;
        return exp_neg(-(v * v) * lc.inv_two_sig2, etab) * lc.inv_norm;
      };
      double fey[KMAX], c0[KMAX], c1[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        fey[k] = c0[k] = c1[k] = 0.0;
        if (k < K) fey[k] = tab[k].f * col_factor(k);  // wave-uniform guard
      }
      const double* rt = rtab + (size_t)(rh * NR) * KMAX * 2;
      const float* dc = simg + (rh * NR) * IMG + j;
// rows per loop iteration (measured at C3: 1 -> 4 +2 %, 8 equal to 4, a full
// unroll of the 24 rows 22x slower)
#ifndef RHMC_PK_ROW_UNROLL
#define RHMC_PK_ROW_UNROLL 4
#endif
#pragma unroll RHMC_PK_ROW_UNROLL
      for (int r = 0; r < NR; ++r) {
        const double* t0 = rt + (size_t)r * KMAX * 2;
        double l0 = c.B;  // Lambda, stars in ascending order (:373-376)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) l0 = fma(t0[2 * k], fey[k], l0);
        const double s0 = fma((double)dc[r * IMG], rcp_nr1(l0), -1.0);  // D/Lambda - 1 (:379)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
          c0[k] = fma(t0[2 * k], s0, c0[k]);
          c1[k] = fma(t0[2 * k + 1], s0, c1[k]);
        }
      }
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {  // wave-uniform
          const double ey = col_factor(k);
          const double dy = ((double)j + 0.5) - tab[k].y;
          A0[k] = fma(ey, c0[k], A0[k]);
          A1[k] = fma(ey, c1[k], A1[k]);
          A2[k] = fma(dy * ey, c0[k], A2[k]);
        }
      }
    }
    gf = gx = gy = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {  // wave-uniform
        const double s0 = half_sum_dpp(A0[k]);
        const double s1 = half_sum_dpp(A1[k]);
        const double s2 = half_sum_dpp(A2[k]);
        if (m == k) {
          const double fk = tab[k].f;
          gf = -s0;                      // :404
          gx = -s1 * fk * lc.inv_var;    // :405
          gy = -s2 * fk * lc.inv_var;    // :406
        }
      }
    }
  }
};

// Two chains per wave, W waves per workgroup, one star per lane (K <= KMAX).
// SOLVER as in leapfrog_kr: RHMC_single_step, an explicit integrator (f_pos =
// the flux wall) or kSolverHmcRandom.
template <int IMG, int KMAX, int SOLVER = RHMC_SOLVER_IMPLICIT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
leapfrog_pk(LeapArgsKR a, int f_pos) {
  using PK = PixK<IMG, KMAX>;
  extern __shared__ double lds[];
  const int W = blockDim.x / kWave;
  exp_tab_fill(lds);
  float* simg = reinterpret_cast<float*>(lds + kExpTab + (size_t)W * PK::CPW * PK::LPC * 4 +
                                         (size_t)W * PK::CPW * PK::row_tab_doubles());
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) simg[e] = a.Df[e];
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (PK::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / PK::LPC, m = lane % PK::LPC;
  const int64_t chain = PK::CPW * wave + h;
  const bool real = chain < a.n_chains;  // ragged tail: mirror the wave's first chain
  const int64_t chain_r = real ? chain : PK::CPW * wave;
  const int64_t cbase = chain_r * 3 * (int64_t)a.K;
  const int slot = (threadIdx.x / kWave) * PK::CPW + h;
  KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + slot * PK::LPC;
  double* rtab = lds + kExpTab + (size_t)W * PK::CPW * PK::LPC * 4 + (size_t)slot * PK::row_tab_doubles();
  const Consts& c = a.c;
  const LeanConsts lc = lean_consts(c);
  const int K = a.K;
  double f[1], x[1], y[1], pf[1], px[1], py[1];
  bool own[1];
  own[0] = m < K;
  const int64_t e = cbase + 3 * (int64_t)(own[0] ? m : 0);
  f[0] = own[0] ? a.q[e] : 1.0;
  x[0] = own[0] ? a.q[e + 1] : 0.0;
  y[0] = own[0] ? a.q[e + 2] : 0.0;
  pf[0] = own[0] ? a.p[e] : 0.0;
  px[0] = own[0] ? a.p[e + 1] : 0.0;
  py[0] = own[0] ? a.p[e + 2] : 0.0;
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  auto grad = [&](const double (&)[1], const double (&)[1], double (&gf)[1], double (&gx)[1],
                  double (&gy)[1]) {
    PK::gradient(lds, simg, tab, rtab, K, c, lc, gf[0], gx[0], gy[0]);
  };
  if constexpr (SOLVER == RHMC_SOLVER_IMPLICIT) {
    km_steps<1>(f, x, y, pf, px, py, own, tab, a.n_steps, (double)(IMG - 1), c, lc, grad, it_p,
                it_q, st);
  } else if constexpr (SOLVER == kSolverHmcRandom) {
    if (km_hmc_random_steps<1>(f, x, y, pf, px, py, own, tab, a.steps[chain_r], a.dtv, c,
                               grad)) {
      st |= RHMC_STATUS_REFLECT_F;  // p_tmp stays the starting momentum (:547-550)
      pf[0] = own[0] ? a.p[e] : 0.0;
      px[0] = own[0] ? a.p[e + 1] : 0.0;
      py[0] = own[0] ? a.p[e + 2] : 0.0;
    }
  } else {
    km_explicit_steps<SOLVER, 1>(f, x, y, pf, px, py, own, tab, a.n_steps, f_pos, c, lc, grad,
                                 st);
  }
  unsigned nf = 0u;
  if (own[0] && real) {
    if (!(isfinite(f[0]) && isfinite(x[0]) && isfinite(y[0]) && isfinite(pf[0]) &&
          isfinite(px[0]) && isfinite(py[0])))
      nf = RHMC_STATUS_NONFINITE;
    a.q[e] = f[0];
    a.q[e + 1] = x[0];
    a.q[e + 2] = y[0];
    a.p[e] = pf[0];
    a.p[e + 1] = px[0];
    a.p[e + 2] = py[0];
  }
  unsigned all = st | nf;
#pragma unroll
  for (int d = 16; d >= 1; d >>= 1) all |= (unsigned)__shfl_xor((int)all, d, kWave);
  if (m == 0 && real) {
    if (a.status) a.status[chain] = (int32_t)all;
    if (a.fp_iters) {
      a.fp_iters[2 * chain] = it_p;
      a.fp_iters[2 * chain + 1] = it_q;
    }
  }
}

}  // namespace rhmc
