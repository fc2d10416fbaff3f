// rhmc_tiledg.hpp — single-star leapfrog with 64/LPC chains per wave64
// (LPC = lanes per chain: 16, 32 or 64).
//
// A launch of C chains holds C/CPW waves (CPW = 64/LPC chains per wave); the
// serial part of a step — PSF factor exps, all-reduces, the p/q fixed-point
// loops — costs the same wave instructions for all CPW chains of a wave, the
// pixel work per chain does not depend on LPC.  At the headline 4096 chains on
// 1024 SIMDs, LPC=16 puts 4 chains in one wave per SIMD (half the serial
// instructions of LPC=32, no second wave to hide latency behind).
//   * lane (h, m): h = lane / LPC selects the chain, m = lane % LPC indexes a
//     GR x GC lane grid over the image: TR = IMG/GR rows x TC = IMG/GC columns
//     per lane;
//   * D in LDS as [TR*TC][LPC] — lanes m, m+LPC, ... read the same address;
//   * the per-chain sums: DPP inside 16-lane rows (+ permlane swaps for
//     LPC = 32, 64), bit-identical in all lanes of the group.
#pragma once
#include "rhmc_tiled.hpp"
#include "rhmc_wave.hpp"

namespace rhmc {

template <int LPC>
__device__ __forceinline__ double group_sum(double v) {
  v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_move<0x141>(v);  // row_half_mirror: 8-lane sums
  v += dpp_move<0x140>(v);  // row_mirror: 16-lane sums
  if constexpr (LPC >= 32) v = swap_add<false>(v);  // v_permlane16_swap
  if constexpr (LPC >= 64) v = swap_add<true>(v);   // v_permlane32_swap
  return v;
}

template <int IMG, int LPC>
struct TiledG {
  static_assert(LPC == 16 || LPC == 32 || LPC == 64, "LPC in {16, 32, 64}");
  static constexpr int CPW = kWave / LPC;         // chains per wave
  static constexpr int GR = (LPC == 64) ? 8 : 4;  // lane grid rows
  static constexpr int GC = LPC / GR;             // lane grid columns
  static constexpr int TR = IMG / GR;             // image rows per lane
  static constexpr int TC = IMG / GC;             // image columns per lane
  static constexpr int NPIX = IMG * IMG;
  static constexpr int TAB = CPW * 4 * IMG;       // per wave: (ex,dx) rows + (ey,dy) cols
  static constexpr int NE = (2 * IMG + LPC - 1) / LPC;  // factor entries per lane
  static_assert(IMG % GR == 0 && IMG % GC == 0 && IMG <= 64, "image tiling");
  static_assert((TR * TC) % 2 == 0, "pixel pairs");

  static __host__ __device__ constexpr size_t lds_doubles(int waves) {
    return (size_t)NPIX + (size_t)waves * TAB;
  }
  static __device__ __forceinline__ int tiled_index(int r, int c) {
    const int m = (r / TR) * GC + (c / TC);
    return ((r % TR) * TC + (c % TC)) * LPC + m;
  }

  // dphidq of the group's chain (every lane of the group gets it).
  template <bool PROF = false>
  static __device__ __forceinline__ void gradient(const double* __restrict__ sDm, double* tab,
                                                  double f, double x, double y, const Consts& c,
                                                  const LeanConsts& lc, double& gf, double& gx,
                                                  double& gy, long long* t_tab = nullptr) {
    long long t0 = 0;
    if constexpr (PROF) t0 = clock64();
    const int lane = lane_id();
    const int h = lane / LPC, m = lane % LPC;
    const int ta = m / GC, tb = m % GC;
    double* t = tab + h * 4 * IMG;  // this chain: rows [IMG][2], cols [IMG][2]
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = n * LPC + m;
      if (e < 2 * IMG) {
        const bool row = e < IMG;
        const int d = row ? e : e - IMG;
        const double ctr = row ? x : y;
        const double v = (d + 0.5) - ctr;
        double val = exp(-(v * v) * lc.inv_two_sig2);
        if (!row) val *= lc.inv_norm;
        t[2 * e] = val;
        t[2 * e + 1] = ((double)d - ctr) + 0.5;
      }
    }
    wave_lds_sync();
    double ex[TR], dx[TR], ey[TC], dy[TC];
#pragma unroll
    for (int k = 0; k < TR; ++k) {
      ex[k] = t[2 * (ta * TR + k)];
      dx[k] = t[2 * (ta * TR + k) + 1];
    }
#pragma unroll
    for (int k = 0; k < TC; ++k) {
      ey[k] = t[2 * IMG + 2 * (tb * TC + k)];
      dy[k] = t[2 * IMG + 2 * (tb * TC + k) + 1];
    }
    wave_lds_sync();
    if constexpr (PROF) *t_tab += clock64() - t0;

    // s_ij = D_ij / Lambda_ij - 1; separability (PSF_ij = ex_i ey_j):
    //   sum PSF s = sum_i ex_i R_i, sum PSF s dx = sum_i ex_i dx_i R_i,
    //   sum PSF s dy = sum_j ey_j dy_j C_j, R_i = sum_j ey_j s_ij, C_j = sum_i ex_i s_ij.
    double fex[TR], R[TR], C[TC];
#pragma unroll
    for (int k = 0; k < TR; ++k) {
      fex[k] = f * ex[k];
      R[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < TC; ++k) C[k] = 0.0;
#pragma unroll
    for (int pp = 0; pp < TR * TC; pp += 2) {
      const int i1 = pp / TC, j1 = pp % TC, i2 = (pp + 1) / TC, j2 = (pp + 1) % TC;
      const double d1 = sDm[pp * LPC], d2 = sDm[(pp + 1) * LPC];
      const double l1 = fma(fex[i1], ey[j1], c.B), l2 = fma(fex[i2], ey[j2], c.B);  // :373-376
      const double L = l1 * l2;
      double r = __builtin_amdgcn_rcp(L);
      r = fma(r, fma(-L, r, 1.0), r);
      const double s1 = fma(d1, l2 * r, -1.0), s2 = fma(d2, l1 * r, -1.0);  // D/Lambda - 1 (:379)
      R[i1] = fma(ey[j1], s1, R[i1]);
      C[j1] = fma(ex[i1], s1, C[j1]);
      R[i2] = fma(ey[j2], s2, R[i2]);
      C[j2] = fma(ex[i2], s2, C[j2]);
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
    const double s0 = group_sum<LPC>(a0);
    const double s1 = group_sum<LPC>(a1);
    const double s2 = group_sum<LPC>(a2);
    gf = -s0;                                          // :404
    gx = -s1 * f * lc.inv_var;                         // :405
    gy = -s2 * f * lc.inv_var;                         // :406
    if (c.use_prior) gf += c.alpha * rcp_nr(f);        // :408-409
    gf += metric_flux_term_lean(f, lc);                // :459-463
  }
};

// PROF: phase timing instead of iteration counts (tools only): fp_iters[c] =
// (table cycles, pixel+reduction cycles) per step, status[c] = loop cycles per step.
template <int IMG, int LPC, int WPE, bool PROF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
leapfrog_k1_tiledg(LeapArgsK1 a) {
  using TL = TiledG<IMG, LPC>;
  extern __shared__ double lds[];
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < TL::NPIX; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    lds[TL::tiled_index(r, cc)] = a.D[e];
  }
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / LPC;
  const int64_t chain = TL::CPW * wave + h;
  const bool real = chain < a.n_chains;            // ragged tail: mirror the wave's first chain
  const int64_t base = (real ? chain : TL::CPW * wave) * 3;
  double* tab = lds + TL::NPIX + (threadIdx.x / kWave) * TL::TAB;
  const double* sDm = lds + (lane % LPC);

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const double hdt = c.hdt;
  const LeanConsts lc = lean_consts(c);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  long long t_tab = 0, t_grad = 0, t_loop = 0, t1 = 0;

  for (int s = 0;; ++s) {
    double gf, gx, gy;
    if constexpr (PROF) t1 = clock64();
    TL::template gradient<PROF>(sDm, tab, f, x, y, c, lc, gf, gx, gy, &t_tab);
    if constexpr (PROF) {
      const long long t2 = clock64();
      t_grad += t2 - t1;
      t1 = t2;
    }
    if (s > 0) {
      pf = pf - hdt * gf;                          // :551
      px = px - hdt * gx;
      py = py - hdt * gy;
      if (f < c.f_lim) {                           // :554-564
        pf = -pf;
        st |= RHMC_STATUS_REFLECT_F;
      }
      if (x < 0.0 || x > (double)(IMG - 1)) {
        px = -px;
        st |= RHMC_STATUS_REFLECT_XY;
      }
      if (y < 0.0 || y > (double)(IMG - 1)) {
        py = -py;
        st |= RHMC_STATUS_REFLECT_XY;
      }
    }
    if (s == a.n_steps) break;
    pf = pf - hdt * gf;                            // :525
    px = px - hdt * gx;
    py = py - hdt * gy;
    {                                              // :528-535
      double last;
      it_p += p_loop_spec<2>(pf, dtaudq_coef_lean(f, lc), hdt, c.delta, c.counter_max, last);
      if (last > c.delta) st |= RHMC_STATUS_PLOOP_CAP;
    }
    {                                              // :538-545
      double last;
      it_q += q_loop_spec<4>(f, x, y, pf, px, py, hdt, lc, c.delta, c.counter_max, last);
      if (last > c.delta) st |= RHMC_STATUS_QLOOP_CAP;
    }
    pf = pf - hdt * ((pf * pf) * dtaudq_coef_lean(f, lc) / 2.0);   // :548
    if constexpr (PROF) t_loop += clock64() - t1;
  }
  if constexpr (PROF) {
    const int ns = a.n_steps > 0 ? a.n_steps : 1;
    it_p = (int)(t_tab / ns);
    it_q = (int)((t_grad - t_tab) / ns);
    st = (unsigned)(t_loop / ns);
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
