// rhmc_tiled2.hpp — single-star leapfrog with TWO chains per wave64.
//
// Each half-wave (32 lanes) owns one chain.  In the one-chain-per-wave kernel
// (rhmc_tiled.hpp) about half of a step's VALU work is per-chain overhead that
// does not shrink with more lanes: the PSF factor exps (96 per chain at 48x48,
// 25 % of the lanes idle), three all-reduces and the serial fixed-point loops.
// Two chains per wave run that overhead once for both chains (the loops mask
// off a converged half), while the pixel work per chain is unchanged.
//   * lane (h, m): h = lane >> 5 selects the chain, m = lane & 31 is a 4 x 8
//     grid over the image: TR = IMG/4 rows x TC = IMG/8 columns per lane;
//   * D in LDS as [TR*TC][32] — lanes m and m+32 read the same address;
//   * all-reduce inside each half: DPP row reductions + v_permlane16_swap.
#pragma once
#include "rhmc_tiled.hpp"
#include "rhmc_wave.hpp"

namespace rhmc {

// Sum over the 32 lanes of each half-wave; every lane of a half gets its
// half's sum (rows 0+1 and rows 2+3), bit-identical within the half.
__device__ __forceinline__ double half_sum_dpp(double v) {
  v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_move<0x141>(v);  // row_half_mirror
  v += dpp_move<0x140>(v);  // row_mirror
  return swap_add<false>(v);
}

template <int IMG>
struct Tiled2 {
  static constexpr int TR = IMG / 4;   // rows per lane
  static constexpr int TC = IMG / 8;   // columns per lane
  static constexpr int NPIX = IMG * IMG;
  static constexpr int TAB = 2 * 4 * IMG;  // per wave: 2 chains x (ex,dx rows + ey,dy cols)
  static_assert(IMG % 8 == 0 && IMG <= 64, "IMG multiple of 8, <= 64");
  static_assert((TR * TC) % 2 == 0, "pixel pairs");

  static __host__ __device__ constexpr size_t lds_doubles(int waves) {
    return (size_t)NPIX + (size_t)waves * TAB;
  }
  // LDS index of pixel (r, c): lane m = (r / TR) * 8 + c / TC of either half.
  static __device__ __forceinline__ int tiled_index(int r, int c) {
    const int m = (r / TR) * 8 + (c / TC);
    return ((r % TR) * TC + (c % TC)) * 32 + m;
  }

  // dphidq of the half-wave's chain (every lane of the half gets it).
  static __device__ __forceinline__ void gradient(const double* __restrict__ sDm, double* tab,
                                                  double f, double x, double y, const Consts& c,
                                                  const LeanConsts& lc, double& gf, double& gx,
                                                  double& gy) {
    const int lane = lane_id();
    const int h = lane >> 5, m = lane & 31;
    const int ta = m >> 3, tb = m & 7;
    double* t = tab + h * 4 * IMG;  // this chain: rows [IMG][2], cols [IMG][2]
    // 2*IMG factor entries per chain over 32 lanes
#pragma unroll
    for (int e0 = 0; e0 < 2 * IMG; e0 += 32) {
      const int e = e0 + m;
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

    // s_ij = D_ij / Lambda_ij - 1 and, by separability (PSF_ij = ex_i ey_j),
    //   sum_ij PSF s      = sum_i ex_i R_i,        R_i = sum_j ey_j s_ij
    //   sum_ij PSF s dx_i = sum_i ex_i dx_i R_i
    //   sum_ij PSF s dy_j = sum_j ey_j dy_j C_j,   C_j = sum_i ex_i s_ij
    // so the pixel loop never forms PSF_ij: Lambda = fma(f ex_i, ey_j, B), one
    // reciprocal per pixel pair (+1 Newton step), s, and two fmas.
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
      const double d1 = sDm[pp * 32], d2 = sDm[(pp + 1) * 32];
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
      const double t = ex[k] * R[k];
      a0 += t;
      a1 = fma(t, dx[k], a1);
    }
#pragma unroll
    for (int k = 0; k < TC; ++k) a2 = fma(ey[k] * C[k], dy[k], a2);
    const double s0 = half_sum_dpp(a0);
    const double s1 = half_sum_dpp(a1);
    const double s2 = half_sum_dpp(a2);
    gf = -s0;                                          // :404
    gx = -s1 * f * lc.inv_var;                         // :405
    gy = -s2 * f * lc.inv_var;                         // :406
    if (c.use_prior) gf += c.alpha * rcp_nr(f);        // :408-409
    gf += metric_flux_term_lean(f, lc);                // :459-463
  }
};

template <int IMG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
leapfrog_k1_tiled2(LeapArgsK1 a) {
  using TL = Tiled2<IMG>;
  extern __shared__ double lds[];
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < TL::NPIX; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    lds[TL::tiled_index(r, cc)] = a.D[e];
  }
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (2 * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane >> 5;
  const int64_t chain = 2 * wave + h;
  const bool real = chain < a.n_chains;            // odd count: the last half mirrors
  const int64_t base = (real ? chain : 2 * wave) * 3;
  double* tab = lds + TL::NPIX + (threadIdx.x / kWave) * TL::TAB;
  const double* sDm = lds + (lane & 31);

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const double hdt = c.hdt;
  const LeanConsts lc = lean_consts(c);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;

  for (int s = 0;; ++s) {
    double gf, gx, gy;
    TL::gradient(sDm, tab, f, x, y, c, lc, gf, gx, gy);
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
      const double coef = dtaudq_coef_lean(f, lc);
      const double rho = pf;
      double dp;
      int n = 0;
      do {
        const double pp = rho - hdt * ((pf * pf) * coef / 2.0);
        dp = fabs(pf - pp);
        pf = pp;
        ++n;
      } while (dp > c.delta && n < c.counter_max);
      it_p += n;
      if (dp > c.delta) st |= RHMC_STATUS_PLOOP_CAP;
    }
    {                                              // :538-545
      const double sf = f, sx = x, sy = y;
      double ihff, ihxx;
      inv_metric(sf, lc, ihff, ihxx);
      const double af = pf * ihff, ax = px * ihxx, ay = py * ihxx;
      double dq;
      int n = 0;
      do {
        inv_metric(f, lc, ihff, ihxx);
        const double nf = sf + hdt * (af + pf * ihff);
        const double nx = sx + hdt * (ax + px * ihxx);
        const double ny = sy + hdt * (ay + py * ihxx);
        const double a0 = fabs(f - nf), a1 = fabs(x - nx), a2 = fabs(y - ny);
        const double sum = a0 + a1 + a2;
        dq = (sum != sum) ? sum : fmax(fmax(a0, a1), a2);
        f = nf;
        x = nx;
        y = ny;
        ++n;
      } while (dq > c.delta && n < c.counter_max);
      it_q += n;
      if (dq > c.delta) st |= RHMC_STATUS_QLOOP_CAP;
    }
    pf = pf - hdt * ((pf * pf) * dtaudq_coef_lean(f, lc) / 2.0);   // :548
  }

  if ((lane & 31) == 0 && real) {
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
