// rhmc_tiled.hpp — the specialised single-star leapfrog kernel (the headline
// C1/C2/C4 configurations: K = 1 on an IMG x IMG image, IMG in {16,32,48,64}).
//
// Differences from the generic kernel (rhmc_kernels.hip):
//   * 8 x 8 lane tiling: lane (a, b) owns the T x T pixel block at rows
//     a*T.., cols b*T.. (T = IMG/8), so each lane needs only T row factors
//     ex/dx and T column factors ey/dy of the separable PSF — held in
//     registers for the whole pixel loop (no per-pixel table reads);
//   * D is staged into LDS "lane-tiled" ([T*T][64]): the wave reads one
//     pixel per lane with one conflict-free ds_read_b64;
//   * fully unrolled, branch-free pixel loop (IMG is a template constant);
//   * D/Lambda by v_rcp_f64 + one Newton step + a residual correction
//     (fast_div), wave sums by DPP row reductions + 4 readlanes;
//   * per-row / per-column partial sums exploit separability:
//       sum w*dx = sum_i dx_i (sum_j w_ij),  sum w*dy = sum_j dy_j (sum_i w_ij);
//   * one gradient call site per step (the end-of-step gradient is the next
//     step's first one), so the kernel body is a single loop.
// The chain state is wave-uniform (every lane mirrors star 0), so the
// fixed-point loops need no cross-lane reduction at all.
#pragma once
#include "rhmc_wave.hpp"

namespace rhmc {

// v_rcp_f64 (~2^-23 relative) + 1 Newton step (~2^-46) + residual correction:
// the quotient is the correctly rounded one for all but a vanishing fraction
// of operands (tools/microbench.hip measures the mismatch rate on the
// Lambda/D operand range); Lambda >= B > 0 is never denormal or huge.
__device__ __forceinline__ double fast_div(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  const double q = n * r;
  const double res = fma(-d, q, n);
  return fma(r, res, q);
}

template <int CTRL>
__device__ __forceinline__ double dpp_move(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// gfx950 v_permlane{16,32}_swap on both 32-bit halves of a double, called
// with the same register as both operands: returns (a, b) such that a + b
// adds row r to row r^1 (16) or half h to half h^1 (32), with the SAME
// operand order in both partner rows.
template <bool SWAP32>
__device__ __forceinline__ double swap_add(double v) {
  const long long bits = __double_as_longlong(v);
  const unsigned lo = (unsigned)bits, hi = (unsigned)(bits >> 32);
  unsigned a_lo, b_lo, a_hi, b_hi;
  if (SWAP32) {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a_lo = l[0]; b_lo = l[1]; a_hi = h[0]; b_hi = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    a_lo = l[0]; b_lo = l[1]; a_hi = h[0]; b_hi = h[1];
  }
  const double a = __longlong_as_double(((long long)a_hi << 32) | a_lo);
  const double b = __longlong_as_double(((long long)b_hi << 32) | b_lo);
  return a + b;
}

// All-reduce over the wave: xor-1 / xor-2 quad permutes, half-mirror and
// mirror inside each 16-lane row (partners add the same two values, so every
// lane of a row holds the same bits), then row pairs and half pairs by the
// permlane swaps.  Deterministic and bit-identical in every lane.
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_move<0x141>(v);  // row_half_mirror
  v += dpp_move<0x140>(v);  // row_mirror
  v = swap_add<false>(v);   // rows 0+1, 2+3
  return swap_add<true>(v); // (0+1) + (2+3)
}

template <int IMG>
struct Tiled {
  static constexpr int T = IMG / 8;       // pixels per lane per side
  static constexpr int NPIX = IMG * IMG;
  static constexpr int TAB = 4 * IMG;     // doubles of per-wave tables
  static_assert(IMG % 8 == 0 && IMG <= 64, "tiled kernel: IMG in {8..64}, multiple of 8");

  static __host__ __device__ constexpr size_t lds_doubles(int waves) {
    return (size_t)NPIX + (size_t)waves * TAB;
  }

  // LDS index of image pixel (r, c) in the lane-tiled layout [T*T][64].
  static __device__ __forceinline__ int tiled_index(int r, int c) {
    const int l = (r / T) * 8 + (c / T);
    return ((r % T) * T + (c % T)) * 64 + l;
  }

  // dphidq at (f, x, y) for the wave's chain (every lane gets the result).
  static __device__ __forceinline__ void gradient(const double* __restrict__ sDl, double* tab,
                                                  double f, double x, double y, const Consts& c,
                                                  const LeanConsts& lc, double& gf, double& gx,
                                                  double& gy) {
    const int lane = lane_id();
    const int ta = lane >> 3, tb = lane & 7;
    // separable PSF factors: lane l < IMG builds row l and column l
    if (lane < IMG) {
      const double v = (lane + 0.5) - x;
      const double u = (lane + 0.5) - y;
      tab[2 * lane] = exp(-(v * v) * lc.inv_two_sig2);
      tab[2 * lane + 1] = ((double)lane - x) + 0.5;
      tab[2 * IMG + 2 * lane] = exp(-(u * u) * lc.inv_two_sig2) * lc.inv_norm;
      tab[2 * IMG + 2 * lane + 1] = ((double)lane - y) + 0.5;
    }
    wave_lds_sync();
    double ex[T], dx[T], ey[T], dy[T];
#pragma unroll
    for (int k = 0; k < T; ++k) {
      ex[k] = tab[2 * (ta * T + k)];
      dx[k] = tab[2 * (ta * T + k) + 1];
      ey[k] = tab[2 * IMG + 2 * (tb * T + k)];
      dy[k] = tab[2 * IMG + 2 * (tb * T + k) + 1];
    }
    wave_lds_sync();

    double srow[T], scol[T];
#pragma unroll
    for (int k = 0; k < T; ++k) srow[k] = scol[k] = 0.0;
    // Pixels are taken in pairs sharing one v_rcp_f64: 1/(L1 L2) refined by
    // one Newton step gives 1/L1 = L2/(L1 L2) and 1/L2 = L1/(L1 L2) to ~2^-46,
    // and the residual correction of fast_div brings each D/L to the
    // correctly rounded quotient (tools/microbench.hip).
    static_assert((T * T) % 2 == 0, "pixel pairs");
#pragma unroll
    for (int pp = 0; pp < T * T; pp += 2) {
      const int i1 = pp / T, j1 = pp % T, i2 = (pp + 1) / T, j2 = (pp + 1) % T;
      const double d1 = sDl[pp * 64], d2 = sDl[(pp + 1) * 64];
      const double psf1 = ex[i1] * ey[j1], psf2 = ex[i2] * ey[j2];
      const double l1 = fma(f, psf1, c.B), l2 = fma(f, psf2, c.B);  // B + f PSF (:373-376)
      const double L = l1 * l2;
      double r = __builtin_amdgcn_rcp(L);
      r = fma(r, fma(-L, r, 1.0), r);
      const double r1 = l2 * r, r2 = l1 * r;
      double q1 = d1 * r1, q2 = d2 * r2;                            // D/Lambda (:379)
      q1 = fma(r1, fma(-l1, q1, d1), q1);
      q2 = fma(r2, fma(-l2, q2, d2), q2);
      const double w1 = fma(psf1, q1, -psf1), w2 = fma(psf2, q2, -psf2);  // rho * PSF
      srow[i1] += w1;
      scol[j1] += w1;
      srow[i2] += w2;
      scol[j2] += w2;
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
    for (int k = 0; k < T; ++k) {
      a0 += srow[k];
      a1 = fma(srow[k], dx[k], a1);
      a2 = fma(scol[k], dy[k], a2);
    }
    const double s0 = wave_sum_dpp(a0);
    const double s1 = wave_sum_dpp(a1);
    const double s2 = wave_sum_dpp(a2);
    gf = -s0;                                          // :404
    gx = -s1 * f * lc.inv_var;                         // :405
    gy = -s2 * f * lc.inv_var;                         // :406
    if (c.use_prior) gf += c.alpha * rcp_nr(f);        // :408-409
    gf += metric_flux_term_lean(f, lc);                // dphidq (:459-463)
  }
};

struct LeapArgsK1 {
  double* q;
  double* p;
  int32_t* fp_iters;
  int32_t* status;
  const double* D;
  const float* Df;   // D in fp32 when exact (ctx->img_f32), else nullptr
  int64_t n_chains;
  int n_steps, rows, cols, pad;
  Consts c;
};

// 4 waves per SIMD (<= 128 VGPRs) lets a 4096-chain launch be resident in
// one round on 256 CUs; IMG = 64 needs more registers than that.
template <int IMG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(IMG <= 48 ? 4 : 2)))
leapfrog_k1_tiled(LeapArgsK1 a) {
  using TL = Tiled<IMG>;
  extern __shared__ double lds[];
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < TL::NPIX; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    lds[TL::tiled_index(r, cc)] = a.D[e];
  }
  __syncthreads();
  const int64_t chain = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (chain >= a.n_chains) return;
  const int lane = lane_id();
  double* tab = lds + TL::NPIX + (threadIdx.x / kWave) * TL::TAB;
  const double* sDl = lds + lane;

  // every lane mirrors the single star
  const int64_t base = chain * 3;
  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const double hdt = c.hdt;
  const LeanConsts lc = lean_consts(c);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;

  for (int s = 0;; ++s) {
    double gf, gx, gy;
    TL::gradient(sDl, tab, f, x, y, c, lc, gf, gx, gy);
    if (s > 0) {
      // (5) closing half kick of step s-1 (:551) and (6) reflection (:554-564)
      pf = pf - hdt * gf;
      px = px - hdt * gx;
      py = py - hdt * gy;
      if (f < c.f_lim) {
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

    // (1) opening half kick (:525)
    pf = pf - hdt * gf;
    px = px - hdt * gx;
    py = py - hdt * gy;

    // (2) p fixed point on the flux slot (:528-535)
    {
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
    // (3) q fixed point (:538-545)
    {
      const double sf = f, sx = x, sy = y;
      double ihff, ihxx;
      inv_metric(sf, lc, ihff, ihxx);
      const double af = pf * ihff, ax = px * ihxx, ay = py * ihxx;  // dtaudp(sig, p)
      double dq;
      int n = 0;
      do {
        inv_metric(f, lc, ihff, ihxx);
        const double nf = sf + hdt * (af + pf * ihff);
        const double nx = sx + hdt * (ax + px * ihxx);
        const double ny = sy + hdt * (ay + py * ihxx);
        // max|q - q'| with np.max's NaN propagation: the sum of the three
        // non-negative terms is NaN exactly when one of them is
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
    // (4) p -= dt/2 dtaudq(q, p) (:548)
    pf = pf - hdt * ((pf * pf) * dtaudq_coef_lean(f, lc) / 2.0);
  }

  if (lane == 0) {
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
