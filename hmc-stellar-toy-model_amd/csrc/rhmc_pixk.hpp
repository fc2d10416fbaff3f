// rhmc_pixk.hpp — multi-star leapfrog, PIXEL-MAJOR gradient for small images
// with a few stars (C3: 48x48, K = 10), where every star's window covers most
// of the image and the window-major kernel (rhmc_tiledrk.hpp) evaluates Lambda
// about 3.9 times per pixel.  Here Lambda is evaluated once per image pixel,
// as the reference does (sampler_RHMC.py:373-376, full image), and the three
// per-star sums of dphidq (:404-406) come out of separable accumulations with
// offsets taken from the image centre ctr = IMG/2 (w_i = i + 1/2 - ctr):
//   c0_k(j) = sum_i ex_k(i) s_ij,   c1_k(j) = sum_i ex_k(i) w_i s_ij
//   A0_k = sum_j fey_k(j) c0_k(j)   (= f_k sum PSF_k s)
//   A1_k = sum_j fey_k(j) c1_k(j),  A2_k = sum_j w_j fey_k(j) c0_k(j)
// and sum PSF_k s (i + 1/2 - x_k) f_k = A1_k + (ctr - x_k) A0_k, likewise y:
// so the row table holds ex only and the column factors carry f (fey), which
// serves Lambda and all three sums.  s = D/Lambda - 1.
// 32 lanes per chain (two chains per wave64): lane m = 16 rh + cg owns image
// columns cg, cg + 16, ... and rows rh, rh + 2, ..., rh + IMG - 2 (row pass r
// of the wave covers rows 2r and 2r + 1 of both chains).  Per
// gradient each chain builds two LDS tables, ex_k(i) [IMG][KMAX] and
// fey_k(j) [IMG][KMAX] (2 IMG KMAX / 32 exps per lane); a lane then runs its
// columns CT at a time: fey of its CT columns in registers, each row's ex
// read once (KMAX/2 ds_read_b128, broadcast to the 16 lanes of a row half)
// and used for CT pixels, whose data values sit side by side in the LDS image
// (layout [row][cg][NCP]: one ds_read_b64 per row for a column pair) and
// share one v_rcp_f64.  Row passes interleave the row halves (rows 2r, 2r + 1
// rather than r, r + IMG/2: +1.2 % at C3, profiles/r03_pk_skip/).  The step
// loop is km_steps (rhmc_tiledrk.hpp).
#pragma once
#include "rhmc_tiledrk.hpp"

namespace rhmc {

// Image columns per pass of the pixel-major gradient (1 to 3; capped at the
// lane's column count).
#ifndef RHMC_PK_CT
#define RHMC_PK_CT 3
#endif
// Factor tables by recurrence (PixK::tables_rec; 0: one exp per entry).
#ifndef RHMC_PK_REC
#define RHMC_PK_REC 1
#endif
// The 3 KMAX per-star sums by one 32-lane reduce-scatter (0: one all-reduce
// per sum).
#ifndef RHMC_PK_RS
#define RHMC_PK_RS 1
#endif

// v with the double's halves through update_dpp: lanes of the banks in
// BANKS take src moved by CTRL, the others keep old.
template <int CTRL, int BANKS>
__device__ __forceinline__ double dpp_merge(double old, double src) {
  const long long o = __double_as_longlong(old), v = __double_as_longlong(src);
  const int lo = __builtin_amdgcn_update_dpp((int)o, (int)v, CTRL, 0xF, BANKS, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(v >> 32), CTRL, 0xF, BANKS,
                                             false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Reduce-scatter over a chain's 32 lanes (one half of the wave): on entry
// every lane holds v[0..31], on return lane m (= lane % 32) holds the sum over
// the 32 lanes of v[m].  Butterfly: at each level a lane keeps the half of its
// values whose index bit equals its lane bit and adds the partner's copy of
// that half — rows by v_permlane16_swap (no select: the swap delivers each
// lane the partner's half it keeps), then xor 8 / 4 by row rotations and
// xor 2 / 1 by quad permutes.  31 exchanges and 31 adds for 32 sums instead of
// 5 of each per sum (half_sum_dpp).
__device__ __forceinline__ double reduce_scatter32(const double (&v)[32]) {
  // lane id by a volatile read: the lane-bit masks below are not hoisted out
  // of the step loop (live across the pixel passes they spill)
  int lid;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
  const int m = lid & 31;
  double w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const long long X = __double_as_longlong(v[i]), Y = __double_as_longlong(v[i + 16]);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)X, (unsigned)Y, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(X >> 32), (unsigned)(Y >> 32),
                                                     false, false);
    // row 0: own v[i] + row 1's v[i]; row 1: row 0's v[i + 16] + own v[i + 16]
    w[i] = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) +
           __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
  }
  const bool b3 = m & 8, b2 = m & 4, b1 = m & 2, b0 = m & 1;
  double u[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // xor 8: row_ror:8
    const double keep = b3 ? w[i + 8] : w[i], send = b3 ? w[i] : w[i + 8];
    u[i] = keep + dpp_move<0x128>(send);
  }
  double t[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // xor 4: banks 1, 3 from row_ror:4 (lane - 4), 0, 2 from :12
    const double keep = b2 ? u[i + 4] : u[i], send = b2 ? u[i] : u[i + 4];
    t[i] = keep + dpp_merge<0x124, 0xA>(dpp_move<0x12C>(send), send);
  }
  double z[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // xor 2: quad_perm [2,3,0,1]
    const double keep = b1 ? t[i + 2] : t[i], send = b1 ? t[i] : t[i + 2];
    z[i] = keep + dpp_move<0x4E>(send);
  }
  const double keep = b0 ? z[1] : z[0], send = b0 ? z[0] : z[1];
  return keep + dpp_move<0xB1>(send);  // xor 1: quad_perm [1,0,3,2]
}

template <int IMG, int KMAX, int CT_ = RHMC_PK_CT>
struct PixK {
  static constexpr int LPC = 32;           // lanes per chain
  static constexpr int CPW = kWave / LPC;  // chains per wave
  static constexpr int NC = IMG / 16;      // columns per lane
  static constexpr int NCP = (NC + 1) & ~1;  // LDS image: values per (row, column group)
  static constexpr int NR = IMG / 2;       // rows per lane
  static constexpr int CT = CT_ < NC ? CT_ : NC;
  static constexpr double kCtr = IMG / 2;
  static_assert(IMG == 32 || IMG == 48, "image side");
  static_assert(CT >= 1 && CT <= 3, "columns per pass");
  // per chain: row table ex [IMG][KMAX], then column table fey [IMG][KMAX]
  static constexpr size_t tab_doubles() { return (size_t)2 * IMG * KMAX; }
  // star table entries per chain: K <= KMAX stars, the last entry is never a
  // star (the MH kernel keeps E0 there); 16, not 32, so that two 4-wave
  // workgroups fit one CU's 160 KB at IMG = 48 (two waves per SIMD)
  static constexpr int NSTAR = 16;
  static_assert(KMAX < NSTAR, "star table");
  static constexpr size_t star_doubles(int waves) {
    return (size_t)waves * CPW * NSTAR * (sizeof(KRStar) / sizeof(double));
  }
  // LDS: exp table, star tables (NSTAR per chain), factor tables, image (fp32
  // [IMG][16][NCP]).
  static __host__ __device__ constexpr size_t lds_bytes(int waves) {
    return kExpTab * sizeof(double) + star_doubles(waves) * sizeof(double) +
           (size_t)waves * CPW * tab_doubles() * sizeof(double) +
           (size_t)IMG * 16 * NCP * sizeof(float);
  }
  // LDS image index of pixel (r, col)
  static __device__ __forceinline__ int img_index(int r, int col) {
    return (r * 16 + (col & 15)) * NCP + (col >> 4);
  }

  // Columns ci0 .. ci0 + N - 1 of the lane: accumulate their per-star sums
  // into A0, A1, A2.
  template <int N>
  static __device__ __forceinline__ void columns(int ci0, const float* __restrict__ simg,
                                                 const double* rtab, const double* ctab, int K,
                                                 const Consts& c, double (&A0)[KMAX],
                                                 double (&A1)[KMAX], double (&A2)[KMAX]) {
    const int m = lane_id() & (LPC - 1);
    const int cg = m & 15, rh = m >> 4;
    double fey[N][KMAX], c0[N][KMAX], c1[N][KMAX];
#pragma unroll
    for (int q = 0; q < N; ++q)
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        fey[q][k] = ctab[(cg + 16 * (ci0 + q)) * KMAX + k];
        c0[q][k] = c1[q][k] = 0.0;
      }
    const double* rt = rtab + (size_t)rh * KMAX;          // row 2 r + rh
    const float* dp = simg + (rh * 16 + cg) * NCP + ci0;
// rows per loop iteration
#ifndef RHMC_PK_ROW_UNROLL
#define RHMC_PK_ROW_UNROLL 4
#endif
#pragma unroll RHMC_PK_ROW_UNROLL
    for (int r = 0; r < NR; ++r) {
      double ex[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) ex[k] = rt[2 * r * KMAX + k];
      double l[N], sv[N];
#pragma unroll
      for (int q = 0; q < N; ++q) {
        l[q] = c.B;  // Lambda, stars in ascending order (:373-376)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) l[q] = fma(ex[k], fey[q][k], l[q]);
      }
      if constexpr (N == 3) {  // one reciprocal for the three pixels
        const float4 d = *reinterpret_cast<const float4*>(dp + 2 * r * 16 * NCP);
        const double l01 = l[0] * l[1];
        const double rr = rcp_nr1(l01 * l[2]);
        const double r01 = l[2] * rr;
        sv[0] = fma((double)d.x, l[1] * r01, -1.0);  // D/Lambda - 1 (:379)
        sv[1] = fma((double)d.y, l[0] * r01, -1.0);
        sv[2] = fma((double)d.z, l01 * rr, -1.0);
      } else if constexpr (N == 2) {  // one reciprocal for the pixel pair
        const float2 d = *reinterpret_cast<const float2*>(dp + 2 * r * 16 * NCP);
        const double rr = rcp_nr1(l[0] * l[1]);
        sv[0] = fma((double)d.x, l[1] * rr, -1.0);  // D/Lambda - 1 (:379)
        sv[1] = fma((double)d.y, l[0] * rr, -1.0);
      } else {
        sv[0] = fma((double)dp[2 * r * 16 * NCP], rcp_nr1(l[0]), -1.0);
      }
      const double w = ((double)(2 * r + rh) + 0.5) - kCtr;
#pragma unroll
      for (int q = 0; q < N; ++q) {
        const double t = w * sv[q];
#pragma unroll
        for (int k = 0; k < KMAX; ++k) {
          c0[q][k] = fma(ex[k], sv[q], c0[q][k]);
          c1[q][k] = fma(ex[k], t, c1[q][k]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const double wj = ((double)(cg + 16 * (ci0 + q)) + 0.5) - kCtr;
      // all KMAX slots: a phantom star's (k >= K) table entries are zero, so its
      // sums stay zero (a guard on the runtime K compiled to 180 selects per
      // gradient)
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        A0[k] = fma(fey[q][k], c0[q][k], A0[k]);
        A1[k] = fma(fey[q][k], c1[q][k], A1[k]);
        A2[k] = fma(wj * fey[q][k], c0[q][k], A2[k]);
      }
    }
  }

  // The factor tables by recurrence (utils.py:475-486 evaluated as in
  // rhmc_tiledr.hpp factors_rec): lane m < S KMAX owns star k = m / S and the
  // image rows (for ex) / columns (for fey) of segment m % S, SR = ceil(IMG / S)
  // of them, in runs of up to 8 that start from two exps each,
  //   e(v) = exp(-c v^2), g(v) = exp(-c (2 v + 1)), e(v + 1) = e(v) g(v),
  //   g(v + 1) = g(v) e^{-2c}   (v = i + 1/2 - x_k),
  // i.e. 8 exps per lane for both tables instead of 30 (C3).  Each entry is at
  // most 7 products from an exp (within ~25 ulp of the direct exp).  Returns
  // false (nothing written) when a run of some lane of the wave starts outside
  // the recurrence's range (|v| >= rec_vmax, NaN): the caller then evaluates
  // every entry directly.  Phantom stars (k >= K) get zeros.
  static __device__ __forceinline__ bool tables_rec(const double* __restrict__ etab,
                                                    const KRStar* tab, double* rtab,
                                                    double* ctab, int K, const LeanConsts& lc) {
    constexpr int S = LPC / KMAX;            // segments per star
    constexpr int SR = (IMG + S - 1) / S;    // rows / columns per segment
    constexpr int RUN = 8;                   // entries per exp pair
    static_assert(S >= 1, "stars per chain");
    // lane id by a volatile read: the loop-invariant segment bookkeeping below
    // is recomputed per gradient instead of being hoisted out of the step loop
    // (its registers would stay live across the pixel passes and spill)
    int lid;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
    const int m = lid & (LPC - 1);
    const bool act = m < S * KMAX;
    const int k = act ? m / S : 0, seg = act ? m - (m / S) * S : 0;
    const bool real = act && k < K;
    const double c = lc.inv_two_sig2;
    const KRStar st = tab[real ? k : 0];
    const double xs = real ? st.x : 0.0, ys = real ? st.y : 0.0;
    bool ok = true;
#pragma unroll
    for (int r0 = 0; r0 < SR; r0 += RUN) {
      const double o = (double)(seg * SR + r0) + 0.5;
      ok = ok && fabs(o - xs) < lc.rec_vmax && fabs(o - ys) < lc.rec_vmax;
    }
    if (__builtin_amdgcn_ballot_w64(!ok) != 0) return false;
    if (!act) return true;
    const double fn = real ? st.pad * lc.inv_norm : 0.0;  // pad = flux_fold(f) (kr_publish)
#pragma unroll 1
    for (int t = 0; t < 2; ++t) {  // t = 0: row table ex, t = 1: column table fey
      const double ctr = t ? ys : xs;
      double* dst = (t ? ctab : rtab) + k;
#pragma unroll 1
      for (int r0 = 0; r0 < SR; r0 += RUN) {
        const int ib = seg * SR + r0;
        const double v0 = ((double)ib + 0.5) - ctr;
        double e = exp_neg(-(v0 * v0) * c, etab);
        double g = exp_neg(-fma(2.0, v0, 1.0) * c, etab);
        if (t) e = e * fn;  // f (e N): one rounding more than f * (e * N)
        if (!real) e = 0.0;
#pragma unroll
        for (int l = 0; l < RUN && r0 + l < SR; ++l) {
          if (ib + l < IMG) dst[(ib + l) * KMAX] = e;
          e = e * g;
          g = g * lc.k_row;
        }
      }
    }
    return true;
  }

  // The chain's factor tables ex [IMG][KMAX] (rtab) and fey (ctab) for the
  // stars in `tab`: by recurrence, or every entry directly when a run of the
  // wave is out of the recurrence's range.
  static __device__ __forceinline__ void tables(const double* __restrict__ etab,
                                                const KRStar* tab, double* rtab, double* ctab,
                                                int K, const LeanConsts& lc) {
    const int m = lane_id() & (LPC - 1);
#if RHMC_PK_REC
    if (!tables_rec(etab, tab, rtab, ctab, K, lc))
#endif
    for (int e = m; e < IMG * KMAX; e += LPC) {
      const int i = e / KMAX, k = e - (e / KMAX) * KMAX;
      double ex = 0.0, fey = 0.0;
      if (k < K) {
        const double v = ((double)i + 0.5) - tab[k].x;
        ex = exp_neg(-(v * v) * lc.inv_two_sig2, etab);
        const double u = ((double)i + 0.5) - tab[k].y;
        fey = tab[k].pad * (exp_neg(-(u * u) * lc.inv_two_sig2, etab) * lc.inv_norm);
      }
      rtab[e] = ex;
      ctab[e] = fey;
    }
  }

  // Pixel part of dphidq (:365-425 without metric / prior): lane m < K gets
  // star m's; the star table `tab` holds the chain's (f, x, y).
  static __device__ __forceinline__ void gradient(const double* __restrict__ etab,
                                                  const float* __restrict__ simg,
                                                  const KRStar* tab, double* rtab, int K,
                                                  const Consts& c, const LeanConsts& lc,
                                                  double& gf, double& gx, double& gy) {
    const int m = lane_id() & (LPC - 1);
    double* ctab = rtab + (size_t)IMG * KMAX;
    wave_lds_sync();  // the previous gradient's table reads are done
    tables(etab, tab, rtab, ctab, K, lc);
    wave_lds_sync();
    double A0[KMAX], A1[KMAX], A2[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) A0[k] = A1[k] = A2[k] = 0.0;
#pragma unroll
    for (int ci = 0; ci + CT <= NC; ci += CT)
      columns<CT>(ci, simg, rtab, ctab, K, c, A0, A1, A2);
    if constexpr (NC % CT == 1) columns<1>(NC - 1, simg, rtab, ctab, K, c, A0, A1, A2);
    static_assert(NC % CT <= 1, "column passes");
#if RHMC_PK_RS
    // star k's sums land in lanes k, KMAX + k, 2 KMAX + k (phantom stars' A
    // are zero)
    static_assert(3 * KMAX <= 32, "one reduce-scatter slot per sum");
    double v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i)
      v[i] = i < KMAX ? A0[i] : i < 2 * KMAX ? A1[i - KMAX] : i < 3 * KMAX ? A2[i - 2 * KMAX] : 0.0;
    const double s0 = reduce_scatter32(v);
    const int hb = (lane_id() & 32) + m;  // this lane, in the chain's half of the wave
    const double s1 = __shfl(s0, hb + KMAX, kWave);  // lanes m >= K read past: unused
    const double s2 = __shfl(s0, hb + 2 * KMAX, kWave);
    gf = gx = gy = 0.0;
    if (m < K) {
      const KRStar st = tab[m];
      gf = -s0 / st.pad;                                    // :404 (pad = flux_fold(f))
      gx = -fma(kCtr - st.x, s0, s1) * lc.inv_var;          // :405
      gy = -fma(kCtr - st.y, s0, s2) * lc.inv_var;          // :406
    }
#else  // (K wave-uniform here: not for ragged sets, whose two chains may differ)
    gf = gx = gy = 0.0;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {  // wave-uniform
        const double s0 = half_sum_dpp(A0[k]);
        const double s1 = half_sum_dpp(A1[k]);
        const double s2 = half_sum_dpp(A2[k]);
        if (m == k) {
          const KRStar st = tab[k];
          gf = -s0 / st.pad;                                // :404 (pad = flux_fold(f))
          gx = -fma(kCtr - st.x, s0, s1) * lc.inv_var;      // :405
          gy = -fma(kCtr - st.y, s0, s2) * lc.inv_var;      // :406
        }
      }
    }
#endif
  }
};

// Two chains per wave, W waves per workgroup, one star per lane (K <= KMAX).
// SOLVER as in leapfrog_kr: RHMC_single_step, an explicit integrator (f_pos =
// the flux wall) or kSolverHmcRandom.  Ragged sets (a.Kc): each chain's own
// row and star count; the two chains of a wave may differ in K — everything
// that depends on it is per lane (a chain's lanes), and the pixel passes run
// all KMAX slots with zero tables for the stars a chain lacks — so a chain's
// results are those of a fixed-K launch on it.  RAGGED is a separate
// instantiation, so the fixed-K kernel keeps its wave-uniform K.
template <int IMG, int KMAX, int SOLVER = RHMC_SOLVER_IMPLICIT, bool RAGGED = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
leapfrog_pk(LeapArgsKR a, int f_pos) {
  // (HMC_random ran two columns per pass until the unguarded accumulation
  // freed the registers three need)
  // The all-reduce gradient (RHMC_PK_RS = 0) assumes one K per wave.
  static_assert(!RAGGED || RHMC_PK_RS, "ragged pixel-major launches need the reduce-scatter");
  using PK = PixK<IMG, KMAX, RHMC_PK_CT>;
  extern __shared__ double lds[];
  const int W = blockDim.x / kWave;
  exp_tab_fill(lds);
  float* simg = reinterpret_cast<float*>(lds + kExpTab + PK::star_doubles(W) +
                                         (size_t)W * PK::CPW * PK::tab_doubles());
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x)
    simg[PK::img_index(e / IMG, e % IMG)] = a.Df[e];
  __syncthreads();
  const int64_t wave =
      (int64_t)blockIdx.x * W + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  if (PK::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / PK::LPC, m = lane % PK::LPC;
  const int64_t chain = PK::CPW * wave + h;
  const bool real = chain < a.n_chains;  // ragged tail: mirror the wave's first chain
  const int64_t chain_r = real ? chain : PK::CPW * wave;
  int64_t row = chain_r, ldq = 3 * (int64_t)a.K;
  int K = a.K;
  if constexpr (RAGGED) {  // a ragged set: this chain's row and star count
    row = a.rows ? a.rows[chain_r] : chain_r;
    K = a.Kc[row];
    ldq = a.ld;
  }
  const int64_t cbase = row * ldq;
  const int slot = (threadIdx.x / kWave) * PK::CPW + h;
  KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + slot * PK::NSTAR;
  double* rtab = lds + kExpTab + PK::star_doubles(W) + (size_t)slot * PK::tab_doubles();
  const Consts& c = a.c;
  const LeanConsts lc = lean_consts(c);
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
    km_steps<1, decltype(grad), true>(f, x, y, pf, px, py, own, tab, a.n_steps,
                                      (double)(IMG - 1), c, lc, grad, it_p, it_q, st);
  } else if constexpr (SOLVER == kSolverHmcRandom) {
    if (km_hmc_random_steps<1, decltype(grad), true>(f, x, y, pf, px, py, own, tab,
                                                     a.steps[chain_r], a.dtv, c, grad)) {
      st |= RHMC_STATUS_REFLECT_F;  // p_tmp stays the starting momentum (:547-550)
      pf[0] = own[0] ? a.p[e] : 0.0;
      px[0] = own[0] ? a.p[e + 1] : 0.0;
      py[0] = own[0] ? a.p[e + 2] : 0.0;
    }
  } else {
    km_explicit_steps<SOLVER, 1, decltype(grad), true>(f, x, y, pf, px, py, own, tab,
                                                       a.n_steps, f_pos, c, lc, grad, st);
  }
  // the output index again, from a volatile lane id: the one computed above,
  // held across the step loop, spills
  int lid;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
  const int64_t chain_o = PK::CPW * wave + lid / PK::LPC;
  const int64_t chain_or = chain_o < a.n_chains ? chain_o : PK::CPW * wave;
  const int64_t e_o = (RAGGED ? (a.rows ? a.rows[chain_or] : chain_or) * a.ld
                             : chain_or * 3 * (int64_t)a.K) +
                      3 * (int64_t)(own[0] ? lid % PK::LPC : 0);
  unsigned nf = 0u;
  if (own[0] && real) {
    if (!(isfinite(f[0]) && isfinite(x[0]) && isfinite(y[0]) && isfinite(pf[0]) &&
          isfinite(px[0]) && isfinite(py[0])))
      nf = RHMC_STATUS_NONFINITE;
    a.q[e_o] = f[0];
    a.q[e_o + 1] = x[0];
    a.q[e_o + 2] = y[0];
    a.p[e_o] = pf[0];
    a.p[e_o + 1] = px[0];
    a.p[e_o + 2] = py[0];
  }
  unsigned all = st | nf;
#pragma unroll
  for (int d = 16; d >= 1; d >>= 1) all |= (unsigned)__shfl_xor((int)all, d, kWave);
  if (lid % PK::LPC == 0 && chain_o < a.n_chains) {
    if (a.status) a.status[chain_o] = (int32_t)all;
    if (a.fp_iters) {
      a.fp_iters[2 * chain_o] = it_p;
      a.fp_iters[2 * chain_o + 1] = it_q;
    }
  }
}

}  // namespace rhmc
