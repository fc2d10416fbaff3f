// rhmc_tiledr.hpp — single-star leapfrog on a WIN x WIN pixel window per
// chain (WIN = 28 or 32) with the window's data pixels held in REGISTERS
// across steps: 16 lanes per chain, 4 chains per wave64.
//
// Window.  Rows o_x .. o_x + WIN - 1 with o_x = floor(x + 0.5) - WIN/2 (then
// clamped into the image), likewise columns: every pixel centre left out is
// >= WIN/2 px from the star, where PSF/peak = exp(-(WIN/2)^2 / (2 sigma^2)).
// launch_leapfrog uses a window only when that is <= 2^-62 (WIN = 28:
// sigma <= 1.510 px; WIN = 32: sigma <= 1.726 px; the reference PSF has
// sigma = 3.5/2.354 = 1.487 px, 2^-64 at WIN = 28).  A dropped pixel then
// changes neither its Lambda (f PSF < half an ulp of B for f < 4e5 counts)
// nor the gradient sums beyond their own rounding (every dropped term is
// < 2^-62 of the peak pixel's term; together they stay below one ulp of it).
//
// Operands live in registers, not LDS:
//  * D: the window moves only when round(x) or round(y) changes, so each lane
//    keeps its TR x TC window pixels in VGPRs and re-reads them from the LDS
//    copy of the image only on such a step (a wave-uniform branch: a divergent
//    one would keep the old values live through the loads and double the
//    register footprint).  The cache is fp32 when every image pixel is exactly
//    representable (Poisson counts < 2^24, checked when the image is set: one
//    exact v_cvt_f64_f32 per use), else fp64.
//  * PSF factors: lane (a, b) (a = m / 4, b = m % 4) owns window rows
//    a TR .. a TR + TR - 1 and window columns b, b + 4, ..., b + 4 (TC - 1).
//    Quad-mates (same a) share rows: lane b evaluates rows a TR + b + {0, 4}
//    and DPP quad broadcasts hand them round.  Lanes with the same b share
//    columns: lane a evaluates columns b + 4 (a + {0, 4}) and ds_swizzle in
//    bit mode (and 0x13, or a' << 2: "lane (a', b) of my 16-lane group")
//    hands them round.  Four exps per lane, static slot maps, no LDS tables.
//  * Position moments with offsets linear in the index:
//    sum_i w_i ((o + a TR + i) - x + 0.5) = dxa sum_i w_i + sum_i i w_i.
//
// Reference: dphidq / dVdq sampler_RHMC.py:365-425, :448-465; the step loop is
// rhmc_k1step.hpp (:522-566).
#pragma once
#include "rhmc_exp.hpp"
#include "rhmc_k1step.hpp"
#include "rhmc_wave.hpp"
#include "rhmc_windowed.hpp"

namespace rhmc {

// exp(-(WIN/2)^2 / (2 sigma^2)) <= 2^-62 (62 ln 2 = 42.975)?
__host__ __device__ inline bool reg_window_ok(int win, double inv_two_sig2) {
  const double h = 0.5 * win;
  return h * h * inv_two_sig2 >= 42.98;
}

template <int PAT>
__device__ __forceinline__ double swizzle_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_swizzle((int)b, PAT);
  const int hi = __builtin_amdgcn_ds_swizzle((int)(b >> 32), PAT);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Pixels sharing one v_rcp_f64 in the pixel loop (2 or 4).
#ifndef RHMC_RCP_GROUP
#define RHMC_RCP_GROUP 4
#endif
constexpr int kRcpGroup = RHMC_RCP_GROUP;

// PSF factors by recurrence (factors_rec; 0: four exps per lane, factors).
#ifndef RHMC_FACT_REC
#define RHMC_FACT_REC 1
#endif

// Fold each row sum R_i into the moments as soon as its row is complete
// (same summation order; frees the row-sum registers during the pixel loop).
#ifndef RHMC_RFOLD
#define RHMC_RFOLD 1
#endif

// DT: the type the window pixels are cached in (float when the image is
// exactly representable in fp32, else double).
//
// ROW0 / TR select a row slice of the window for this wave: lane row a owns
// window rows ROW0 + a TR .. + TR - 1 (the whole window: ROW0 = 0, TR = WIN/4).
// A two-wave split (rows 0-11 with the serial step on one wave, rows 12-27 on
// a helper wave, two workgroup barriers per step) was measured at 0.8x of the
// single-wave kernel at 4096 chains and dropped.
template <int IMG, int WIN, typename DT, int ROW0 = 0, int TR_ = WIN / 4>
struct TiledR {
  static constexpr int LPC = 16;           // lanes per chain
  static constexpr int CPW = kWave / LPC;  // chains per wave
  static constexpr int P = IMG + 1;        // LDS row pitch
  static constexpr int TR = TR_;           // window rows per lane
  static constexpr int TC = WIN / 4;       // window columns per lane
  static constexpr int NPX = TR * TC;
  static constexpr int NTR = (TR + 3) / 4; // row factors evaluated per lane
  static_assert(WIN == 28 || WIN == 32, "window side");
  static_assert(IMG >= WIN, "window inside the image");
  static_assert(ROW0 + 4 * TR <= WIN && TR <= 8, "row slice inside the window");

  // LDS: the exp table (64 doubles), then the image as DT [IMG][P].
  static __host__ __device__ constexpr size_t lds_bytes() {
    return kExpTab * sizeof(double) + (size_t)IMG * P * sizeof(DT);
  }
  static __device__ __forceinline__ int origin(double v) {
    if (!(fabs(v) < 1.0e7)) return 0;
    const int o = (int)floor(v + 0.5) - WIN / 2;
    return o < 0 ? 0 : (o > IMG - WIN ? IMG - WIN : o);
  }

  // 16-lane all-reduce (DPP inside a row); every lane of the chain gets the sum.
  static __device__ __forceinline__ double group_sum(double v) {
    v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_move<0x141>(v);  // row_half_mirror
    v += dpp_move<0x140>(v);  // row_mirror
    return v;
  }

  // Window pixels of this lane, the window origin they belong to (as doubles)
  // and the coordinate ranges over which that origin stays the same:
  // x in [xlo, xhi) implies floor(x + 0.5) == the cached unclamped origin
  // (xhi sits 2^-40 below the rounding boundary so that the rounded x + 0.5
  // cannot reach it; a false "moved" only costs a reload).
  struct Cache {
    DT d[NPX];
    double r0, c0;
    double xlo, xhi, ylo, yhi;
  };
  static __device__ __forceinline__ void init(Cache& k) {
    k.xlo = k.ylo = INFINITY;  // first step loads
    k.xhi = k.yhi = -INFINITY;
  }
  static __device__ __forceinline__ void bounds(double v, double& lo, double& hi) {
    if (!(fabs(v) < 1.0e7)) {  // absurd / NaN coordinate: re-check every step
      lo = INFINITY;
      hi = -INFINITY;
      return;
    }
    const double o = floor(v + 0.5);
    lo = o - 0.5;
    hi = (o + 0.5) - 0x1p-40;
  }

  // value of quad lane J (rows) / of lane (J, b) of the 16-lane group (columns)
  template <int J>
  static __device__ __forceinline__ double row_bcast(double v) {
    return dpp_move<J | (J << 2) | (J << 4) | (J << 6)>(v);
  }
  template <int J>
  static __device__ __forceinline__ double col_bcast(double v) {
    return swizzle_d<0x13 | ((J << 2) << 5)>(v);
  }

  // Make the cached window pixels those of the window at (x, y): re-read them
  // from the LDS image when round(x) or round(y) moved (wave-uniform branch).
  static __device__ __forceinline__ void ensure(const DT* __restrict__ sD, Cache& k, double x,
                                                double y) {
    const int m = lane_id() % LPC;
    const int a = m / 4, b = m % 4;
    const bool stay = x >= k.xlo && x < k.xhi && y >= k.ylo && y < k.yhi;
    if (__builtin_amdgcn_ballot_w64(!stay) != 0) {
      const int r0 = origin(x), c0 = origin(y);
      const DT* base = sD + (r0 + ROW0 + TR * a) * P + c0 + b;
#pragma unroll
      for (int i = 0; i < TR; ++i)
#pragma unroll
        for (int j = 0; j < TC; ++j) k.d[i * TC + j] = base[i * P + 4 * j];
      k.r0 = (double)r0;
      k.c0 = (double)c0;
      bounds(x, k.xlo, k.xhi);
      bounds(y, k.ylo, k.yhi);
    }
  }

  // The PSF factors of this lane's window rows (ex) and columns (ey, with the
  // 1/(2 pi sigma^2) normalisation): NTR rows + 2 columns evaluated per lane,
  // then broadcast (utils.py:475-486).
  static __device__ __forceinline__ void factors(const double* __restrict__ etab, const Cache& k,
                                                 double x, double y, const LeanConsts& lc,
                                                 double (&ex)[TR], double (&ey)[TC]) {
    const int m = lane_id() % LPC;
    const int a = m / 4, b = m % 4;
    const double r0 = k.r0, c0 = k.c0;
    double rv[2] = {0.0, 0.0}, cv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (t < NTR) {
        const double er = (double)(ROW0 + TR * a + b + 4 * t) + 0.5;  // exact: (r0 + e) + .5
        const double vr = (r0 + er) - x;
        rv[t] = exp_neg(-(vr * vr) * lc.inv_two_sig2, etab);
      }
      const double ec = (double)(b + 4 * (a + 4 * t)) + 0.5;
      const double vc = (c0 + ec) - y;
      cv[t] = exp_neg(-(vc * vc) * lc.inv_two_sig2, etab) * lc.inv_norm;
    }
#pragma unroll
    for (int i = 0; i < TR; ++i) {
      const double v = rv[i / 4];
      ex[i] = (i % 4 == 0) ? row_bcast<0>(v)
            : (i % 4 == 1) ? row_bcast<1>(v)
            : (i % 4 == 2) ? row_bcast<2>(v) : row_bcast<3>(v);
    }
#pragma unroll
    for (int j = 0; j < TC; ++j) {
      const double v = cv[j / 4];
      ey[j] = (j % 4 == 0) ? col_bcast<0>(v)
            : (j % 4 == 1) ? col_bcast<1>(v)
            : (j % 4 == 2) ? col_bcast<2>(v) : col_bcast<3>(v);
    }
  }

  // The same factors (ey times `scale`) from ONE exp per lane and two
  // multiplicative recurrences.  With v = r0 + i + 1/2 - x and c = 1/(2 sigma^2),
  //   ex(v + 1) = ex(v) g(v),  g(v) = exp(-c (2 v + 1)),  g(v + 1) = g(v) e^{-2c};
  // with w = c0 + j + 1/2 - y,
  //   ey(w + 4) = ey(w) h(w),  h(w) = exp(-c (8 w + 16)), h(w + 4) = h(w) e^{-32c}.
  // Lane (a, b) evaluates b = 0: ex at row group a's first row, b = 1: its g,
  // b = 2: ey at column a, b = 3: its h; DPP quad broadcasts hand the row
  // values round the quad, ds_bpermute the column values (lane (b, 2), (b, 3)).
  // Each factor is at most TR - 1 products from an exp: within ~25 ulp of the
  // direct exp (the direct factors already differ from the reference's
  // exp(-(dx^2 + dy^2) c) by a few ulp).  A wave with a chain so far from its
  // window that a base exp or a ratio could leave the fp64 range
  // (|v0| or |w0| >= rec_vmax, or NaN) takes the direct factors instead.
  static __device__ __forceinline__ void factors_rec(const double* __restrict__ etab,
                                                     const Cache& k, double x, double y,
                                                     const LeanConsts& lc, double scale,
                                                     double (&ex)[TR], double (&ey)[TC]) {
#if RHMC_FACT_REC
    const int lane = lane_id();
    const int m = lane % LPC;
    const int a = m / 4;
    const double v0 = (k.r0 + ((double)(ROW0 + TR * a) + 0.5)) - x;  // row group a, first row
    const double w0 = (k.c0 + ((double)a + 0.5)) - y;                // column a
    const bool ok = fabs(v0) < lc.rec_vmax && fabs(w0) < lc.rec_vmax;
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
      factors_from(etab, v0, w0, lc, scale, ex, ey);
      return;
    }
#endif
    factors(etab, k, x, y, lc, ex, ey);
#pragma unroll
    for (int j = 0; j < TC; ++j) ey[j] = scale * ey[j];
  }

  // The recurrence of factors_rec from the lane's row-group / column offsets
  // v0, w0 (in range for every chain of the wave).
  static __device__ __forceinline__ void factors_from(const double* __restrict__ etab, double v0,
                                                      double w0, const LeanConsts& lc,
                                                      double scale, double (&ex)[TR],
                                                      double (&ey)[TC]) {
    {
      const int lane = lane_id();
      const int m = lane % LPC;
      const int b = m % 4;
      const double c = lc.inv_two_sig2;
      const double z = (b < 2) ? v0 : w0;
      const double lin = (b < 2) ? fma(2.0, z, 1.0) : fma(8.0, z, 16.0);
      const double t = ((b & 1) ? lin : z * z) * -c;
      const double e = exp_neg(t, etab);
      const double ex0 = row_bcast<0>(e), g0 = row_bcast<1>(e);
      const int src = (lane & ~(LPC - 1)) + 4 * b;
      const double ey0 = __shfl(e, src + 2, kWave) * (lc.inv_norm * scale);
      const double h0 = __shfl(e, src + 3, kWave);
      ex[0] = ex0;
      double g = g0;
#pragma unroll
      for (int i = 1; i < TR; ++i) {
        ex[i] = ex[i - 1] * g;
        if (i + 1 < TR) g = g * lc.k_row;
      }
      ey[0] = ey0;
      double h = h0;
#pragma unroll
      for (int j = 1; j < TC; ++j) {
        ey[j] = ey[j - 1] * h;
        if (j + 1 < TC) h = h * lc.k_col4;
      }
    }
  }

  // The window's part of the chain's potential V (sampler_RHMC.py:294-302,
  // Lambda :373-376) relative to the background-only image:
  //   sum_window (Lambda - B) - D (ln Lambda - ln B).
  // Outside the window Lambda == B (the window bound), so
  // V = sum_image (B - D ln B) + this (every lane of the chain gets it).
  // lnB must be log_pos(B) (the same log on both sides of the difference).
  static __device__ __forceinline__ double potential_window(const double* __restrict__ etab,
                                                            const DT* __restrict__ sD, Cache& k,
                                                            double f, double x, double y,
                                                            const Consts& c,
                                                            const LeanConsts& lc, double lnB) {
    ensure(sD, k, x, y);
    double ex[TR], ey[TC];
    factors_rec(etab, k, x, y, lc, 1.0, ex, ey);
    double v = 0.0;
#pragma unroll
    for (int i = 0; i < TR; ++i) {
      const double fe = f * ex[i];
#pragma unroll
      for (int j = 0; j < TC; ++j) {
        const double lam = fma(fe, ey[j], c.B);
        v += (lam - c.B) - (double)k.d[i * TC + j] * (log_pos(lam) - lnB);
      }
    }
    return group_sum(v);
  }

  // The row slice's sums of the chain's dphidq pixel terms, all three scaled
  // by the flux fs = flux_fold(f) (out): s0 = fs sum psf s, s1 = fs sum psf s dx,
  // s2 = fs sum psf s dy
  // (s = D/Lambda - 1; every lane of the chain gets them).  The column
  // factors carry f (fey = f ey serves Lambda and both sums), so no separate
  // f ex row factors are held: 14 VGPRs and 7 products fewer.
  // PROFG (tools only): fenced clock reads split the gradient into gp[3] window
  // check, gp[0] PSF factors, gp[1] pixel loop, gp[2] moments + reductions.
  template <bool PROFG = false>
  static __device__ __forceinline__ void partial(const double* __restrict__ etab,
                                                 const DT* __restrict__ sD, Cache& k, double f,
                                                 double x, double y, const Consts& c,
                                                 const LeanConsts& lc, double& s0, double& s1,
                                                 double& s2, double& fs, long long* gp = nullptr) {
    long long t0 = 0;
    auto gmark = [&](int bkt) {
      if constexpr (PROFG) {
        __builtin_amdgcn_sched_barrier(0);
        const long long t1 = clock64();
        if (bkt >= 0) gp[bkt] += t1 - t0;
        t0 = t1;
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    gmark(-1);
    const int m = lane_id() % LPC;
    const int a = m / 4, b = m % 4;
    double ex[TR], ey[TC];
    ensure(sD, k, x, y);
    gmark(3);
    fs = flux_fold(f);
    factors_rec(etab, k, x, y, lc, fs, ex, ey);  // ey carries fs (= f but at |f| < 2^-547)
    const double r0 = k.r0, c0 = k.c0;
    gmark(0);

    // s_ij = D_ij / Lambda_ij - 1 with one reciprocal per group of kRcpGroup
    // pixels (row-major): 1/(l0 l1 l2 l3) by v_rcp_f64 + one Newton step, then
    // 1/l0 = l1 l2 l3 r etc. by products (v_rcp_f64 issues at a quarter of the
    // FMA rate); then the separable row / column sums (rhmc_tiled2.hpp).
    double R[TR], C[TC];
    // a0 = sum_i ex_i R_i is also sum_j fey_j C_j: it serves both moments
    double a0 = 0.0, a1 = 0.0, w1 = 0.0;
    auto fold = [&](int i) {  // row i's sum into the moments (in row order)
      const double tt = ex[i] * R[i];
      a0 += tt;
      if (i > 0) a1 = fma(tt, (double)i, a1);
    };
    auto lam = [&](int pp) {  // Lambda at pixel pp (:373-376)
      return fma(ex[pp / TC], ey[pp % TC], c.B);
    };
    auto acc = [&](int pp, double sv) {  // row / column sums of s (D/Lambda - 1, :379)
      const int i = pp / TC, j = pp % TC;
      R[i] = (j == 0) ? ey[j] * sv : fma(ey[j], sv, R[i]);
      C[j] = (i == 0) ? ex[i] * sv : fma(ex[i], sv, C[j]);
      if (RHMC_RFOLD && j == TC - 1) fold(i);
    };
    auto rcpn = [](double L) {
      const double r = __builtin_amdgcn_rcp(L);
      return fma(r, fma(-L, r, 1.0), r);
    };
    constexpr int G = kRcpGroup;
    constexpr int NG = NPX / G * G;
#pragma unroll
    for (int pp = 0; pp < NG; pp += G) {
      if constexpr (G == 4) {
        const double l0 = lam(pp), l1 = lam(pp + 1), l2 = lam(pp + 2), l3 = lam(pp + 3);
        const double l01 = l0 * l1, l23 = l2 * l3;
        const double r = rcpn(l01 * l23);
        const double r01 = l23 * r, r23 = l01 * r;
        acc(pp, fma((double)k.d[pp], l1 * r01, -1.0));
        acc(pp + 1, fma((double)k.d[pp + 1], l0 * r01, -1.0));
        acc(pp + 2, fma((double)k.d[pp + 2], l3 * r23, -1.0));
        acc(pp + 3, fma((double)k.d[pp + 3], l2 * r23, -1.0));
      } else {
        const double l0 = lam(pp), l1 = lam(pp + 1);
        const double r = rcpn(l0 * l1);
        acc(pp, fma((double)k.d[pp], l1 * r, -1.0));
        acc(pp + 1, fma((double)k.d[pp + 1], l0 * r, -1.0));
      }
    }
    if constexpr (NPX - NG >= 2) {
      constexpr int pp = NG;
      const double l0 = lam(pp), l1 = lam(pp + 1);
      const double r = rcpn(l0 * l1);
      acc(pp, fma((double)k.d[pp], l1 * r, -1.0));
      acc(pp + 1, fma((double)k.d[pp + 1], l0 * r, -1.0));
    }
    if constexpr ((NPX - NG) % 2 == 1) {  // last pixel on its own
      constexpr int pp = NPX - 1;
      acc(pp, fma((double)k.d[pp], rcpn(lam(pp)), -1.0));
    }
    gmark(1);
    if (!RHMC_RFOLD) {
#pragma unroll
      for (int i = 0; i < TR; ++i) fold(i);
    }
#pragma unroll
    for (int j = 1; j < TC; ++j) w1 = fma(ey[j] * C[j], (double)(4 * j), w1);
    const double dxa = ((r0 + (double)(ROW0 + TR * a)) - x) + 0.5;  // lane's row 0 offset
    const double dyb = ((c0 + (double)b) - y) + 0.5;                // lane's column 0 offset
    s0 = group_sum(a0);
    s1 = group_sum(fma(dxa, a0, a1));
    s2 = group_sum(fma(dyb, a0, w1));
    if constexpr (PROFG) {  // the sums must be complete at the mark
      asm volatile("" ::"v"(s0), "v"(s1), "v"(s2));
      gmark(2);
    }
  }

  // Pixel part of the chain's dphidq over the slice (the whole window for the
  // default slice).  partial's sums carry f: gx, gy need no f, gf one 1/f.
  template <bool PROFG = false>
  static __device__ __forceinline__ void gradient(const double* __restrict__ etab,
                                                  const DT* __restrict__ sD, Cache& k,
                                                  double f, double x, double y, const Consts& c,
                                                  const LeanConsts& lc, double& gf, double& gx,
                                                  double& gy, long long* gp = nullptr) {
    double s0, s1, s2, fs;
    partial<PROFG>(etab, sD, k, f, x, y, c, lc, s0, s1, s2, fs, gp);
    gf = -s0 * rcp_nr1(fs);                            // :404 (fs = flux_fold(f): f but for |f| < 2^-547)
    gx = -s1 * lc.inv_var;                             // :405
    gy = -s2 * lc.inv_var;                             // :406
  }
};

// One wave = 4 chains x 16 lanes; W waves per workgroup share the LDS image.
template <int IMG, int WIN, typename DT, bool PROF = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
leapfrog_k1_tiledr(LeapArgsK1 a) {
  using TL = TiledR<IMG, WIN, DT>;
  extern __shared__ double lds[];
  DT* simg = reinterpret_cast<DT*>(lds + kExpTab);
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    simg[r * TL::P + cc] = gimg[e];
  }
  exp_tab_fill(lds);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / TL::LPC;
  const int64_t chain = TL::CPW * wave + h;
  const bool real = chain < a.n_chains;            // ragged tail: mirror the wave's first chain
  const int64_t base = (real ? chain : TL::CPW * wave) * 3;

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  long long prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  k1_steps<PROF, TL::LPC>(f, x, y, pf, px, py, a.n_steps, (double)(IMG - 1), c, lc,
                 [&](double f_, double x_, double y_, double& gf, double& gx, double& gy) {
                   TL::template gradient<PROF>(lds, simg, cache, f_, x_, y_, c, lc, gf, gx, gy,
                                               prof + 4);
                 },
                 it_p, it_q, st, prof);
  if constexpr (PROF) {  // tools only: cycles per step per phase replace the state
    const double ns = a.n_steps > 0 ? a.n_steps : 1;
    f = prof[0] / ns;
    x = prof[1] / ns;
    y = prof[2] / ns;
    pf = prof[3] / ns;
    px = prof[4] / ns;  // gradient: window check + factors
    py = prof[5] / ns;  // pixel loop (prof[6], moments + reductions: it_p)
    it_p = (int)(prof[6] / ns);
    it_q = (int)(prof[7] / ns);  // window check
  }

  if ((lane % TL::LPC) == 0 && real) {
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

// The explicit integrators of single_gym for one star
// on the register-window gradient: plain HMC, unit metric (sampler_RHMC.py
// :628-645), explicit RHMC naive (:690-708) and leap_frog (:709-728).
// dVdq_RHMC's flux slot (:427-446), ((p_f^2 (-H_ff'/H_ff^2)) + H_ff'/H_ff +
// 2 H_xx'/H_xx)/2, is p_f^2 coef/2 + mterm of the division-lean FluxMetric,
// and p/H is p A (flux) / p s/g_xx (position).  The metric and gradient at
// the end of a step are the next step's first ones (same q).
template <int IMG, int WIN, typename DT, int SOLVER>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
integrate_k1_tiledr(LeapArgsK1 a, int f_pos) {
  using TL = TiledR<IMG, WIN, DT>;
  extern __shared__ double lds[];
  DT* simg = reinterpret_cast<DT*>(lds + kExpTab);
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    simg[r * TL::P + cc] = gimg[e];
  }
  exp_tab_fill(lds);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int64_t chain = TL::CPW * wave + lane / TL::LPC;
  const bool real = chain < a.n_chains;            // ragged tail: mirror the wave's first chain
  const int64_t base = (real ? chain : TL::CPW * wave) * 3;

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  const double dt = c.dt;
  unsigned st = 0u;
  FluxMetric fm{};
  double gf, gx, gy;
  auto grad = [&]() {                              // dVdq (:365-425)
    TL::gradient(lds, simg, cache, f, x, y, c, lc, gf, gx, gy);
    if (c.use_prior) gf += (SOLVER == RHMC_SOLVER_HMC) ? c.alpha / f : fm.prior;  // :408-409
  };
  auto dvdq_rhmc_f = [&](double p_f) { return (p_f * p_f) * fm.coef / 2.0 + fm.mterm; };
  // One gradient call site: pass s closes step s - 1 and opens step s (p holds
  // the half-step momentum across the gradient); naive's gradient opens its step.
  for (int s = 0;; ++s) {
    if constexpr (SOLVER != RHMC_SOLVER_HMC) fm = flux_metric(f, c, lc);
    grad();
    if (s > 0) {
      if constexpr (SOLVER == RHMC_SOLVER_HMC) {   // :630-638
        pf = pf - dt * gf / 2.0;
      } else if constexpr (SOLVER == RHMC_SOLVER_RHMC_LEAPFROG) {  // :711-726
        const double hf = pf;
        pf = hf - dt * (gf + dvdq_rhmc_f(hf)) / 2.0;
        if (f_pos && f < c.f_lim) {
          pf = hf * -1.0;
          st |= RHMC_STATUS_REFLECT_F;
        }
      }
      if constexpr (SOLVER != RHMC_SOLVER_RHMC_NAIVE) {
        px = px - dt * gx / 2.0;
        py = py - dt * gy / 2.0;
      }
    }
    if (s == a.n_steps) break;
    if constexpr (SOLVER == RHMC_SOLVER_HMC) {
      pf = pf - dt * gf / 2.0;
      px = px - dt * gx / 2.0;
      py = py - dt * gy / 2.0;
      f = f + dt * pf;
      x = x + dt * px;
      y = y + dt * py;
    } else if constexpr (SOLVER == RHMC_SOLVER_RHMC_NAIVE) {  // :692-705
      const double ihxx = fm.s * lc.inv_gxx;
      const double nf = f + (dt * pf) * fm.A, nx = x + (dt * px) * ihxx,
                   ny = y + (dt * py) * ihxx;
      const double pf_old = pf;
      pf = pf - dt * (gf + dvdq_rhmc_f(pf));
      px = px - dt * gx;
      py = py - dt * gy;
      if (f_pos && nf < c.f_lim) {
        pf = pf_old * -1.0;
        st |= RHMC_STATUS_REFLECT_F;
      }
      f = nf;
      x = nx;
      y = ny;
    } else {
      const double ihxx = fm.s * lc.inv_gxx;
      pf = pf - dt * (gf + dvdq_rhmc_f(pf)) / 2.0;
      px = px - dt * gx / 2.0;
      py = py - dt * gy / 2.0;
      f = f + (dt * pf) * fm.A;
      x = x + (dt * px) * ihxx;
      y = y + (dt * py) * ihxx;
    }
  }
  if ((lane % TL::LPC) == 0 && real) {
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
  }
}

// samplers.lightsource_gym.HMC_random's trajectory (samplers.py:519-552) for one
// star on the register-window gradient: unit-mass leapfrog with the step vector
// dtv[3], the chain's length steps[chain] >= 1 (wave lanes of finished chains
// idle; every cross-lane exchange stays inside a chain's 16 lanes), the flux wall
// at c.f_lim with the reference's quirks (hmc_random_win_kernel: the flip mask
// is never cleared; a trajectory whose last step flipped keeps its starting
// momentum, status RHMC_STATUS_REFLECT_F).  dVdq without the metric (:365-425).
template <int IMG, typename DT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
hmc_random_k1_tiledr(LeapArgsK1 a, const double* __restrict__ dtv,
                     const int32_t* __restrict__ steps) {
  using TL = TiledR<IMG, 28, DT>;
  extern __shared__ double lds[];
  DT* simg = reinterpret_cast<DT*>(lds + kExpTab);
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    simg[r * TL::P + cc] = gimg[e];
  }
  exp_tab_fill(lds);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int64_t chain = TL::CPW * wave + lane / TL::LPC;
  const bool real = chain < a.n_chains;            // ragged tail: mirror the wave's first chain
  const int64_t cr = real ? chain : TL::CPW * wave;
  const int64_t base = cr * 3;
  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const double dtf = dtv[0], dtx = dtv[1], dty = dtv[2];
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  double gf, gx, gy;
  auto grad = [&]() {                              // dVdq (:365-425)
    TL::gradient(lds, simg, cache, f, x, y, c, lc, gf, gx, gy);
    if (c.use_prior) gf += c.alpha / f;            // :408-409
  };
  grad();
  double hf = pf - dtf * gf / 2.0, hx = px - dtx * gx / 2.0,  // :519
         hy = py - dty * gy / 2.0;
  bool iflip = false, flip = false;
  const int n = steps[cr];
  for (int t = 0; t < n; ++t) {
    f = f + dtf * hf;                                          // :523
    x = x + dtx * hx;
    y = y + dty * hy;
    flip = f < c.f_lim;                                        // :526-529 (one star)
    iflip = iflip || flip;
    grad();
    const double kept = -hf;                                   // :531
    hf = hf - dtf * gf;                                        // :532, :535
    hx = hx - dtx * gx;
    hy = hy - dty * gy;
    if (flip && iflip) hf = kept;                              // :533
  }
  unsigned st = 0u;
  if (flip) {
    st |= RHMC_STATUS_REFLECT_F;  // p_tmp stays the starting momentum (:547-550)
  } else {                        // :551-552, dVdq at the same q as the last step
    pf = hf + dtf * gf / 2.0;
    px = hx + dtx * gx / 2.0;
    py = hy + dty * gy / 2.0;
  }
  if ((lane % TL::LPC) == 0 && real) {
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
  }
}

}  // namespace rhmc
