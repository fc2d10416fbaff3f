// rhmc_tiledrk.hpp — multi-star leapfrog (2 <= K <= 64, square images of side
// >= 32) on per-star pixel windows held in registers: 32 lanes per chain, two
// chains per wave64.  The many-star counterpart of rhmc_tiledr.hpp (C5:
// 256x256, K = 64; C3: 48x48, K = 10).
//
// Window.  Star k's window is 28 rows x 32 columns: rows
// floor(x + 0.5) - 14 .., columns floor(y + 0.5) - 16 .. (clamped into the
// image).  Every pixel left out is >= 14 px (rows) / 16 px (columns) from the
// star, where PSF/peak <= exp(-14^2 / (2 sigma^2)) <= 2^-62 — the bound
// rhmc_tiledr.hpp uses (reg_window_ok(28)): such a term changes neither
// Lambda (f PSF < half an ulp of B) nor the gradient sums beyond their own
// rounding.
//
// Gradient, star-major.  For star k (wave-uniform loop) every lane of a chain
// owns 28 pixels of k's window: lane m = 8 a + b owns rows 7 a .. 7 a + 6 and
// columns b, b + 8, b + 16, b + 24.  Lambda at those pixels sums B, star k and
// every star whose own window overlaps k's window (sampler_RHMC.py:373-376;
// any other star is outside its window on all of them, so its term is below
// half an ulp of B); the overlap mask is the union over the wave's two chains
// (a ballot), so a star counted for one chain only is still exact for the
// other.  PSF factors are separable (utils.py:475-486): lane (a, b) evaluates
// the row 7 a + b and the column b + 8 a factor — two exps per star — and
// ds_swizzle hands them round its row group / column group.  Then
// s = D/Lambda - 1 with one v_rcp_f64 per pixel pair, the separable row and
// column sums of rhmc_tiledr.hpp, and three 32-lane all-reduces
// (:379, :404-406).  The data pixels come from the fp32 copy of D when it is
// exact (else fp64), L2-resident and shared by every chain.
//
// Chain state: lane m holds stars m and m + 32 (SLOTS = 1 or 2) in registers;
// each gradient reads the chain's (f, x, y) per star from a per-wave LDS table
// written after every q-loop.  Fixed-point loops (:528-545) run over all the
// chain's stars at once with np.max's NaN rule via two ballots.
#pragma once
#include "rhmc_exp.hpp"
#include "rhmc_k1step.hpp"
#include "rhmc_tiledr.hpp"
#include "rhmc_wave.hpp"

namespace rhmc {

struct LeapArgsKR {
  double* q;
  double* p;
  int32_t* fp_iters;
  int32_t* status;
  const double* D;
  const float* Df;  // D in fp32 when exact, else nullptr
  int64_t n_chains;
  int K, n_steps, side, pad;
  Consts c;
  const double* dtv;      // kSolverHmcRandom: per-coordinate steps [3K]
  const int32_t* steps;   // kSolverHmcRandom: trajectory length per chain
  // ragged sets (rhmc_leapfrog_ragged_device; the pixel-major kernel's implicit
  // step only): chain i is row rows[i] (null: i) of [*][ld] arrays with Kc[row]
  // stars; K is then the set's largest star count
  const int32_t* Kc = nullptr;
  const int64_t* rows = nullptr;
  int64_t ld = 0;
};

// leapfrog_kr's SOLVER for samplers.HMC_random trajectories (not a C-ABI
// solver: rhmc_hmc_random selects it).
constexpr int kSolverHmcRandom = 100;

struct KRStar {  // LDS star table entry
  double f, x, y;
  double pad;     // flux_fold(f): the flux the pixel-major kernel folds into its factors
};

// TAB variant: Lambda over all stars in an unrolled loop (A/B knob), for at
// most TABK stars (kr_tables in rhmc_kernels.hip: K <= 16).
#ifndef RHMC_KR_ALLSTARS
#define RHMC_KR_ALLSTARS 1
#endif
constexpr bool kAllStarsTab = RHMC_KR_ALLSTARS;
constexpr int TABK = 16;
// TAB variant: the image staged in LDS instead of read from L2 (A/B knob).
#ifndef RHMC_KR_IMG_LDS
#define RHMC_KR_IMG_LDS 1
#endif
constexpr bool kImgLds = RHMC_KR_IMG_LDS;
// Window-major variant without tables (C5): the three per-window sums go to a
// per-chain LDS buffer and are reduced 8 windows at a time (0: three 32-lane
// all-reduces per window).
#ifndef RHMC_KR_DEFER
#define RHMC_KR_DEFER 1
#endif
constexpr bool kDeferRed = RHMC_KR_DEFER;

// This chain's half of a wave ballot (lanes 0-31 or 32-63).
__device__ __forceinline__ bool half_any(bool v) {
  const unsigned long long b = __builtin_amdgcn_ballot_w64(v);
  const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
  return (lane_id() < 32 ? lo : hi) != 0u;
}

// TAB: PSF factors read from per-chain LDS tables over the whole image
// (K x (rows + cols) doubles, rebuilt once per gradient) instead of two exps
// and eleven swizzles per (window, star) pair — for small images, where every
// window overlaps every other star's (C3: 48x48, K = 10).
template <typename DT, int SLOTS, bool TAB = false>
struct TiledRK {
  static constexpr int LPC = 32;           // lanes per chain
  static constexpr int CPW = kWave / LPC;  // chains per wave
  static constexpr int KMAX = LPC * SLOTS;
  static constexpr int WR = 28, WC = 32;   // window rows x columns
  static constexpr int TR = 7, TC = 4;     // rows x columns per lane
  static constexpr int NPX = TR * TC;
  static_assert(SLOTS == 1 || SLOTS == 2, "K <= 64");
  // all-stars Lambda loop: fp32-image variant only (the fp64-image one would
  // spill: its window pixels take twice the registers)
  static constexpr bool kAll = TAB && kAllStarsTab && sizeof(DT) == sizeof(float);
  // deferred sums: [8 windows x 3 sums] rows of RP doubles (32 lanes + pad:
  // 16-byte aligned rows, rows 4 banks apart)
  static constexpr bool kDefer = !TAB && kDeferRed;
  static constexpr int RB = 8, RP = 34;
  static constexpr int RED_DOUBLES = kDefer ? RB * 3 * RP : 0;

  // LDS: exp table, per-chain star tables, then (TAB) per-chain factor tables
  // and the image (DT [side][side], read by every window of the workgroup).
  // ws > 1 (window split, leapfrog_kr): per group of ws waves, two gradient
  // exchange buffers [CPW][KMAX][3] after everything else.
  static __host__ __device__ constexpr size_t xchg_doubles(int waves, int ws) {
    return ws > 1 ? (size_t)(waves / ws) * 2 * CPW * KMAX * 3 : 0;
  }
  static __host__ __device__ constexpr size_t lds_bytes(int waves, int K, int side,
                                                        int ws = 1) {
    return kExpTab * sizeof(double) + (size_t)waves * CPW * KMAX * sizeof(KRStar) +
           (TAB ? (size_t)waves * CPW * K * 2 * side * sizeof(double) +
                      (kImgLds ? (size_t)side * side * sizeof(DT) : 0)
                : (size_t)waves * CPW * RED_DOUBLES * sizeof(double)) +
           xchg_doubles(waves, ws) * sizeof(double);
  }
  static __device__ __forceinline__ int origin(double v, int half, int omax) {
    if (!(fabs(v) < 1.0e7)) return 0;
    const int o = (int)floor(v + 0.5) - half;
    return o < 0 ? 0 : (o > omax ? omax : o);
  }

  // PSF factors of a star at (xs, ys) on the window with origin (r0, c0):
  // ex[t] at row r0 + 7a + t, ey[u] at column c0 + b + 8u (carries `cscale`:
  // 1/(2 pi s^2), or f/(2 pi s^2) for a neighbour, whose factors only feed
  // Lambda — one product per lane before the exchange instead of TC after it).
  static __device__ __forceinline__ void factors(const double* __restrict__ etab, double r0,
                                                 double c0, double xs, double ys, int a, int b,
                                                 const LeanConsts& lc, double cscale,
                                                 double (&ex)[TR], double (&ey)[TC]) {
    const double vr = (r0 + ((double)(7 * a + b) + 0.5)) - xs;  // exact offsets
    const double er = exp_neg(-(vr * vr) * lc.inv_two_sig2, etab);
    const double vc = (c0 + ((double)(b + 8 * a) + 0.5)) - ys;
    const double ec = exp_neg(-(vc * vc) * lc.inv_two_sig2, etab) * cscale;
    // rows: lane (a, t) of my 8-lane row group; columns: lane (u, b)
    ex[0] = swizzle_d<0x18 | (0 << 5)>(er);
    ex[1] = swizzle_d<0x18 | (1 << 5)>(er);
    ex[2] = swizzle_d<0x18 | (2 << 5)>(er);
    ex[3] = swizzle_d<0x18 | (3 << 5)>(er);
    ex[4] = swizzle_d<0x18 | (4 << 5)>(er);
    ex[5] = swizzle_d<0x18 | (5 << 5)>(er);
    ex[6] = swizzle_d<0x18 | (6 << 5)>(er);
    ey[0] = swizzle_d<0x07 | (0 << 5)>(ec);
    ey[1] = swizzle_d<0x07 | (8 << 5)>(ec);
    ey[2] = swizzle_d<0x07 | (16 << 5)>(ec);
    ey[3] = swizzle_d<0x07 | (24 << 5)>(ec);
  }

  // TAB: the chain's factor tables, [K][rows | cols] (utils.py:475-486 per axis).
  static __device__ __forceinline__ void build_tables(const double* __restrict__ etab,
                                                      double* ftab, const KRStar* tab, int K,
                                                      int side, const LeanConsts& lc) {
    const int m = lane_id() & (LPC - 1);
    const int per = 2 * side, total = K * per;
    wave_lds_sync();  // the previous gradient's reads are done
    for (int e = m; e < total; e += LPC) {
      const int k = e / per, r = e - k * per;
      const bool col = r >= side;
      const int i = col ? r - side : r;
      const KRStar sk = tab[k];
      const double v = ((double)i + 0.5) - (col ? sk.y : sk.x);
      const double val = exp_neg(-(v * v) * lc.inv_two_sig2, etab);
      ftab[e] = col ? val * lc.inv_norm : val;
    }
    wave_lds_sync();
  }

  // Factors of star s on the window (R0, C0): exps + swizzles, or table reads.
  static __device__ __forceinline__ void star_factors(const double* __restrict__ etab,
                                                      const double* ftab, int side, int s,
                                                      const KRStar& ss, int R0, int C0, int a,
                                                      int b, const LeanConsts& lc,
                                                      double (&ex)[TR], double (&ey)[TC]) {
    if constexpr (TAB) {
      const double* tr = ftab + (size_t)s * 2 * side + R0 + TR * a;
      const double* tc = ftab + (size_t)s * 2 * side + side + C0 + b;
#pragma unroll
      for (int i = 0; i < TR; ++i) ex[i] = tr[i];
#pragma unroll
      for (int j = 0; j < TC; ++j) ey[j] = tc[8 * j];
    } else {
      factors(etab, (double)R0, (double)C0, ss.x, ss.y, a, b, lc, lc.inv_norm, ex, ey);
    }
  }

  // Pixel part of dphidq for every star of the chain (:365-425 without the
  // metric / prior terms): lane m receives stars m + 32 t in slot t.
  // Window split (WS > 1): the WS waves of a group hold the same two chains
  // (identical replicated state); wave wsub evaluates the windows of stars
  // m = wsub (mod WS) and the group swaps the results through xb (this
  // gradient's exchange buffer, [CPW][KMAX][3]) across one workgroup barrier.
  // Every window's sums are the same operations in the same order as with
  // WS = 1, so the results are bit-identical.
  template <int WS = 1>
  static __device__ __forceinline__ void gradient(const double* __restrict__ etab,
                                                  const DT* __restrict__ img, int side,
                                                  const KRStar* tab, double* ftab, int K,
                                                  const double (&xs)[SLOTS],
                                                  const double (&ys)[SLOTS],
                                                  const bool (&own)[SLOTS], const Consts& c,
                                                  const LeanConsts& lc, double (&gf)[SLOTS],
                                                  double (&gx)[SLOTS], double (&gy)[SLOTS],
                                                  int wsub = 0, double* xb = nullptr) {
    const int m = lane_id() & (LPC - 1);
    const int a = m >> 3, b = m & 7;
    const int rmax = side - WR, cmax = side - WC;
    if constexpr (TAB) build_tables(etab, ftab, tab, K, side, lc);
    int ro[SLOTS], co[SLOTS];
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      ro[t] = origin(xs[t], WR / 2, rmax);
      co[t] = origin(ys[t], WC / 2, cmax);
      gf[t] = gx[t] = gy[t] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
#pragma unroll 1
      for (int li = 0;; ++li) {  // this wave's windows: kk = wsub + WS li
        const int kk = wsub + WS * li;
        const int k = LPC * t + kk;
        if (kk >= LPC || k >= K) break;
        const KRStar sk = tab[k];
        const int R0 = origin(sk.x, WR / 2, rmax), C0 = origin(sk.y, WC / 2, cmax);
        // data pixels of the window (issued before the neighbour work)
        DT d[NPX];
        const DT* base = img + (size_t)(R0 + TR * a) * side + (C0 + b);
#pragma unroll
        for (int i = 0; i < TR; ++i)
#pragma unroll
          for (int j = 0; j < TC; ++j) d[i * TC + j] = base[(size_t)i * side + 8 * j];

        const double r0 = (double)R0, c0 = (double)C0;
        double lam[NPX];
        // Lambda = B + the stars' terms; the first star's FMAs take B itself as
        // the addend (no copies of B into the NPX accumulators: same values)
        bool started = false;  // wave-uniform
        auto add_scaled = [&](const double (&ex)[TR], const double (&fy)[TC]) {
          if (started) {
#pragma unroll
            for (int i = 0; i < TR; ++i)
#pragma unroll
              for (int j = 0; j < TC; ++j) lam[i * TC + j] = fma(ex[i], fy[j], lam[i * TC + j]);
          } else {
#pragma unroll
            for (int i = 0; i < TR; ++i)
#pragma unroll
              for (int j = 0; j < TC; ++j) lam[i * TC + j] = fma(ex[i], fy[j], c.B);
          }
          started = true;
        };
        auto add_star = [&](double fs, const double (&ex)[TR], const double (&ey)[TC]) {
          // f scales the TC column factors (fewer products than the TR rows)
          double fy[TC];
#pragma unroll
          for (int j = 0; j < TC; ++j) fy[j] = fs * ey[j];
          add_scaled(ex, fy);
        };
        if constexpr (kAll) {
          // Small images (C3): nearly every window overlaps every star, so
          // Lambda sums ALL the chain's stars in ascending order, as the
          // reference does (:373-376), in a fully unrolled loop: table reads
          // at constant offsets and no mask bookkeeping.  A star whose window
          // misses k's adds less than half an ulp of B (the window bound).
#pragma unroll
          for (int s = 0; s < TABK; ++s) {
            if (s < K) {  // wave-uniform
              double ex[TR], ey[TC];
              star_factors(etab, ftab, side, s, tab[s], R0, C0, a, b, lc, ex, ey);
              add_star(tab[s].f, ex, ey);
            }
          }
        } else {
          // stars whose PSF support reaches k's window (rows R0 .. R0 + WR - 1, columns
          // C0 .. C0 + WC - 1): every pixel 14 px or more from a star in rows or in
          // columns gets PSF/peak <= 2^-62 (the window bound, reg_window_ok(28)), so
          // the star counts when x lies in (R0 - 13.5, R0 + WR + 13.5) and y in
          // (C0 - 13.5, C0 + WC + 13.5) — and always when x or y is NaN (the reference
          // spreads it); union over the two chains
          const double rlo = (double)R0 - 13.5, rhi = (double)(R0 + WR) + 13.5;
          const double clo = (double)C0 - 13.5, chi = (double)(C0 + WC) + 13.5;
          unsigned long long nbm = 0ull;
#pragma unroll
          for (int t2 = 0; t2 < SLOTS; ++t2) {
            const int j = LPC * t2 + m;
            const bool nb = own[t2] && j != k && !(xs[t2] <= rlo || xs[t2] >= rhi) &&
                            !(ys[t2] <= clo || ys[t2] >= chi);
            const unsigned long long bl = __builtin_amdgcn_ballot_w64(nb);
            nbm |= (unsigned long long)((unsigned)bl | (unsigned)(bl >> 32)) << (LPC * t2);
          }
          while (nbm) {  // wave-uniform
            const int s = __builtin_ctzll(nbm);
            nbm &= nbm - 1;
            const KRStar ss = tab[s];
            double ex[TR], ey[TC];
            if constexpr (TAB) {
              star_factors(etab, ftab, side, s, ss, R0, C0, a, b, lc, ex, ey);
              add_star(ss.f, ex, ey);
            } else {  // ey = f ey: the flux folded in before the exchange
              factors(etab, (double)R0, (double)C0, ss.x, ss.y, a, b, lc, ss.f * lc.inv_norm,
                      ex, ey);
              add_scaled(ex, ey);
            }
          }
        }
        double ex[TR], ey[TC];
        star_factors(etab, ftab, side, k, sk, R0, C0, a, b, lc, ex, ey);
        if constexpr (!kAll) add_star(sk.f, ex, ey);
        // s = D/Lambda - 1, one reciprocal per pixel pair (rhmc_tiledr.hpp)
        double R[TR], C[TC];
        auto acc = [&](int pp, double sv) {
          const int i = pp / TC, j = pp % TC;
          R[i] = (j == 0) ? ey[j] * sv : fma(ey[j], sv, R[i]);
          C[j] = (i == 0) ? ex[i] * sv : fma(ex[i], sv, C[j]);
        };
        static_assert(NPX % 4 == 0, "pixel groups of four");
#pragma unroll
        for (int pp = 0; pp < NPX; pp += kRcpGroup) {
          if constexpr (kRcpGroup == 4) {  // one v_rcp_f64 per 4 pixels (rhmc_tiledr.hpp)
            const double l0 = lam[pp], l1 = lam[pp + 1], l2 = lam[pp + 2], l3 = lam[pp + 3];
            const double l01 = l0 * l1, l23 = l2 * l3;
            const double r = rcp_nr1(l01 * l23);
            const double r01 = l23 * r, r23 = l01 * r;
            acc(pp, fma((double)d[pp], l1 * r01, -1.0));
            acc(pp + 1, fma((double)d[pp + 1], l0 * r01, -1.0));
            acc(pp + 2, fma((double)d[pp + 2], l3 * r23, -1.0));
            acc(pp + 3, fma((double)d[pp + 3], l2 * r23, -1.0));
          } else {
            const double l0 = lam[pp], l1 = lam[pp + 1];
            const double r = rcp_nr1(l0 * l1);
            acc(pp, fma((double)d[pp], l1 * r, -1.0));
            acc(pp + 1, fma((double)d[pp + 1], l0 * r, -1.0));
          }
        }
        double a0 = 0.0, a1 = 0.0, w0 = 0.0, w1 = 0.0;
#pragma unroll
        for (int i = 0; i < TR; ++i) {
          const double tt = ex[i] * R[i];
          a0 += tt;
          a1 = fma(tt, (double)i, a1);
        }
#pragma unroll
        for (int j = 0; j < TC; ++j) {
          const double w = ey[j] * C[j];
          w0 += w;
          w1 = fma(w, (double)(8 * j), w1);
        }
        const double dxa = ((r0 + (double)(TR * a)) - sk.x) + 0.5;
        const double dyb = ((c0 + (double)b) - sk.y) + 0.5;
        if constexpr (kDefer) {
          // this lane's share of the window's three sums -> the chain's buffer;
          // every RB windows (and after the slot's last) lane 3 w + c sums row
          // (w, c) over the 32 lanes and lane kk0 + w collects window w's three
          // (ftab is the buffer here)
          double* row = ftab + (size_t)((li % RB) * 3) * RP + m;
          row[0] = a0;
          row[RP] = fma(dxa, a0, a1);
          row[2 * RP] = fma(dyb, w0, w1);
          if (li % RB == RB - 1 || k + WS >= K || kk + WS >= LPC) {  // wave-uniform
            wave_lds_sync();
            const int li0 = li - li % RB;
            const double* rr = ftab + (size_t)(m < 3 * RB ? m : 0) * RP;
            double v[LPC / 2];  // pairwise tree over the 32 lanes' shares
#pragma unroll
            for (int l = 0; l < LPC / 2; ++l) v[l] = rr[2 * l] + rr[2 * l + 1];
#pragma unroll
            for (int n = LPC / 4; n >= 1; n /= 2)
#pragma unroll
              for (int l = 0; l < n; ++l) v[l] = v[l] + v[l + n];
            const double sum = v[0];
            // this lane's window in the batch (lane m: star m of the slot)
            const int mf = WS > 1 ? lane_id_fresh() & (LPC - 1) : m;
            const bool mine = mf >= wsub && (mf - wsub) % WS == 0;
            const int w = mine ? (mf - wsub) / WS - li0 : -1;
            const int src = (lane_id() & 32) + 3 * (w >= 0 && w < RB ? w : 0);
            const double s0 = __shfl(sum, src, kWave);
            const double s1 = __shfl(sum, src + 1, kWave);
            const double s2 = __shfl(sum, src + 2, kWave);
            if (w >= 0 && w <= li - li0) {
              const double fk = tab[LPC * t + m].f;
              gf[t] = -s0;                          // :404
              gx[t] = -s1 * fk * lc.inv_var;        // :405
              gy[t] = -s2 * fk * lc.inv_var;        // :406
            }
            wave_lds_sync();                        // reads done before the next batch
          }
        } else {
          const double s0 = half_sum_dpp(a0);
          const double s1 = half_sum_dpp(fma(dxa, a0, a1));
          const double s2 = half_sum_dpp(fma(dyb, w0, w1));
          if (m == kk) {
            gf[t] = -s0;                            // :404
            gx[t] = -s1 * sk.f * lc.inv_var;        // :405
            gy[t] = -s2 * sk.f * lc.inv_var;        // :406
          }
        }
      }
    }
    if constexpr (WS > 1) {
      // the group's swap: lane m publishes its stars evaluated here and reads
      // the others' (one buffer per gradient, alternating: a barrier between
      // a buffer's writes and the next writes to it is the next gradient's)
      const int lf = lane_id_fresh(), mf = lf & (LPC - 1);
      double* xc = xb + (size_t)(lf >> 5) * KMAX * 3;  // this chain's rows
      const bool here = mf % WS == wsub;
#pragma unroll
      for (int t = 0; t < SLOTS; ++t)
        if (own[t] && here) {
          double* e = xc + 3 * (LPC * t + mf);
          e[0] = gf[t];
          e[1] = gx[t];
          e[2] = gy[t];
        }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < SLOTS; ++t)
        if (own[t] && !here) {
          const double* e = xc + 3 * (LPC * t + mf);
          gf[t] = e[0];
          gx[t] = e[1];
          gy[t] = e[2];
        }
    }
    if (c.use_Vc) {  // repulsion (:411-418), O(K^2) from the star table
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        double sx = 0.0, sy = 0.0;
        for (int jj = 0; jj < K; ++jj) {
          const KRStar o = tab[jj];
          const double ddx = o.x - xs[t], ddy = o.y - ys[t];
          double Rr = sqrt(ddx * ddx + ddy * ddy);
          if (fabs(Rr) < 1e-10) Rr = 1e32;
          const double tr = pow(1.0 / Rr, c.vc_pow + 2.0);
          sx += tr * ddx;
          sy += tr * ddy;
        }
        gx[t] += c.beta * sx * c.vc_pow;
        gy[t] += c.beta * sy * c.vc_pow;
      }
    }
  }
};

// The chain's star table: lane m writes its slot stars (f, x, y).
template <int SLOTS>
__device__ __forceinline__ void kr_publish(KRStar* tab, const double (&f)[SLOTS],
                                           const double (&x)[SLOTS], const double (&y)[SLOTS],
                                           const bool (&own)[SLOTS]) {
  const int m = lane_id() & 31;
  wave_lds_sync();  // every lane has finished reading the previous table
#pragma unroll
  for (int t = 0; t < SLOTS; ++t)
    if (own[t]) {
      KRStar e;
      e.f = f[t];
      e.x = x[t];
      e.y = y[t];
      e.pad = flux_fold(f[t]);
      tab[32 * t + m] = e;
    }
  wave_lds_sync();
}

// The chain's (f, x, y) back from its star table (RELOAD step loops: the
// state is not held in registers across a gradient that reads it from the
// table anyway; lanes without a star get the placeholder 1, 0, 0).
template <int SLOTS>
__device__ __forceinline__ void kr_reload(const KRStar* tab, double (&f)[SLOTS],
                                          double (&x)[SLOTS], double (&y)[SLOTS],
                                          const bool (&own)[SLOTS]) {
  const int m = lane_id() & 31;
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    const KRStar e = tab[own[t] ? 32 * t + m : 0];
    f[t] = own[t] ? e.f : 1.0;
    x[t] = own[t] ? e.x : 0.0;
    y[t] = own[t] ? e.y : 0.0;
  }
}

// n_steps steps of RHMC_single_step (sampler_RHMC.py:522-566) for the chain's
// stars (lane m: stars m + 32 t).  The end-of-step gradient is carried into
// the next step; the flux metric is computed once per distinct f
// (rhmc_k1step.hpp); the loops stop on np.max(|dq|) <= delta, NaN included.
template <int SLOTS, class GRAD, bool RELOAD = false>
__device__ __forceinline__ void km_steps(double (&f)[SLOTS], double (&x)[SLOTS],
                                         double (&y)[SLOTS], double (&pf)[SLOTS],
                                         double (&px)[SLOTS], double (&py)[SLOTS],
                                         const bool (&own)[SLOTS], KRStar* tab, int n_steps,
                                         double edge, const Consts& c, const LeanConsts& lc,
                                         GRAD grad, int& it_p, int& it_q, unsigned& st) {
  const double hdt = c.hdt;
  FluxMetric fm[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) fm[t] = flux_metric(f[t], c, lc);
  kr_publish<SLOTS>(tab, f, x, y, own);
  unsigned long long near_bal = 0ull;
  for (int s = 0;; ++s) {
    double gf[SLOTS], gx[SLOTS], gy[SLOTS];
    if (s > 0) {
      // near-wall test of this iteration's position reflections (below; x, y
      // are unchanged until the next q-loop), kept as a wave-uniform ballot
      // mask in SGPRs: these loops run at the VGPR limit
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        const bool nx = (x[t] < 0.0 || x[t] > edge) && near_edge(x[t], edge);
        const bool ny = (y[t] < 0.0 || y[t] > edge) && near_edge(y[t], edge);
        near_bal |= __builtin_amdgcn_ballot_w64(own[t] && (nx || ny));
      }
    }
    grad(x, y, gf, gx, gy);
    if constexpr (RELOAD) kr_reload<SLOTS>(tab, f, x, y, own);
    // Recompute the flux metric instead of keeping it live through the
    // gradient (register pressure): the asm hides f's value from CSE.
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      double fr = f[t];
      asm volatile("" : "+v"(fr));
      fm[t] = flux_metric(fr, c, lc);
    }
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      if (c.use_prior) gf[t] += fm[t].prior;       // :408-409
      gf[t] += fm[t].mterm;                        // :459-463
      if (s > 0) {
        pf[t] = pf[t] - hdt * gf[t];               // :551
        px[t] = px[t] - hdt * gx[t];
        py[t] = py[t] - hdt * gy[t];
        if (f[t] < c.f_lim) {                      // :554-564
          pf[t] = -pf[t];
          if (own[t]) st |= RHMC_STATUS_REFLECT_F;
          if (own[t] && f[t] >= c.near_f) st |= RHMC_STATUS_NEAR_WALL;
        }
        if (x[t] < 0.0 || x[t] > edge) {
          px[t] = -px[t];
          if (own[t]) st |= RHMC_STATUS_REFLECT_XY;
        }
        if (y[t] < 0.0 || y[t] > edge) {
          py[t] = -py[t];
          if (own[t]) st |= RHMC_STATUS_REFLECT_XY;
        }
      }
    }
    if (s == n_steps) break;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      pf[t] = pf[t] - hdt * gf[t];                 // :525
      px[t] = px[t] - hdt * gx[t];
      py[t] = py[t] - hdt * gy[t];
    }
    {  // p-loop (:528-535), flux slots only (dtaudq is 0 on x, y)
      double rho[SLOTS], hc[SLOTS];
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        rho[t] = pf[t];
        hc[t] = hdt * (fm[t].coef * 0.5);
      }
      int n = 0;
      bool more;
      do {
        bool go = false, nan = false;
#pragma unroll
        for (int t = 0; t < SLOTS; ++t) {
          const double P = fma(-hc[t], pf[t] * pf[t], rho[t]);
          const double d = fabs(pf[t] - P);
          pf[t] = P;
          if (own[t]) {
            go |= d > c.delta;
            nan |= d != d;
          }
        }
        ++n;
        more = half_any(go) && !half_any(nan);
      } while (more && n < c.counter_max);
      it_p += n;
      if (more) st |= RHMC_STATUS_PLOOP_CAP;
    }
    {  // q-loop (:538-545): q' = q_s + hdt (p/H(q_s) + p/H(q)), affine in f and g(f)
      double bf[SLOTS], cf[SLOTS], bx[SLOTS], cx[SLOTS], by[SLOTS], cy[SLOTS];
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        const double ihxx_s = fm[t].s * lc.inv_gxx;
        bf[t] = hdt * (pf[t] * lc.inv_gff2);
        cf[t] = f[t] + hdt * (pf[t] * fm[t].A + pf[t] * lc.c0);
        bx[t] = hdt * (px[t] * lc.inv_gxx);
        cx[t] = x[t] + hdt * (px[t] * ihxx_s);
        by[t] = hdt * (py[t] * lc.inv_gxx);
        cy[t] = y[t] + hdt * (py[t] * ihxx_s);
      }
      int n = 0;
      bool more;
      do {
        bool go = false, nan = false;
#pragma unroll
        for (int t = 0; t < SLOTS; ++t) {
          const double F = fma(bf[t], f[t], cf[t]);
          const double fl = (f[t] < lc.f_low) ? lc.f_low : f[t];
          const double u = rcp_nr1(fl);
          const double g = u * fma(lc.Bg2, u, lc.inv_g1);
          const double X = fma(bx[t], g, cx[t]);
          const double Y = fma(by[t], g, cy[t]);
          const double a0 = fabs(f[t] - F), a1 = fabs(x[t] - X), a2 = fabs(y[t] - Y);
          const double sum = a0 + a1 + a2;
          f[t] = F;
          x[t] = X;
          y[t] = Y;
          if (own[t]) {
            go |= fmax(fmax(a0, a1), a2) > c.delta;
            nan |= sum != sum;
          }
        }
        ++n;
        more = half_any(go) && !half_any(nan);
      } while (more && n < c.counter_max);
      it_q += n;
      if (more) st |= RHMC_STATUS_QLOOP_CAP;
    }
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      fm[t] = flux_metric(f[t], c, lc);
      pf[t] = pf[t] - hdt * ((pf[t] * pf[t]) * fm[t].coef / 2.0);  // :548
    }
    kr_publish<SLOTS>(tab, f, x, y, own);
  }
  // the chain's 32-lane half of the near-wall mask
  if ((near_bal >> (lane_id() & 32)) & 0xFFFFFFFFull) st |= RHMC_STATUS_NEAR_WALL;
}

// n_steps steps of single_gym's explicit integrators for
// the chain's stars: plain HMC, unit metric (sampler_RHMC.py:628-645), explicit
// RHMC naive (:690-708) and leap_frog (:709-728), flux wall under f_pos.
// dVdq_RHMC's flux slot (:427-446) is p_f^2 coef/2 + mterm of the division-
// lean FluxMetric; p/H is p A (flux) and p s/g_xx (positions).  The gradient
// and metric at the end of a step are the next step's first ones; the metric
// is recomputed after each gradient rather than held across it (km_steps).
template <int SOLVER, int SLOTS, class GRAD, bool RELOAD = false>
__device__ __forceinline__ void km_explicit_steps(double (&f)[SLOTS], double (&x)[SLOTS],
                                                  double (&y)[SLOTS], double (&pf)[SLOTS],
                                                  double (&px)[SLOTS], double (&py)[SLOTS],
                                                  const bool (&own)[SLOTS], KRStar* tab,
                                                  int n_steps, int f_pos, const Consts& c,
                                                  const LeanConsts& lc, GRAD grad,
                                                  unsigned& st) {
  const double dt = c.dt;
  FluxMetric fm[SLOTS];
  double gf[SLOTS], gx[SLOTS], gy[SLOTS];
  auto metric = [&]() {
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      double fr = f[t];
      asm volatile("" : "+v"(fr));
      fm[t] = flux_metric(fr, c, lc);
    }
  };
  auto gradient = [&]() {  // dVdq (:365-425) at the published state
    grad(x, y, gf, gx, gy);
    if constexpr (RELOAD) kr_reload<SLOTS>(tab, f, x, y, own);
#pragma unroll
    for (int t = 0; t < SLOTS; ++t)
      if (c.use_prior) gf[t] += c.alpha / f[t];     // :408-409
    // leap_frog needs the metric at the new f right away; naive computes it
    // at the start of its next step (fewer live registers at SLOTS = 2)
    if constexpr (SOLVER == RHMC_SOLVER_RHMC_LEAPFROG) metric();
  };
  auto dvdq_rhmc_f = [&](int t, double p_f) {
    return (p_f * p_f) * fm[t].coef / 2.0 + fm[t].mterm;
  };
  kr_publish<SLOTS>(tab, f, x, y, own);
  if constexpr (SOLVER == RHMC_SOLVER_RHMC_NAIVE) {  // :692-705
    // the gradient opens each step (nothing of it lives across steps)
    for (int s = 0; s < n_steps; ++s) {
      gradient();
      metric();
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        const double ihxx = fm[t].s * lc.inv_gxx;
        const double nf = f[t] + (dt * pf[t]) * fm[t].A;
        x[t] = x[t] + (dt * px[t]) * ihxx;
        y[t] = y[t] + (dt * py[t]) * ihxx;
        const double pf_old = pf[t];
        pf[t] = pf[t] - dt * (gf[t] + dvdq_rhmc_f(t, pf[t]));
        px[t] = px[t] - dt * gx[t];
        py[t] = py[t] - dt * gy[t];
        if (f_pos && nf < c.f_lim) {
          pf[t] = pf_old * -1.0;
          if (own[t]) st |= RHMC_STATUS_REFLECT_F;
        }
        f[t] = nf;
      }
      kr_publish<SLOTS>(tab, f, x, y, own);
    }
    return;
  }
  // HMC (:630-638) / leap_frog (:711-726): one gradient call site (code size:
  // the gradient is most of the kernel), pass s closes step s - 1 and opens
  // step s; p holds the half-step momentum across the gradient.
  for (int s = 0;; ++s) {
    gradient();
    if (s > 0) {
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        if constexpr (SOLVER == RHMC_SOLVER_HMC) {
          pf[t] = pf[t] - dt * gf[t] / 2.0;
        } else {
          const double hf = pf[t];
          pf[t] = hf - dt * (gf[t] + dvdq_rhmc_f(t, hf)) / 2.0;
          if (f_pos && f[t] < c.f_lim) {
            pf[t] = hf * -1.0;
            if (own[t]) st |= RHMC_STATUS_REFLECT_F;
          }
        }
        px[t] = px[t] - dt * gx[t] / 2.0;
        py[t] = py[t] - dt * gy[t] / 2.0;
      }
    }
    if (s == n_steps) break;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      if constexpr (SOLVER == RHMC_SOLVER_HMC) {
        pf[t] = pf[t] - dt * gf[t] / 2.0;
        px[t] = px[t] - dt * gx[t] / 2.0;
        py[t] = py[t] - dt * gy[t] / 2.0;
        f[t] = f[t] + dt * pf[t];
        x[t] = x[t] + dt * px[t];
        y[t] = y[t] + dt * py[t];
      } else {
        const double ihxx = fm[t].s * lc.inv_gxx;
        pf[t] = pf[t] - dt * (gf[t] + dvdq_rhmc_f(t, pf[t])) / 2.0;
        px[t] = px[t] - dt * gx[t] / 2.0;
        py[t] = py[t] - dt * gy[t] / 2.0;
        f[t] = f[t] + (dt * pf[t]) * fm[t].A;
        x[t] = x[t] + (dt * px[t]) * ihxx;
        y[t] = y[t] + (dt * py[t]) * ihxx;
      }
    }
    kr_publish<SLOTS>(tab, f, x, y, own);
  }
}

// samplers.lightsource_gym.HMC_random's trajectory (samplers.py:519-552) for the
// chain's stars: unit mass, per-coordinate steps dtv, n leapfrog steps, the
// flux wall at c.f_lim with the reference's quirks (hmc_random_win_kernel: a
// star's flip flag is never cleared; the flip applies on every step where ANY
// of the chain's stars is below the wall).  p holds the half-step momentum;
// returns true when the last step flipped — the caller then keeps the
// starting momentum (:547-550).  dVdq without the metric (:365-425).
template <int SLOTS, class GRAD, bool RELOAD = false>
__device__ __forceinline__ bool km_hmc_random_steps(double (&f)[SLOTS], double (&x)[SLOTS],
                                                    double (&y)[SLOTS], double (&pf)[SLOTS],
                                                    double (&px)[SLOTS], double (&py)[SLOTS],
                                                    const bool (&own)[SLOTS], KRStar* tab,
                                                    int n, const double* __restrict__ dtv,
                                                    const Consts& c, GRAD grad) {
  const int m = lane_id() & 31;
  // the steps are re-read from memory (L1/L2) where used instead of being held
  // in registers across the gradient (register pressure at two slots)
  // (the index goes through an empty asm so that the loads are not hoisted)
  auto dti = [&](int t, int j) {
    int i = 3 * (own[t] ? 32 * t + m : 0) + j;
    asm volatile("" : "+v"(i));
    return dtv[i];
  };
  auto dtf = [&](int t) { return dti(t, 0); };
  auto dtx = [&](int t) { return dti(t, 1); };
  auto dty = [&](int t) { return dti(t, 2); };
  bool iflip[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) iflip[t] = false;
  double gf[SLOTS], gx[SLOTS], gy[SLOTS];
  auto gradient = [&]() {
    grad(x, y, gf, gx, gy);
    if constexpr (RELOAD) kr_reload<SLOTS>(tab, f, x, y, own);
#pragma unroll
    for (int t = 0; t < SLOTS; ++t)
      if (c.use_prior) gf[t] += c.alpha / f[t];    // :408-409
  };
  kr_publish<SLOTS>(tab, f, x, y, own);
  gradient();
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {                // :519
    pf[t] = pf[t] - dtf(t) * gf[t] / 2.0;
    px[t] = px[t] - dtx(t) * gx[t] / 2.0;
    py[t] = py[t] - dty(t) * gy[t] / 2.0;
  }
  bool flip = false;
  for (int s = 0; s < n; ++s) {
    bool below_any = false;
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      f[t] = f[t] + dtf(t) * pf[t];                // :523
      x[t] = x[t] + dtx(t) * px[t];
      y[t] = y[t] + dty(t) * py[t];
      const bool below = own[t] && f[t] < c.f_lim; // :526-529
      iflip[t] = iflip[t] || below;
      below_any = below_any || below;
    }
    flip = half_any(below_any);
    kr_publish<SLOTS>(tab, f, x, y, own);
    gradient();
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {
      const double kept = -pf[t];                  // :531
      pf[t] = pf[t] - dtf(t) * gf[t];              // :532, :535
      px[t] = px[t] - dtx(t) * gx[t];
      py[t] = py[t] - dty(t) * gy[t];
      if (flip && iflip[t]) pf[t] = kept;          // :533
    }
  }
  if (!flip) {
#pragma unroll
    for (int t = 0; t < SLOTS; ++t) {              // :551-552
      pf[t] = pf[t] + dtf(t) * gf[t] / 2.0;
      px[t] = px[t] + dtx(t) * gx[t] / 2.0;
      py[t] = py[t] + dty(t) * gy[t] / 2.0;
    }
  }
  return flip;
}

// Two chains per wave (32 lanes each), W waves per workgroup; two waves per
// SIMD (<= 256 VGPRs) except the fp64-image / K > 32 variant, which needs more.
// SOLVER: RHMC_SOLVER_IMPLICIT = RHMC_single_step (km_steps), else one of the
// explicit integrators (km_explicit_steps; f_pos = the flux wall).
// WS > 1 (implicit solver only: every wave of a workgroup calls the gradient
// equally often): groups of WS consecutive waves run the same two chains and
// split their windows (TiledRK::gradient), for launches with too few chains
// to fill the GPU (C5 split over 8 GPUs: 1024 chains per GPU); group g holds
// chains 2g, 2g + 1, and waves past the last chain mirror chain 0 rather
// than leave (the barrier counts them).
template <typename DT, int SLOTS, bool TAB, int SOLVER = RHMC_SOLVER_IMPLICIT, int WS = 1>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(sizeof(DT) == 8 && SLOTS == 2 ? 1 : 2)))
leapfrog_kr(LeapArgsKR a, int f_pos) {
  static_assert(WS == 1 || SOLVER == RHMC_SOLVER_IMPLICIT, "window split: implicit steps only");
  using TK = TiledRK<DT, SLOTS, TAB>;
  extern __shared__ double lds[];
  const DT* img;
  if constexpr (sizeof(DT) == sizeof(float)) img = reinterpret_cast<const DT*>(a.Df);
  else img = reinterpret_cast<const DT*>(a.D);
  exp_tab_fill(lds);
  if constexpr (TAB && kImgLds) {  // image after the factor tables (lds_bytes)
    const int nw = blockDim.x / kWave;
    DT* simg = reinterpret_cast<DT*>(
        lds + kExpTab + (size_t)nw * TK::CPW * TK::KMAX * (sizeof(KRStar) / 8) +
        (size_t)nw * TK::CPW * a.K * 2 * a.side);
    for (int e = threadIdx.x; e < a.side * a.side; e += blockDim.x) simg[e] = img[e];
    img = simg;
  }
  __syncthreads();
  const int64_t gwave = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  const int64_t wave = gwave / WS;      // the chain-pair group
  const int wsub = (int)(gwave % WS);   // this wave's share of the group's windows
  if (WS == 1 && TK::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int h = lane / TK::LPC, m = lane % TK::LPC;
  const int64_t chain = TK::CPW * wave + h;
  // ragged tail: mirror the wave's first chain; a whole group past the end
  // mirrors the first chain of its own workgroup (never past the end: the
  // workgroup's first group is real), whose write after the step loop the
  // workgroup's barriers order after this read; only wave 0 of a group writes
  // its real chains (after the loop)
  const int64_t chain_r =
      chain < a.n_chains ? chain
      : (TK::CPW * wave < a.n_chains
             ? TK::CPW * wave
             : TK::CPW * ((int64_t)blockIdx.x * (blockDim.x / kWave) / WS));
  const int64_t cbase = chain_r * 3 * (int64_t)a.K;
  const int W = blockDim.x / kWave;
  const int slot = (threadIdx.x / kWave) * TK::CPW + h;  // chain slot in the workgroup
  KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + slot * TK::KMAX;
  // TAB: the chain's factor tables; otherwise its deferred-sum buffer
  double* ftab = lds + kExpTab + (size_t)W * TK::CPW * TK::KMAX * (sizeof(KRStar) / 8) +
                 (TAB ? (size_t)slot * a.K * 2 * a.side : (size_t)slot * TK::RED_DOUBLES);
  // WS > 1: the group's two exchange buffers, after the tables / sum buffers
  double* xbuf = lds + TK::lds_bytes(W, a.K, a.side) / sizeof(double) +
                 (size_t)((threadIdx.x / kWave) / WS) * 2 * TK::CPW * TK::KMAX * 3;
  int xpar = 0;
  const Consts& c = a.c;
  const LeanConsts lc = lean_consts(c);
  const int K = a.K;

  double f[SLOTS], x[SLOTS], y[SLOTS], pf[SLOTS], px[SLOTS], py[SLOTS];
  bool own[SLOTS];
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    const int j = TK::LPC * t + m;
    own[t] = j < K;
    const int64_t e = cbase + 3 * (int64_t)(own[t] ? j : 0);
    f[t] = own[t] ? a.q[e] : 1.0;
    x[t] = own[t] ? a.q[e + 1] : 0.0;
    y[t] = own[t] ? a.q[e + 2] : 0.0;
    pf[t] = own[t] ? a.p[e] : 0.0;
    px[t] = own[t] ? a.p[e + 1] : 0.0;
    py[t] = own[t] ? a.p[e + 2] : 0.0;
  }
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  const int side = a.side;
  auto grad = [&](const double (&xs)[SLOTS], const double (&ys)[SLOTS], double (&gf)[SLOTS],
                  double (&gx)[SLOTS], double (&gy)[SLOTS]) {
    TK::template gradient<WS>(lds, img, side, tab, ftab, K, xs, ys, own, c, lc, gf, gx, gy,
                              wsub, xbuf + (size_t)xpar * TK::CPW * TK::KMAX * 3);
    xpar ^= 1;
  };
  if constexpr (SOLVER == RHMC_SOLVER_IMPLICIT) {
    km_steps<SLOTS>(f, x, y, pf, px, py, own, tab, a.n_steps, (double)(side - 1), c, lc, grad,
                    it_p, it_q, st);
  } else if constexpr (SOLVER == kSolverHmcRandom) {
    if (km_hmc_random_steps<SLOTS>(f, x, y, pf, px, py, own, tab, a.steps[chain_r], a.dtv, c,
                                   grad)) {
      st |= RHMC_STATUS_REFLECT_F;  // p_tmp stays the starting momentum (:547-550)
#pragma unroll
      for (int t = 0; t < SLOTS; ++t) {
        const int64_t e = cbase + 3 * (int64_t)(own[t] ? TK::LPC * t + m : 0);
        pf[t] = own[t] ? a.p[e] : 0.0;
        px[t] = own[t] ? a.p[e + 1] : 0.0;
        py[t] = own[t] ? a.p[e + 2] : 0.0;
      }
    }
  } else {
    km_explicit_steps<SOLVER, SLOTS>(f, x, y, pf, px, py, own, tab, a.n_steps, f_pos, c, lc,
                                     grad, st);
  }

  // the output indices again from a volatile lane id (held across the step
  // loop they cost registers the loop needs: the window-split variants spill)
  const int lo = lane_id_fresh(), mo = lo % TK::LPC;
  const int64_t chain_o = TK::CPW * wave + lo / TK::LPC;
  const bool real_o = chain_o < a.n_chains && wsub == 0;
  const int64_t cbase_o = chain_o * 3 * (int64_t)a.K;
  unsigned nf = 0u;
#pragma unroll
  for (int t = 0; t < SLOTS; ++t) {
    if (TK::LPC * t + mo >= K || !real_o) continue;
    if (!(isfinite(f[t]) && isfinite(x[t]) && isfinite(y[t]) && isfinite(pf[t]) &&
          isfinite(px[t]) && isfinite(py[t])))
      nf = RHMC_STATUS_NONFINITE;
    const int64_t e = cbase_o + 3 * (int64_t)(TK::LPC * t + mo);
    a.q[e] = f[t];
    a.q[e + 1] = x[t];
    a.q[e + 2] = y[t];
    a.p[e] = pf[t];
    a.p[e + 1] = px[t];
    a.p[e + 2] = py[t];
  }
  unsigned all = st | nf;
#pragma unroll
  for (int d = 16; d >= 1; d >>= 1) all |= (unsigned)__shfl_xor((int)all, d, kWave);
  if (mo == 0 && real_o) {
    if (a.status) a.status[chain_o] = (int32_t)all;
    if (a.fp_iters) {
      a.fp_iters[2 * chain_o] = it_p;
      a.fp_iters[2 * chain_o + 1] = it_q;
    }
  }
}

}  // namespace rhmc
