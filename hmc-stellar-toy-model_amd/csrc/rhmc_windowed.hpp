// rhmc_windowed.hpp — the catch-all path: any square image, 1 <= K <= 1024
// stars per chain (lanes = stars, SLOTS stars per lane).
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
// Stars.  One wave per chain; star k lives in lane k % 64, register slot
// k / 64 (SLOTS = 1, 2, 4: K <= 64, 128, 256 — the reference takes any
// 3 * Nobjs, and its own drivers run K = 100 and grow K to N_max = 120 by
// births: RHMC-big-sim3.py:18-19, RHMC-big-sim4.py:77).  From 65 stars the
// launcher takes WinGG below (the tables in global memory: LDS-sized tables
// cap a CU at one or two waves); beyond 256 stars (SLOTS = 8, 16: K <= 512,
// 1024) the register states spill to scratch — a completeness path.
//
// Gradient, star-major: for star k (wave-uniform), lane (r = l>>5, c = l&31)
// owns window column c and rows r, r+2, .., r+30 (16 pixels); Lambda at those
// pixels sums over the stars whose windows overlap star k's window (one ballot
// per slot: wave-uniform 64-bit masks), in ascending star order like the
// reference; one division per pixel; three wave sums per star.
// D stays in global memory (512 KB at 256x256, L2-resident and shared by all
// chains).  Per-wave LDS: windowed PSF factor tables, 2 x K x 33 doubles.
#pragma once
#include "rhmc_exp.hpp"
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

// The wave's table writes visible to its own later reads: LDS tables need
// only the wavefront-scope ordering; tables in global memory (GT) a
// workgroup-scope fence, which waits for the stores.
template <bool GT>
__device__ __forceinline__ void tab_sync() {
  if constexpr (GT) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  } else {
    wave_lds_sync();
  }
}

// Diagnostic build (-DRHMC_TABLE_CANARY, never the product library): each
// wave's global table region starts with a 64-bit counter to which lane 0 adds
// the call's tag when a gradient (tag 1) or potential (tag 2^32) starts and
// again when it ends; anything else that bumped it in between (another call
// in the same region at the same time) is counted in g_tab_conflicts:
// [0] calls that saw a bump, [1] / [2] gradients / potentials that saw one,
// [3] / [4] the gradient / potential bumps they saw (enter + leave of every
// foreign call); rhmc_debug_table_conflicts() reads them.  Other writers
// (not tagged) show as a bump of neither kind.
#ifdef RHMC_TABLE_CANARY
#ifndef RHMC_TABLE_DIAG
#define RHMC_TABLE_DIAG 1  // the pool modes of RHMC_OPT_TABLES
#endif
constexpr int kTabHeader = 8;  // doubles before a wave's tables
__device__ unsigned long long g_tab_conflicts[6];
__device__ unsigned long long g_tab_seen[9];  // [0] count, then the first 8 foreign header values
__device__ __forceinline__ unsigned long long canary_enter(double* hdr, int kind) {
  unsigned long long v = 0;
  const unsigned long long tag = kind == 1 ? 1ull : (1ull << 32);
  if (lane_id() == 0) v = atomicAdd((unsigned long long*)hdr, tag);
  return v;
}
__device__ __forceinline__ void canary_leave(double* hdr, unsigned long long v, int kind) {
  if (lane_id() == 0) {
    const unsigned long long tag = kind == 1 ? 1ull : (1ull << 32);
    const unsigned long long now = atomicAdd((unsigned long long*)hdr, tag);
    if (now != v + tag) {
      const unsigned long long d = now - (v + tag);
      atomicAdd(&g_tab_conflicts[0], 1ull);
      atomicAdd(&g_tab_conflicts[kind], 1ull);
      atomicAdd(&g_tab_conflicts[3], d & 0xffffffffull);
      atomicAdd(&g_tab_conflicts[4], d >> 32);
      const unsigned long long slot = atomicAdd(&g_tab_seen[0], 1ull);
      if (slot < 8ull) atomicExch(&g_tab_seen[1 + slot], now);
    }
  }
}
#else
constexpr int kTabHeader = 0;
#endif

// Does lane `lane` hold a star in slot t?
__device__ __forceinline__ bool win_own(int t, int K) { return kWave * t + lane_id() < K; }

// Windowed PSF factor tables for K stars (star 64 t + l in lane l, slot t);
// the entries of a slot are flattened over (star, axis, index) so all 64 lanes
// work.
template <int SLOTS, bool GT = false>
__device__ __forceinline__ void win_build_tables(const WinTables& t, int K,
                                                 const double (&x)[SLOTS],
                                                 const double (&y)[SLOTS], const int (&bx)[SLOTS],
                                                 const int (&by)[SLOTS], const LeanConsts& lc) {
  const int lane = lane_id();
  const int per_star = 2 * kTabW;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int k0 = kWave * s;
    if (k0 >= K) break;  // wave-uniform
    const int Ks = min(kWave, K - k0);
    const int total = Ks * per_star;
    const int iters = (total + kWave - 1) / kWave;
    for (int m = 0; m < iters; ++m) {  // uniform trip count: shuffles see all lanes
      const int e = lane + kWave * m;
      const int kl = min(e / per_star, Ks - 1);
      const double xk = __shfl(x[s], kl, kWave), yk = __shfl(y[s], kl, kWave);
      const int bxk = __shfl(bx[s], kl, kWave), byk = __shfl(by[s], kl, kWave);
      if (e < total) {
        const int r = e - kl * per_star;
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
        (axis == 0 ? t.ex : t.ey)[(k0 + kl) * kTabW + d] = val;
      }
    }
  }
  tab_sync<GT>();
}

// Repulsion gradient (sampler_RHMC.py:411-418), lanes = stars: every star of
// slot s sums over all K stars in ascending order.
template <int SLOTS>
__device__ __forceinline__ void vc_gradient(int K, const double (&x)[SLOTS],
                                            const double (&y)[SLOTS], const Consts& c,
                                            double (&gx)[SLOTS], double (&gy)[SLOTS]) {
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    double sx = 0.0, sy = 0.0;
#pragma unroll
    for (int s2 = 0; s2 < SLOTS; ++s2) {
      for (int jl = 0; jl < kWave && kWave * s2 + jl < K; ++jl) {
        const double X = bcast(x[s2], jl), Y = bcast(y[s2], jl);
        const double ddx = X - x[s], ddy = Y - y[s];
        double R = sqrt(ddx * ddx + ddy * ddy);
        if (fabs(R) < 1e-10) R = 1e32;
        const double tr = pow(1.0 / R, c.vc_pow + 2.0);
        sx += tr * ddx;
        sy += tr * ddy;
      }
    }
    gx[s] += c.beta * sx * c.vc_pow;
    gy[s] += c.beta * sy * c.vc_pow;
  }
}

// dVdq (+ dphidq metric term) of the wave's chain; lane l gets star 64 s + l's
// in slot s.
template <int SLOTS, bool GT = false>
__device__ void win_gradient(const double* __restrict__ D, const WinTables& t, int K,
                             const double (&f)[SLOTS], const double (&x)[SLOTS],
                             const double (&y)[SLOTS], int rows, int cols, const Consts& c,
                             const LeanConsts& lc, bool with_metric, double (&gf)[SLOTS],
                             double (&gx)[SLOTS], double (&gy)[SLOTS]) {
  const int lane = lane_id();
#ifdef RHMC_TABLE_CANARY
  const unsigned long long cv = GT ? canary_enter(t.ex - kTabHeader, 1) : 0ull;
#endif
  int bx[SLOTS], by[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    bx[s] = win_base(x[s]);
    by[s] = win_base(y[s]);
    gf[s] = gx[s] = gy[s] = 0.0;
  }
  win_build_tables<SLOTS, GT>(t, K, x, y, bx, by, lc);
  const int lrow = lane >> 5, lcol = lane & 31;

#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    for (int kl = 0; kl < kWave; ++kl) {
      const int k = kWave * s + kl;
      if (k >= K) break;  // wave-uniform
      const double xk = bcast(x[s], kl), fk = bcast(f[s], kl);
      const int bxk = readlane_i(bx[s], kl), byk = readlane_i(by[s], kl);
      const int j = byk + lcol;
      const bool colok = (unsigned)j < (unsigned)cols;

      double lam[16], psk[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        lam[u] = c.B;
        psk[u] = 0.0;
      }
      // Lambda = B + sum_{stars overlapping this window} f PSF, ascending order (:373-376)
#pragma unroll
      for (int s2 = 0; s2 < SLOTS; ++s2) {
        const bool ov = win_own(s2, K) && abs(bx[s2] - bxk) < kWin && abs(by[s2] - byk) < kWin;
        unsigned long long mm = __builtin_amdgcn_ballot_w64(ov);
        while (mm) {
          const int kl2 = __builtin_ctzll(mm);
          mm &= mm - 1;
          const int kk = kWave * s2 + kl2;
          const double fkk = bcast(f[s2], kl2);
          const int bxkk = readlane_i(bx[s2], kl2), bykk = readlane_i(by[s2], kl2);
          const unsigned v = min((unsigned)(j - bykk), (unsigned)kWin);
          const double eyv = t.ey[kk * kTabW + v];
          const double* exrow = t.ex + kk * kTabW;
          const int u0 = bxk + lrow - bxkk;
          if (kk == k) {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const unsigned uu = min((unsigned)(u0 + 2 * u), (unsigned)kWin);
              const double p = exrow[uu] * eyv;
              psk[u] = p;
              lam[u] = fma(fkk, p, lam[u]);
            }
          } else {
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const unsigned uu = min((unsigned)(u0 + 2 * u), (unsigned)kWin);
              lam[u] = fma(fkk, exrow[uu] * eyv, lam[u]);
            }
          }
        }
      }
      // rho * PSF_k and its three moments over this lane's 16 pixels
      double a0 = 0.0, a1 = 0.0;
#pragma unroll
      for (int u = 0; u < 16; u += 2) {
        const int i1 = bxk + lrow + 2 * u, i2 = i1 + 2;
        const bool ok1 = colok && (unsigned)i1 < (unsigned)rows;
        const bool ok2 = colok && (unsigned)i2 < (unsigned)rows;
        const double d1 = ok1 ? D[(size_t)i1 * cols + j] : 0.0;
        const double d2 = ok2 ? D[(size_t)i2 * cols + j] : 0.0;
        const double l1 = lam[u], l2 = lam[u + 1];
        const double L = l1 * l2;
        double r = __builtin_amdgcn_rcp(L);
        r = fma(r, fma(-L, r, 1.0), r);
        const double r1 = l2 * r, r2 = l1 * r;
        double q1 = d1 * r1, q2 = d2 * r2;
        q1 = fma(r1, fma(-l1, q1, d1), q1);
        q2 = fma(r2, fma(-l2, q2, d2), q2);
        const double p1 = ok1 ? psk[u] : 0.0, p2 = ok2 ? psk[u + 1] : 0.0;
        const double w1 = fma(p1, q1, -p1), w2 = fma(p2, q2, -p2);
        a0 += w1;
        a1 = fma(w1, ((double)i1 - xk) + 0.5, a1);
        a0 += w2;
        a1 = fma(w2, ((double)i2 - xk) + 0.5, a1);
      }
      const double yk = bcast(y[s], kl);
      const double a2 = a0 * (((double)j - yk) + 0.5);  // the lane's column is fixed
      const double s0 = wave_sum_dpp(a0);
      const double s1 = wave_sum_dpp(a1);
      const double s2v = wave_sum_dpp(a2);
      if (lane == kl) {
        gf[s] = -s0;                      // :404
        gx[s] = -s1 * fk * lc.inv_var;    // :405
        gy[s] = -s2v * fk * lc.inv_var;   // :406
      }
    }
  }
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    if (c.use_prior) gf[s] += c.alpha / f[s];               // :408-409
    if (with_metric) gf[s] += metric_flux_term(f[s], c);    // :459-463
  }
  if (c.use_Vc) vc_gradient<SLOTS>(K, x, y, c, gx, gy);     // :411-418
  tab_sync<GT>();
#ifdef RHMC_TABLE_CANARY
  if (GT) canary_leave(t.ex - kTabHeader, cv, 1);
#endif
}

// Column factor tables only (the potential's; the row factors are per-row
// scalars there): ey [K][kTabW], flattened over (star, index) like
// win_build_tables.
template <int SLOTS, bool GT = false>
__device__ __forceinline__ void win_build_ey(double* ey, int K, const double (&y)[SLOTS],
                                             const int (&by)[SLOTS], const LeanConsts& lc) {
  const int lane = lane_id();
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int k0 = kWave * s;
    if (k0 >= K) break;  // wave-uniform
    const int Ks = min(kWave, K - k0);
    const int total = Ks * kTabW;
    const int iters = (total + kWave - 1) / kWave;
    for (int m = 0; m < iters; ++m) {  // uniform trip count: shuffles see all lanes
      const int e = lane + kWave * m;
      const int kl = min(e / kTabW, Ks - 1);
      const double yk = __shfl(y[s], kl, kWave);
      const int byk = __shfl(by[s], kl, kWave);
      if (e < total) {
        const int d = e - kl * kTabW;
        double val = 0.0;
        if (d < kWin) {
          const double v = ((double)(byk + d) + 0.5) - yk;
          val = exp(-(v * v) * lc.inv_two_sig2) * lc.inv_norm;
        }
        ey[(k0 + kl) * kTabW + d] = val;
      }
    }
  }
  tab_sync<GT>();
}

// e[l] = exp(-c (v0 + l)^2), l < 8: by recurrence from two exps when v0 is
// within the recurrence's range (e(v + 1) = e(v) g(v), g(v + 1) = g(v) e^-2c,
// g(v) = exp(-c (2 v + 1)); Consts::rec_vmax), else eight direct exps (a far
// or NaN star: a per-lane branch).  Scaled by `scale`.
__device__ __forceinline__ void gauss_run8(double v0, double scale, const double* __restrict__ etab,
                                           const LeanConsts& lc, double (&e)[8]) {
  const double c = lc.inv_two_sig2;
  if (fabs(v0) < lc.rec_vmax) {
    double ev = exp_neg(-(v0 * v0) * c, etab) * scale;
    double g = exp_neg(-fma(2.0, v0, 1.0) * c, etab);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      e[l] = ev;
      ev = ev * g;
      g = g * lc.k_row;
    }
  } else {
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const double v = v0 + (double)l;
      e[l] = exp_neg(-(v * v) * c, etab) * scale;
    }
  }
}

// V of the wave's chain on a large image (sampler_RHMC.py:294-351), pixel-major
// in groups of kPotRows image rows (uniform) with lanes over columns in blocks
// of 64.  Only the stars whose window rows meet the group and whose window
// columns reach the block contribute (one ballot per slot for each): one
// column-factor load from the ey table per (star, block) serves all rows of
// the group, the row factors f ex(i) being per-row scalars of the star's lane
// (gauss_run8's recurrence from two table exps, zero outside its window
// rows).  A block no star reaches has Lambda == B exactly (the window bound)
// and adds B - D ln B per pixel without a log.  ln by log_pos (rhmc_exp.hpp:
// within 2 ulp, ~25 VALU).
constexpr int kPotRows = 8;  // a multiple of 8 (gauss_run8)

template <int SLOTS, bool GT = false>
__device__ double win_potential(const double* __restrict__ D, double* ey,
                                const double* __restrict__ etab, int K,
                                const double (&f)[SLOTS], const double (&x)[SLOTS],
                                const double (&y)[SLOTS], int rows, int cols, const Consts& c,
                                const LeanConsts& lc) {
  constexpr int R = kPotRows;
  const int lane = lane_id();
#ifdef RHMC_TABLE_CANARY
  const unsigned long long cv = GT ? canary_enter(ey - kTabHeader, 2) : 0ull;
#endif
  int bx[SLOTS], by[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    bx[s] = win_base(x[s]);
    by[s] = win_base(y[s]);
  }
  win_build_ey<SLOTS, GT>(ey, K, y, by, lc);
  const double lnB = log_pos(c.B);
  double v = 0.0;
  for (int i0 = 0; i0 < rows; i0 += R) {
    unsigned long long rm[SLOTS];
    double fex[SLOTS][R];
    bool any_row = false;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const bool meet = win_own(s, K) && bx[s] < i0 + R && i0 < bx[s] + kWin;
      rm[s] = __builtin_amdgcn_ballot_w64(meet);
      any_row = any_row || rm[s] != 0ull;
#pragma unroll
      for (int r = 0; r < R; ++r) fex[s][r] = 0.0;
      if (meet) {  // per lane: the star's f ex(i) on the group's window rows
#pragma unroll
        for (int h = 0; h < R; h += 8) {
          double e[8];
          gauss_run8(((double)(i0 + h) + 0.5) - x[s], f[s], etab, lc, e);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int i = i0 + h + r;
            fex[s][h + r] = (bx[s] <= i && i < bx[s] + kWin) ? e[r] : 0.0;
          }
        }
      }
    }
    const int nr = min(R, rows - i0);
    for (int cb = 0; cb < cols; cb += kWave) {
      const int j = cb + lane;
      const bool jin = j < cols;
      unsigned long long bm[SLOTS];
      bool any = false;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        bm[s] = any_row ? rm[s] & __builtin_amdgcn_ballot_w64(by[s] < cb + kWave &&
                                                                by[s] + kWin > cb)
                        : 0ull;
        any = any || bm[s] != 0ull;
      }
      double d[R];
#pragma unroll
      for (int r = 0; r < R; ++r)
        d[r] = (jin && r < nr) ? D[(size_t)(i0 + r) * cols + j] : 0.0;
      if (!any) {  // wave-uniform: Lambda == B on the whole block
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (jin && r < nr) v += c.B - d[r] * lnB;
        continue;
      }
      double lam[R];
#pragma unroll
      for (int r = 0; r < R; ++r) lam[r] = c.B;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        unsigned long long mm = bm[s];
        while (mm) {
          const int kl = __builtin_ctzll(mm);
          mm &= mm - 1;
          const int kk = kWave * s + kl;
          const unsigned vv = min((unsigned)(j - readlane_i(by[s], kl)), (unsigned)kWin);
          const double e = ey[kk * kTabW + vv];
#pragma unroll
          for (int r = 0; r < R; ++r) lam[r] = fma(bcast(fex[s][r], kl), e, lam[r]);
        }
      }
      // The R rows' logs unconditionally (lam is finite on masked rows), so
      // their independent chains interleave; masked terms dropped by select.
      double lg[R];
#pragma unroll
      for (int r = 0; r < R; ++r) lg[r] = log_pos(lam[r]);
#pragma unroll
      for (int r = 0; r < R; ++r)
        v += (jin && r < nr) ? lam[r] - d[r] * lg[r] : 0.0;
    }
  }
  tab_sync<GT>();
#ifdef RHMC_TABLE_CANARY
  if (GT) canary_leave(ey - kTabHeader, cv, 2);
#endif
  return wave_sum_dpp(v);
}

// Gradient policy of the slotted kernels (rhmc_kernels.hip) on windowed
// tables: any square image, D read from global memory (L2).
struct WinG {
  static __host__ __device__ size_t lds_bytes(int waves, int K) {
    return (kExpTab + (size_t)waves * win_table_doubles(K)) * sizeof(double);
  }
  struct Ctx {
    WinTables tab;
    const double* etab;
    const double* D;
    int rows, cols;
  };
  static __device__ __forceinline__ Ctx setup(double* lds, const double* D, int K, int rows,
                                              int cols, double* /*work*/) {
    exp_tab_fill(lds);
    __syncthreads();
    double* base = lds + kExpTab + (threadIdx.x / kWave) * win_table_doubles(K);
    Ctx g;
    g.etab = lds;
    g.tab = WinTables{base, base + K * kTabW};
    g.D = D;
    g.rows = rows;
    g.cols = cols;
    return g;
  }
  template <int SLOTS>
  static __device__ __forceinline__ void gradient(const Ctx& g, int K, const double (&f)[SLOTS],
                                                  const double (&x)[SLOTS],
                                                  const double (&y)[SLOTS], const Consts& c,
                                                  const LeanConsts& lc, bool with_metric,
                                                  double (&gf)[SLOTS], double (&gx)[SLOTS],
                                                  double (&gy)[SLOTS]) {
    win_gradient<SLOTS>(g.D, g.tab, K, f, x, y, g.rows, g.cols, c, lc, with_metric, gf, gx, gy);
  }
  template <int SLOTS>
  static __device__ __forceinline__ double potential(const Ctx& g, int K,
                                                     const double (&f)[SLOTS],
                                                     const double (&x)[SLOTS],
                                                     const double (&y)[SLOTS], const Consts& c,
                                                     const LeanConsts& lc) {
    return win_potential<SLOTS>(g.D, g.tab.ex, g.etab, K, f, x, y, g.rows, g.cols, c, lc);
  }
};

// The potential-only policy of the energy kernel on windowed tables: the
// column tables alone (K x 33 doubles per wave, half WinG's), so twice the
// waves fit a CU (C5: 2 per SIMD instead of 1).
struct WinEG {
  static __host__ __device__ size_t lds_bytes(int waves, int K) {
    return (kExpTab + (size_t)waves * K * kTabW) * sizeof(double);
  }
  struct Ctx {
    double* ey;
    const double* etab;
    const double* D;
    int rows, cols;
  };
  static __device__ __forceinline__ Ctx setup(double* lds, const double* D, int K, int rows,
                                              int cols, double* /*work*/) {
    exp_tab_fill(lds);
    __syncthreads();
    Ctx g;
    g.etab = lds;
    g.ey = lds + kExpTab + (threadIdx.x / kWave) * (size_t)K * kTabW;
    g.D = D;
    g.rows = rows;
    g.cols = cols;
    return g;
  }
  template <int SLOTS>
  static __device__ __forceinline__ double potential(const Ctx& g, int K,
                                                     const double (&f)[SLOTS],
                                                     const double (&x)[SLOTS],
                                                     const double (&y)[SLOTS], const Consts& c,
                                                     const LeanConsts& lc) {
    return win_potential<SLOTS>(g.D, g.ey, g.etab, K, f, x, y, g.rows, g.cols, c, lc);
  }
};

// From 65 stars on the windowed path (SLOTS 2 / 4 / 8 / 16): WinG's gradient
// and potential with each chain's factor tables in global memory — work +
// (launch wave) x 2 K 33 doubles, 0.5 MB per chain at K = 1024, allocated by
// the launcher on the launch's stream (Geometry::work) — and only the exp
// table in LDS, so four waves share a workgroup (1.3-1.8x the LDS-table
// kernel from 100 to 200 stars).  Past 256 stars the state spills.
struct WinGG {
  static __host__ __device__ size_t lds_bytes(int, int) { return kExpTab * sizeof(double); }
  static __host__ __device__ size_t work_doubles(int K) {
    return win_table_doubles(K) + kTabHeader;
  }
  using Ctx = WinG::Ctx;
  static __device__ __forceinline__ Ctx setup(double* lds, const double* D, int K, int rows,
                                              int cols, double* work) {
    exp_tab_fill(lds);
    __syncthreads();
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    double* base = work + wave * (int64_t)work_doubles(K) + kTabHeader;
    Ctx g;
    g.etab = lds;
    g.tab = WinTables{base, base + K * kTabW};
    g.D = D;
    g.rows = rows;
    g.cols = cols;
    return g;
  }
  template <int SLOTS>
  static __device__ __forceinline__ void gradient(const Ctx& g, int K, const double (&f)[SLOTS],
                                                  const double (&x)[SLOTS],
                                                  const double (&y)[SLOTS], const Consts& c,
                                                  const LeanConsts& lc, bool with_metric,
                                                  double (&gf)[SLOTS], double (&gx)[SLOTS],
                                                  double (&gy)[SLOTS]) {
    win_gradient<SLOTS, true>(g.D, g.tab, K, f, x, y, g.rows, g.cols, c, lc, with_metric, gf, gx,
                              gy);
  }
  template <int SLOTS>
  static __device__ __forceinline__ double potential(const Ctx& g, int K,
                                                     const double (&f)[SLOTS],
                                                     const double (&x)[SLOTS],
                                                     const double (&y)[SLOTS], const Consts& c,
                                                     const LeanConsts& lc) {
    return win_potential<SLOTS, true>(g.D, g.tab.ex, g.etab, K, f, x, y, g.rows, g.cols, c, lc);
  }
};

}  // namespace rhmc
