// rhmc_dense.hpp — the gradient and potential of MANY stars on a SMALL image
// (32 or 48 px; the reference's own many-star drivers: RHMC-big-sim3.py,
// K = 100, and RHMC-big-sim4.py, K up to N_max = 120, both on 32x32), for the
// slotted one-wave-per-chain kernels of rhmc_kernels.hip (star 64 s + lane in
// register slot s, K <= 256).
//
// On such an image every star's window covers most of the image, so the
// window-major kernels evaluate Lambda once per (pixel, window): ~K times per
// pixel.  Here, as the reference does (sampler_RHMC.py:373-406, full image):
//
//   pass 1 (pixel-major)  Lambda = B + sum_k f_k ex_k(i) ey_k(j), stars in
//       ascending order; lane (a, b) owns the BS x BS pixel block at rows
//       a BS.., columns b BS.. (BS = IMG / 8) with its accumulators in
//       registers; the separable PSF factors come from LDS tables of TK = 16
//       stars at a time (ex_k(i) and f_k ey_k(j) / (2 pi s^2), utils.py:475-486),
//       built by recurrence (runs of 8 entries from two exps, rhmc_pixk.hpp
//       tables_rec: within ~25 ulp of the direct exp).  One FMA per
//       pixel-star and 2 BS LDS reads per BS^2 FMAs.
//   pass 2   s = D / Lambda - 1 (:379), one v_rcp_f64 per four pixels,
//       written to the wave's LDS region (over the tables).
//   pass 3 (star-major)  lane = (star, row group): A0 = sum_ij ex(i) ey(j) s_ij,
//       A1 = sum_ij ex(i) (i + 1/2 - x) ey(j) s_ij, A2 likewise with
//       (j + 1/2 - y), by column chunks of 16: R_i = sum_j ey(j) s_ij,
//       C_j += ex(i) s_ij (s rows read as LDS broadcasts), the lane's own
//       factors by recurrence in registers.  Two FMAs per pixel-star; a star's
//       rows are split over G = 1, 2 or 4 lanes (dense_log2_groups: few stars
//       would leave most lanes idle) whose partial sums one or two quad DPP
//       adds combine.
//   dVdq = (-A0, -A1 f / var, -A2 f / var) (:404-406).
//
// Nothing is truncated (full image, any PSF width).
#pragma once
#include "rhmc_exp.hpp"
#include "rhmc_tiledr.hpp"
#include "rhmc_wave.hpp"
#include "rhmc_windowed.hpp"

namespace rhmc {

// gauss_run8: rhmc_windowed.hpp.

// Two adjacent doubles of LDS in one 16-byte read (ds_read_b128: 4 LDS cycles
// per wave-instruction at 256 B/clk/CU, where the two 8-byte reads the
// compiler forms without the alignment, ds_read2_b64, take 8 at 128 B/clk).
// Every such pair below starts on a 16-byte boundary (even double offsets).
__device__ __forceinline__ void lds_pair(const double* p, double& a, double& b) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  const v2d t = *reinterpret_cast<const v2d*>(p);
  a = t.x;
  b = t.y;
}

// Row groups per star in the dense kernel's pass 3 (log2): the G in {1, 2, 4}
// with the fewest row-units ceil(G K / 64) / G per lane, the smallest on a
// tie — K <= 16: 4 (a quarter of the rows per lane), K <= 32: 2, K = 100: 4
// (7 rounds of a quarter against 2 full rounds).
__host__ __device__ __forceinline__ int dense_log2_groups(int K) {
  int best = 0, best_cost = 4 * ((K + 63) / 64);
  for (int lg = 1; lg <= 2; ++lg) {
    const int cost = (4 >> lg) * (((K << lg) + 63) / 64);
    if (cost < best_cost) {
      best = lg;
      best_cost = cost;
    }
  }
  return best;
}

template <int IMG>
struct DenseG {
  static_assert(IMG == 32 || IMG == 48, "image side");
  static constexpr int BS = IMG / 8;    // pixel block side per lane (8 x 8 blocks)
  static constexpr int TK = 16;         // stars per factor-table tile (divides 64)
  static constexpr int CW = 16;         // pass-3 column chunk
  static constexpr int NCH = IMG / CW;
  // LDS bank spreading (64 banks of 4 bytes): the tile tables' rows are TP
  // doubles apart (a 16-byte multiple whose 16 rows start in 16 different bank
  // quads: 32 px 68 dwords = 4 mod 64, 48 px 100 = 36 mod 64), so the table
  // builder's stores (one row per lane) do not conflict; s is [IMG][IMG] with
  // the rows of pass-3 row group g shifted by 2 g doubles (16 g bytes), so
  // the G groups' simultaneous row reads hit different banks.
  static constexpr int TP = IMG + 2;
  // lds_pair's 16-byte alignment: every region and row offset an even double count
  static_assert(BS % 2 == 0 && TP % 2 == 0 && IMG % 2 == 0 && kExpTab % 2 == 0 && CW % 2 == 0,
                "16-byte LDS pairs");
  // per wave: the tile tables ex [TK][TP] + fey [TK][TP], later s (+ skews)
  static __host__ __device__ constexpr size_t wave_doubles() {
    return 2 * TK * TP > IMG * IMG + 8 ? (size_t)2 * TK * TP : (size_t)IMG * IMG + 8;
  }
  // LDS: exp table, the image (fp64, [IMG][IMG]), the waves' regions
  static_assert(wave_doubles() % 2 == 0, "16-byte LDS pairs");
  static __host__ __device__ constexpr size_t lds_bytes(int waves) {
    return (kExpTab + (size_t)IMG * IMG + (size_t)waves * wave_doubles()) * sizeof(double);
  }

  struct Ctx {
    const double* etab;
    const double* img;  // LDS [IMG][IMG]
    double* w;          // this wave's region
  };

  // Block-wide prologue (every thread of the block, before any early exit).
  static __device__ __forceinline__ Ctx setup(double* lds, const double* __restrict__ D, int,
                                              int, int, double* /*work*/) {
    exp_tab_fill(lds);
    double* img = lds + kExpTab;
    for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) img[e] = D[e];
    __syncthreads();
    Ctx g;
    g.etab = lds;
    g.img = img;
    g.w = lds + kExpTab + (size_t)IMG * IMG + (size_t)(threadIdx.x / kWave) * wave_doubles();
    return g;
  }

  // Slot s's register, s wave-uniform.
  template <int SLOTS>
  static __device__ __forceinline__ double pick(const double (&v)[SLOTS], int s) {
    double r = v[0];
#pragma unroll
    for (int t = 1; t < SLOTS; ++t) r = (s == t) ? v[t] : r;
    return r;
  }

  // Pass 1: Lambda over the lane's pixel block (:373-376).  Ends with the
  // tables read: the caller may overwrite the wave's region after a sync.
  template <int SLOTS>
  static __device__ __forceinline__ void lambda(const Ctx& g, int K, const double (&f)[SLOTS],
                                                const double (&x)[SLOTS],
                                                const double (&y)[SLOTS], const Consts& c,
                                                const LeanConsts& lc, double (&lam)[BS * BS]) {
    const int lane = lane_id();
    const int a = lane >> 3, b = lane & 7;
#pragma unroll
    for (int u = 0; u < BS * BS; ++u) lam[u] = c.B;
    double* ext = g.w;              // [TK][TP]
    double* fyt = g.w + TK * TP;    // [TK][TP]
    // table builder: lane -> (row rr = lane / 2: star rr % 16, axis rr / 16;
    // half h = lane % 2 of the entries)
    const int rr = lane >> 1, h = lane & 1;
    const int rs = rr & (TK - 1), axis = rr >> 4;
    constexpr int HALF = IMG / 2;
    for (int k0 = 0; k0 < K; k0 += TK) {  // wave-uniform
      const int s = k0 / kWave;
      const int src = (k0 & (kWave - 1)) + rs;
      const double xs = __shfl(pick<SLOTS>(x, s), src, kWave);
      const double ys = __shfl(pick<SLOTS>(y, s), src, kWave);
      const double fs = __shfl(pick<SLOTS>(f, s), src, kWave);
      const double ctr = axis ? ys : xs;
      const double scale = axis ? fs * lc.inv_norm : 1.0;
      double* dst = (axis ? fyt : ext) + rs * TP + h * HALF;
      wave_lds_sync();  // the previous tile's reads are done
#pragma unroll
      for (int r0 = 0; r0 < HALF; r0 += 8) {
        double e[8];
        gauss_run8(((double)(h * HALF + r0) + 0.5) - ctr, scale, g.etab, lc, e);
#pragma unroll
        for (int l = 0; l < 8; ++l) dst[r0 + l] = e[l];
      }
      wave_lds_sync();
      const int nk = min(TK, K - k0);
      for (int r = 0; r < nk; ++r) {  // stars in ascending order
        double ex[BS], fy[BS];
#pragma unroll
        for (int u = 0; u < BS; u += 2) lds_pair(ext + r * TP + a * BS + u, ex[u], ex[u + 1]);
#pragma unroll
        for (int v = 0; v < BS; v += 2) lds_pair(fyt + r * TP + b * BS + v, fy[v], fy[v + 1]);
#pragma unroll
        for (int u = 0; u < BS; ++u)
#pragma unroll
          for (int v = 0; v < BS; ++v) lam[u * BS + v] = fma(ex[u], fy[v], lam[u * BS + v]);
      }
    }
    wave_lds_sync();  // every lane is done with the tables
  }

  // dVdq (+ the dphidq metric term) of the chain; lane l gets star 64 s + l's
  // in slot s (sampler_RHMC.py:365-425, :448-465).
  template <int SLOTS>
  static __device__ __forceinline__ void gradient(const Ctx& g, int K, const double (&f)[SLOTS],
                                                  const double (&x)[SLOTS],
                                                  const double (&y)[SLOTS], const Consts& c,
                                                  const LeanConsts& lc, bool with_metric,
                                                  double (&gf)[SLOTS], double (&gx)[SLOTS],
                                                  double (&gy)[SLOTS]) {
    const int lgG = dense_log2_groups(K);
    const int rows = IMG >> lgG;
    {
      const int lane = lane_id();
      double lam[BS * BS];
      lambda<SLOTS>(g, K, f, x, y, c, lc, lam);
      // pass 2: s = D / Lambda - 1 (:379) into the wave's region
      const int a = lane >> 3, b = lane & 7;
#pragma unroll
      for (int u = 0; u < BS; ++u) {
        const int i = a * BS + u;
        const double* drow = g.img + i * IMG + b * BS;
        double* srow = g.w + i * IMG + 2 * (i / rows) + b * BS;
#pragma unroll
        for (int v = 0; v < BS; v += 2) {
          const double l0 = lam[u * BS + v], l1 = lam[u * BS + v + 1];
          const double r = rcp_nr1(l0 * l1);
          double d0, d1;
          lds_pair(drow + v, d0, d1);
          srow[v] = fma(d0, l1 * r, -1.0);
          srow[v + 1] = fma(d1, l0 * r, -1.0);
        }
      }
    }
    wave_lds_sync();
    // pass 3: work item t = 64 r + lane of round r is (star t / G, row group
    // t % G); the G lanes of a star sum their partial A0, A1, A2 (quad DPP)
    // and the star's owner lane (64 s + l in slot s) reads them.
    const int lane = lane_id();
    const int G = 1 << lgG;
    const int rounds = (K * G + kWave - 1) / kWave;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) gf[s] = gx[s] = gy[s] = 0.0;
    for (int r = 0; r < rounds; ++r) {  // wave-uniform
      const int k0 = (kWave * r) >> lgG;             // the round's first star
      const int ks = k0 / kWave;                      // its slot (64 / G divides 64)
      const int t = kWave * r + lane;
      const int src = (t >> lgG) & (kWave - 1);
      const int ib = (t & (G - 1)) * rows;            // the item's first row
      const double* sbase = g.w + 2 * (t & (G - 1));  // the row group's skew
      const double xs = __shfl(pick<SLOTS>(x, ks), src, kWave);
      const double ys = __shfl(pick<SLOTS>(y, ks), src, kWave);
      double A0 = 0.0, A1 = 0.0, A2 = 0.0;
#pragma unroll 1
      for (int ch = 0; ch < NCH; ++ch) {
        const int j0 = ch * CW;
        double ey[CW], C[CW];
        {
          double e[8];
          gauss_run8(((double)j0 + 0.5) - ys, lc.inv_norm, g.etab, lc, e);
#pragma unroll
          for (int l = 0; l < 8; ++l) ey[l] = e[l];
          gauss_run8(((double)(j0 + 8) + 0.5) - ys, lc.inv_norm, g.etab, lc, e);
#pragma unroll
          for (int l = 0; l < 8; ++l) ey[8 + l] = e[l];
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) C[j] = 0.0;
#pragma unroll 1
        for (int di = 0; di < rows; di += 8) {       // rows: wave-uniform
          const int i0 = ib + di;
          double ex[8];
          gauss_run8(((double)i0 + 0.5) - xs, 1.0, g.etab, lc, ex);
#pragma unroll
          for (int l = 0; l < 8; ++l) {
            if (di + l >= rows) break;                 // wave-uniform (48 px, G = 4)
            const double* sr = sbase + (i0 + l) * IMG + j0;  // G distinct rows: broadcasts
            double r0 = 0.0, r1 = 0.0;
#pragma unroll
            for (int j = 0; j < CW; j += 2) {
              double s0, s1;
              lds_pair(sr + j, s0, s1);
              r0 = fma(ey[j], s0, r0);
              r1 = fma(ey[j + 1], s1, r1);
              C[j] = fma(ex[l], s0, C[j]);
              C[j + 1] = fma(ex[l], s1, C[j + 1]);
            }
            const double R = r0 + r1;
            const double wi = ((double)(i0 + l) - xs) + 0.5;
            A0 = fma(ex[l], R, A0);
            A1 = fma(ex[l] * wi, R, A1);
          }
        }
#pragma unroll
        for (int j = 0; j < CW; ++j) A2 = fma(ey[j] * (((double)(j0 + j) - ys) + 0.5), C[j], A2);
      }
      if (lgG >= 1) {  // sum over the star's G lanes (every lane gets the same bits)
        A0 += dpp_move<0xB1>(A0);
        A1 += dpp_move<0xB1>(A1);
        A2 += dpp_move<0xB1>(A2);
      }
      if (lgG >= 2) {
        A0 += dpp_move<0x4E>(A0);
        A1 += dpp_move<0x4E>(A1);
        A2 += dpp_move<0x4E>(A2);
      }
      // owner lanes of the round's stars: k0 % 64 <= lane < k0 % 64 + 64 / G
      const int rel = lane - (k0 & (kWave - 1));
      const bool mine = rel >= 0 && rel < (kWave >> lgG) && k0 + rel < K;
      const int from = mine ? rel << lgG : lane;
      const double a0 = __shfl(A0, from, kWave), a1 = __shfl(A1, from, kWave),
                   a2 = __shfl(A2, from, kWave);
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (s == ks && mine) {
          gf[s] = -a0;                        // :404
          gx[s] = -a1 * f[s] * lc.inv_var;    // :405
          gy[s] = -a2 * f[s] * lc.inv_var;    // :406
        }
      }
    }
    wave_lds_sync();  // s is read; the next gradient's tables may overwrite it
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      if (c.use_prior) gf[s] += c.alpha / f[s];               // :408-409
      if (with_metric) gf[s] += metric_flux_term(f[s], c);    // :459-463
    }
    if (c.use_Vc) vc_gradient<SLOTS>(K, x, y, c, gx, gy);     // :411-418
  }

  // sum over the image of Lambda - D ln Lambda (:322-328); every lane gets it.
  template <int SLOTS>
  static __device__ __forceinline__ double potential(const Ctx& g, int K,
                                                     const double (&f)[SLOTS],
                                                     const double (&x)[SLOTS],
                                                     const double (&y)[SLOTS], const Consts& c,
                                                     const LeanConsts& lc) {
    const int lane = lane_id();
    const int a = lane >> 3, b = lane & 7;
    double lam[BS * BS];
    lambda<SLOTS>(g, K, f, x, y, c, lc, lam);
    double v = 0.0;
#pragma unroll
    for (int u = 0; u < BS; ++u)
#pragma unroll
      for (int w = 0; w < BS; ++w)
        v += lam[u * BS + w] - g.img[(a * BS + u) * IMG + b * BS + w] * log(lam[u * BS + w]);
    return wave_sum_dpp(v);
  }
};

}  // namespace rhmc
