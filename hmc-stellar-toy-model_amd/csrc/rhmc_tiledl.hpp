// rhmc_tiledl.hpp — single-star leapfrog for LARGE chain counts: LPC = 1 or 4
// lanes per chain (64 / 16 chains per wave64), every chain on its own
// WIN x WIN pixel window (the window and the 2^-62 truncation bound of the
// register-window kernel, rhmc_tiledr.hpp), pixels read from the workgroup's
// LDS copy of the image.
//
// Why: the register-window kernel spreads one chain over 16 lanes, so the
// step's serial part (kicks, both fixed-point loops, the flux metric) and the
// PSF factor exchange run replicated on all 16 lanes — over half of its VALU
// instructions (profiles/pmc_c2.json).  With 4096 chains there is no other way
// to fill 1024 SIMDs.  With >= 64 Ki chains per GPU (C4: 2^20 over 8 GPUs)
// there is: LPC lanes per chain shrink the replicated share 16/LPC times while
// the pixel work (~8 VALU per pixel, 784 pixels) stays the same.
//
// Lane g of a chain's group owns window rows g, g + LPC, ...  Every lane
// evaluates all WIN column factors ey_j and ew_j = ey_j (c0 + j + 1/2 - y), so
// a row costs one exp (its row factor ex_i) and the pixel loop keeps two
// running sums per row,
//   R_i = sum_j ey_j s_ij,  Ry_i = sum_j ew_j s_ij,   s = D/Lambda - 1,
// with one v_rcp_f64 + Newton step per pixel pair (as rhmc_tiledr.hpp).  Then
//   s0 = sum_i ex_i R_i,  s1 = sum_i ex_i (r0 + i + 1/2 - x) R_i,
//   s2 = sum_i ex_i Ry_i,
// summed over the group's LPC lanes with DPP.
//
// LDS image layout: 16-byte vectors V[r][c] = D[r][c .. c + NV - 1] (NV = 4
// fp32 pixels when the image is exact in fp32, else 2 fp64), one per (row,
// start column), so any window row is WIN/NV aligned ds_read_b128 from an
// arbitrary column origin (the lanes of a wave read unrelated windows; a
// 16-lane b128 group spreads over 64 banks instead of 32).  48x48 fp32:
// 48 x 45 x 16 B = 34.6 KB.
//
// Reference: dphidq / dVdq sampler_RHMC.py:365-425, :448-465; gauss_PSF
// utils.py:475-486; the step loop (:522-566) is rhmc_k1step.hpp.
#pragma once
#include "rhmc_exp.hpp"
#include "rhmc_k1step.hpp"
#include "rhmc_tiledr.hpp"
#include "rhmc_wave.hpp"

namespace rhmc {

#ifndef RHMC_LANE_QUAD_RCP
#define RHMC_LANE_QUAD_RCP 1
#endif
constexpr bool kQuadRcp = RHMC_LANE_QUAD_RCP;  // A/B knob (tools/variants)
// PSF factors by recurrence (0: one exp per row and per column)
#ifndef RHMC_LANE_REC
#define RHMC_LANE_REC 1
#endif
constexpr bool kLaneRec = RHMC_LANE_REC;

template <typename DT>
struct Vec16;
template <>
struct Vec16<float> {
  using T = float __attribute__((ext_vector_type(4)));
  static constexpr int N = 4;
};
template <>
struct Vec16<double> {
  using T = double __attribute__((ext_vector_type(2)));
  static constexpr int N = 2;
};

template <int IMG, int WIN, typename DT, int LPC>
struct TiledL {
  static_assert(LPC == 1 || LPC == 2 || LPC == 4, "lanes per chain");
  static_assert(IMG >= WIN, "window inside the image");
  using V = typename Vec16<DT>::T;
  static constexpr int NV = Vec16<DT>::N;   // pixels per 16-byte vector
  static_assert(WIN % NV == 0, "window row = whole vectors");
  static constexpr int CPW = kWave / LPC;   // chains per wave
  static constexpr int PC = IMG - NV + 1;   // vectors per image row
  static constexpr int NR = (WIN + LPC - 1) / LPC;  // window rows per lane (last may idle)

  // LDS: the exp table (64 doubles = 512 B, keeps V 16-byte aligned), then V[IMG][PC].
  static __host__ __device__ constexpr size_t lds_bytes() {
    return kExpTab * sizeof(double) + (size_t)IMG * PC * sizeof(V);
  }
  static __device__ __forceinline__ void fill(V* sv, const DT* __restrict__ g) {
    for (int e = threadIdx.x; e < IMG * PC; e += blockDim.x) {
      const int r = e / PC, c = e - (e / PC) * PC;
      V v;
#pragma unroll
      for (int k = 0; k < NV; ++k) v[k] = g[r * IMG + c + k];
      sv[e] = v;
    }
  }
  static __device__ __forceinline__ int origin(double v) {
    return TiledR<IMG, WIN, DT>::origin(v);
  }
  static __device__ __forceinline__ double group_sum(double v) {
    if constexpr (LPC >= 2) v += dpp_move<0xB1>(v);  // quad_perm [1,0,3,2]
    if constexpr (LPC >= 4) v += dpp_move<0x4E>(v);  // quad_perm [2,3,0,1]
    return v;
  }

  // The chain's sums of dphidq pixel terms over its window (every lane of the
  // group gets them): s0 = sum psf s, s1 = sum psf s dx, s2 = sum psf s dy.
  // PSF factors by recurrence (RHMC_LANE_REC; utils.py:475-486 as in
  // PixK::tables_rec): runs of kRun entries start from two exps,
  //   e(v) = exp(-c v^2),  g(v) = exp(-c (2 s v + s^2)),  e(v + s) = e(v) g(v),
  //   g(v + s) = g(v) exp(-2 c s^2)
  // (s = 1 for the columns, LPC for the lane's rows): 8 exps per chain for the
  // 28 columns instead of 28, and 4 per row run instead of one per row; each
  // entry is at most kRun - 1 products from an exp (within ~25 ulp of the
  // direct exp).  A lane whose window offsets reach rec_vmax (far or NaN
  // chain) evaluates its factors directly: the choice depends on nothing but
  // the chain's own state.
  static constexpr int kRun = 7;
  static __device__ __forceinline__ void partial(const double* __restrict__ etab,
                                                 const V* __restrict__ sv, double f, double x,
                                                 double y, const Consts& c, const LeanConsts& lc,
                                                 double& s0, double& s1, double& s2) {
    const int g = lane_id() % LPC;
    const int r0 = origin(x), c0 = origin(y);
    const double cc = lc.inv_two_sig2;
    // ratio of successive row ratios, exp(-2 c LPC^2)
    const double KR = LPC == 1 ? lc.k_row
                    : LPC == 4 ? lc.k_col4 : (lc.k_row * lc.k_row) * (lc.k_row * lc.k_row);
    const double vfirst = ((double)c0 + 0.5) - y, vlast = ((double)(c0 + WIN - 1) + 0.5) - y;
    const double ufirst = ((double)(r0 + g) + 0.5) - x;
    const double ulast = ((double)(r0 + g + LPC * (NR - 1)) + 0.5) - x;
    const bool rec_c = kLaneRec && fabs(vfirst) < lc.rec_vmax && fabs(vlast) < lc.rec_vmax;
    const bool rec_r = kLaneRec && fabs(ufirst) < lc.rec_vmax && fabs(ulast) < lc.rec_vmax;
    double ey[WIN], ew[WIN];
    if (rec_c) {
#pragma unroll
      for (int j0 = 0; j0 < WIN; j0 += kRun) {
        const double v = ((double)(c0 + j0) + 0.5) - y;  // exact offsets
        double e = exp_neg(-(v * v) * cc, etab) * lc.inv_norm;
        double h = exp_neg(-fma(2.0, v, 1.0) * cc, etab);
#pragma unroll
        for (int l = 0; l < kRun && j0 + l < WIN; ++l) {
          ey[j0 + l] = e;
          e = e * h;
          h = h * lc.k_row;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < WIN; ++j) {
        const double v = ((double)(c0 + j) + 0.5) - y;  // exact offsets
        ey[j] = exp_neg(-(v * v) * cc, etab) * lc.inv_norm;
      }
    }
#pragma unroll
    for (int j = 0; j < WIN; ++j) ew[j] = ey[j] * (((double)(c0 + j) + 0.5) - y);
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    double er = 0.0, gr = 0.0;  // row run state (rec_r)
#pragma unroll 2
    for (int t = 0; t < NR; ++t) {
      const int i = g + LPC * t;
      if (WIN % LPC != 0 && i >= WIN) break;
      const V* row = sv + (r0 + i) * PC + c0;
      const double u = ((double)(r0 + i) + 0.5) - x;
      double ex;
      if (rec_r) {
        if (t % kRun == 0) {  // wave-uniform
          er = exp_neg(-(u * u) * cc, etab);
          gr = exp_neg(-fma(2.0 * LPC, u, (double)(LPC * LPC)) * cc, etab);
        }
        ex = er;
        er = er * gr;
        gr = gr * KR;
      } else {
        ex = exp_neg(-(u * u) * cc, etab);
      }
      const double fe = f * ex;
      double R = 0.0, Ry = 0.0;
      auto acc = [&](int j, double q) {
        R = fma(ey[j], q, R);
        Ry = fma(ew[j], q, Ry);
      };
#pragma unroll
      for (int jv = 0; jv < WIN / NV; ++jv) {
        const V d = row[jv * NV];
        if constexpr (kQuadRcp && NV == 4) {
          // one v_rcp_f64 per 4 pixels: 1/(l0 l1 l2 l3), then the pair
          // reciprocals and the single ones by products (Lambda >= B > 0)
          const int j = jv * NV;
          const double l0 = fma(fe, ey[j], c.B), l1 = fma(fe, ey[j + 1], c.B);
          const double l2 = fma(fe, ey[j + 2], c.B), l3 = fma(fe, ey[j + 3], c.B);
          const double p01 = l0 * l1, p23 = l2 * l3;
          const double r = rcp_nr1(p01 * p23);
          const double r01 = p23 * r, r23 = p01 * r;
          acc(j, fma((double)d[0], l1 * r01, -1.0));               // D/Lambda - 1 (:379)
          acc(j + 1, fma((double)d[1], l0 * r01, -1.0));
          acc(j + 2, fma((double)d[2], l3 * r23, -1.0));
          acc(j + 3, fma((double)d[3], l2 * r23, -1.0));
        } else {
#pragma unroll
          for (int k = 0; k < NV; k += 2) {
            const int j = jv * NV + k;
            const double l0 = fma(fe, ey[j], c.B), l1 = fma(fe, ey[j + 1], c.B);
            const double r = rcp_nr1(l0 * l1);
            acc(j, fma((double)d[k], l1 * r, -1.0));                // D/Lambda - 1 (:379)
            acc(j + 1, fma((double)d[k + 1], l0 * r, -1.0));
          }
        }
      }
      const double tt = ex * R;
      a0 += tt;
      a1 = fma(tt, u, a1);
      a2 = fma(ex, Ry, a2);
    }
    s0 = group_sum(a0);
    s1 = group_sum(a1);
    s2 = group_sum(a2);
  }

  static __device__ __forceinline__ void gradient(const double* __restrict__ etab,
                                                  const V* __restrict__ sv, double f, double x,
                                                  double y, const Consts& c, const LeanConsts& lc,
                                                  double& gf, double& gx, double& gy) {
    double s0, s1, s2;
    partial(etab, sv, f, x, y, c, lc, s0, s1, s2);
    gf = -s0;                   // :404
    gx = -s1 * f * lc.inv_var;  // :405
    gy = -s2 * f * lc.inv_var;  // :406
  }
};

// 4 waves per workgroup share the LDS image; CPW chains per wave.
template <int IMG, int WIN, typename DT, int LPC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
leapfrog_k1_tiledl(LeapArgsK1 a) {
  using TL = TiledL<IMG, WIN, DT, LPC>;
  extern __shared__ __attribute__((aligned(16))) double lds_l[];
  typename TL::V* sv = reinterpret_cast<typename TL::V*>(lds_l + kExpTab);
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  TL::fill(sv, gimg);
  exp_tab_fill(lds_l);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n_chains) return;
  const int lane = lane_id();
  const int64_t chain = TL::CPW * wave + lane / LPC;
  const bool real = chain < a.n_chains;  // ragged tail: mirror the wave's first chain
  const int64_t base = (real ? chain : TL::CPW * wave) * 3;

  double f = a.q[base], x = a.q[base + 1], y = a.q[base + 2];
  double pf = a.p[base], px = a.p[base + 1], py = a.p[base + 2];
  const LeanConsts lc = lean_consts(c);
  int it_p = 0, it_q = 0;
  unsigned st = 0u;
  k1_steps(f, x, y, pf, px, py, a.n_steps, (double)(IMG - 1), c, lc,
           [&](double f_, double x_, double y_, double& gf, double& gx, double& gy) {
             TL::gradient(lds_l, sv, f_, x_, y_, c, lc, gf, gx, gy);
           },
           it_p, it_q, st);

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
