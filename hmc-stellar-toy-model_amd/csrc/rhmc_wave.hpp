// rhmc_wave.hpp — wave64 building blocks and the per-star metric of the RHMC
// step, written for gfx950 (CDNA4).  One wavefront owns one chain; lane k < K
// owns star k's (f, x, y) and (p_f, p_x, p_y).
//
// Reference formulas (file:line into jaekor91/HMC-stellar-toy-model):
//   H_ff  sampler_RHMC.py:283-292   H_xx sampler_RHMC.py:260-280
//   dphidq metric term :459-463     dtaudq :467-483     dtaudp :485-492
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rhmc {

constexpr int kWave = 64;

// Constants derived on the host from rhmc_params exactly the way the reference
// derives them (sigma = FWHM/2.354, 2*sigma**2, pi*2*sigma**2, var, (B/g0)/g_ff).
struct Consts {
  double dt, hdt, delta;
  double B, f_lim, f_low;
  double two_sig2, psf_norm, var;
  double g_xx, g_ff, g_ff2, g0, g1, g2, c0;
  double alpha, beta, vc_pow, vprior;
  // reciprocals for the division-lean forms, computed once on the host (a
  // device-side computation gets re-materialised inside the step loop)
  double inv_gff2, inv_g1, Bg2, inv_gxx, inv_two_sig2, inv_norm, inv_var;
  double two_Bg2;  // 2 B/g2 (exact), a kernel argument so it stays in SGPRs
  // PSF factor recurrences (rhmc_tiledr.hpp factors): ratio of successive row
  // ratios exp(-2/(2 sigma^2)), of column ratios 4 apart exp(-32/(2 sigma^2)),
  // and the largest |window offset| for which the recurrence stays in range
  double k_row, k_col4, rec_vmax;
  // near-wall threshold of the flux wall: f_lim - 2^-40 max(1, |f_lim|)
  double near_f;
  int counter_max, use_prior, use_Vc, pad;
};

// The flux folded into a star's PSF factors (the kernels scale the column
// factors by f, so that one product serves Lambda and the sums, and divide the
// flux sum by f again).  At f = 0 that gives 0/0 where the reference's
// -sum psf (D/Lambda - 1) (:404) is finite, and a subnormal f underflows.  The
// fold is f pushed 2^-600 away from zero: copysign(|f| + 2^-600, f).  For
// |f| >= 2^-546 that IS f (2^-600 is below half its ulp; in [2^-547, 2^-546)
// it is exactly half an ulp and rounds an odd mantissa up), so every ordinary
// chain is bit-identical; for smaller |f| (0 included) the flux sum comes
// back exactly by the division and Lambda still rounds to B as with f psf.
// The x, y sums then carry the fold for f: they differ from the reference's
// (f/var) sum by less than 2^-599 relative to the sum, far below any
// momentum's ulp.  Two VALU instructions, no compare or branch.
__device__ __forceinline__ double flux_fold(double f) {
  return copysign(fabs(f) + 0x1p-600, f);
}

// A position reflection (v < 0 or v > edge, sampler_RHMC.py:561-564) whose
// coordinate lies within 2^-40 (9.1e-13) of its wall, relative to max(1, wall)
// (edge >= 1): RHMC_STATUS_NEAR_WALL.  Only meaningful when v
// reflected.  Powers of two keep the constants inline literals (no registers).
__device__ __forceinline__ bool near_edge(double v, double edge) {
  return v >= -0x1p-40 && (v - edge) <= edge * 0x1p-40;
}

// ---------------------------------------------------------------- lane moves
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }
// The lane id by a volatile read: values derived from it are recomputed where
// used instead of being hoisted out of a step loop and held in VGPRs.
__device__ __forceinline__ int lane_id_fresh() {
  int lid;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
  return lid;
}

// Broadcast lane `src` (wave-uniform) of a double to every lane: two
// v_readlane_b32 into SGPRs, no LDS traffic.
__device__ __forceinline__ double bcast(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Butterfly all-reduce; every lane ends with the same, deterministic sum.
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

// NaN-propagating max, matching np.max on an array holding a NaN.
__device__ __forceinline__ double nanmax2(double a, double b) {
  return (a != a || a > b) ? a : b;
}
__device__ __forceinline__ double wave_nanmax(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = nanmax2(v, __shfl_xor(v, m, kWave));
  return v;
}

// Wave-local LDS hand-off (tables written by some lanes, read by others).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ------------------------------------------------------------ per-star metric
// H_ff(f) = 1/(f/g_ff2 + (B/g0)/g_ff)                       (:290)
__device__ __forceinline__ double H_ff(double f, const Consts& c) {
  return 1.0 / (f / c.g_ff2 + c.c0);
}
// dH_ff/df as the reference writes it: -1/(f + (B/g0)/g_ff)**2 — ignores
// g_ff2, the true derivative only when g_ff2 == 1 (quirk kept, :292).
__device__ __forceinline__ double H_ff_grad(double f, const Consts& c) {
  const double t = f + c.c0;
  return -1.0 / (t * t);
}
// H_xx(f) = g_xx / (1/(g1 f) + B/(g2 f^2)), f clamped to f_low (:267-273).
__device__ __forceinline__ double H_xx_s(double f, const Consts& c) {
  return 1.0 / (c.g1 * f) + c.B / (c.g2 * (f * f));
}
__device__ __forceinline__ double H_xx(double f, const Consts& c) {
  const double fl = (f < c.f_low) ? c.f_low : f;
  return c.g_xx * (1.0 / H_xx_s(fl, c));
}
// dH_xx/df, 0 when clamped (:275-278).
__device__ __forceinline__ double H_xx_grad(double f, const Consts& c) {
  if (f < c.f_low) return 0.0;
  const double s = H_xx_s(f, c);
  const double a = 1.0 / (c.g1 * (f * f)) + 2.0 * c.B / (c.g2 * (f * f * f));
  return c.g_xx * a * (1.0 / (s * s));
}

// ---------------------------------------------------------------------------
// Division-lean form of the same metric for the single-star kernel.  Every
// quantity the step needs is a few FMAs of
//   A  = f/g_ff2 + (B/g0)/g_ff        (= 1/H_ff)
//   Bf = f + (B/g0)/g_ff              (H_ff' = -1/Bf^2)
//   u  = 1/max(f, f_low),  s = u/g1 + (B/g2) u^2   (H_xx = g_xx/s)
// with one reciprocal per evaluation instead of the reference's chain of
// divides; results agree with the reference expressions to a few ulp.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double rcp_nr(double d) {  // ~correctly rounded 1/d
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

struct LeanConsts {
  double inv_gff2, c0, inv_g1, Bg2, two_Bg2, inv_gxx, f_low;
  double inv_two_sig2, inv_norm, inv_var;  // PSF exponent / normalisation, 1/var
  double k_row, k_col4, rec_vmax;          // PSF factor recurrences (Consts)
};

__device__ __forceinline__ LeanConsts lean_consts(const Consts& c) {
  LeanConsts l;
  l.inv_gff2 = c.inv_gff2;
  l.c0 = c.c0;
  l.inv_g1 = c.inv_g1;
  l.Bg2 = c.Bg2;
  l.two_Bg2 = c.two_Bg2;
  l.inv_gxx = c.inv_gxx;
  l.f_low = c.f_low;
  l.inv_two_sig2 = c.inv_two_sig2;
  l.inv_norm = c.inv_norm;
  l.inv_var = c.inv_var;
  l.k_row = c.k_row;
  l.k_col4 = c.k_col4;
  l.rec_vmax = c.rec_vmax;
  return l;
}

// 1/H_ff, 1/H_xx at flux f (the q-loop's dtaudp = p * (1/H)).
__device__ __forceinline__ void inv_metric(double f, const LeanConsts& l, double& ihff,
                                           double& ihxx) {
  ihff = fma(f, l.inv_gff2, l.c0);
  const double fl = (f < l.f_low) ? l.f_low : f;
  const double u = rcp_nr(fl);
  ihxx = (u * fma(l.Bg2, u, l.inv_g1)) * l.inv_gxx;
}

// The two fixed-point loops of RHMC_single_step, evaluated SPEC iterations
// per pass: the iterates of one pass depend on each other only through the
// flux chain, so the reciprocals and the convergence tests of SPEC iterations
// overlap instead of paying one dependent chain + one branch per iteration.
// The state and iteration count returned are those of the first iteration
// whose test stops the reference's loop (`while dp > delta and counter <
// counter_max`, NaN stops); later speculative iterates are discarded.

// p-loop (:528-535) on the flux momentum (dtaudq is zero on x, y): returns the
// iteration count, `last` = the final |dp|.
template <int SPEC>
__device__ __forceinline__ int p_loop_spec(double& pf, double coef, double hdt, double delta,
                                           int cmax, double& last) {
  const double rho = pf;
  int n = 0;
  for (;;) {
    double P[SPEC + 1], d[SPEC];
    P[0] = pf;
#pragma unroll
    for (int k = 0; k < SPEC; ++k) {
      P[k + 1] = rho - hdt * ((P[k] * P[k]) * coef / 2.0);
      d[k] = fabs(P[k] - P[k + 1]);
    }
    bool stop = false;
    double sel = P[SPEC], dsel = d[SPEC - 1];
    int take = SPEC;
#pragma unroll
    for (int k = SPEC - 1; k >= 0; --k) {
      if (!(d[k] > delta) || n + k + 1 >= cmax) {
        stop = true;
        take = k + 1;
        sel = P[k + 1];
        dsel = d[k];
      }
    }
    pf = sel;
    n += take;
    if (stop) {
      last = dsel;
      return n;
    }
  }
}

// q-loop (:538-545): q_{n+1} = q_s + hdt (p/H(q_s) + p/H(q_n)).
template <int SPEC>
__device__ __forceinline__ int q_loop_spec(double& f, double& x, double& y, double pf, double px,
                                           double py, double hdt, const LeanConsts& lc,
                                           double delta, int cmax, double& last);

// -H_ff'/H_ff^2 = (A/Bf)^2  (dtaudq's coefficient, :479)
__device__ __forceinline__ double dtaudq_coef_lean(double f, const LeanConsts& l) {
  const double A = fma(f, l.inv_gff2, l.c0);
  const double t = A * rcp_nr(f + l.c0);
  return t * t;
}

template <int SPEC>
__device__ __forceinline__ int q_loop_spec(double& f, double& x, double& y, double pf, double px,
                                           double py, double hdt, const LeanConsts& lc,
                                           double delta, int cmax, double& last) {
  const double sf = f, sx = x, sy = y;
  double ihff, ihxx;
  inv_metric(sf, lc, ihff, ihxx);
  const double af = pf * ihff, ax = px * ihxx, ay = py * ihxx;
  int n = 0;
  for (;;) {
    double F[SPEC + 1], X[SPEC + 1], Y[SPEC + 1], d[SPEC];
    F[0] = f;
    X[0] = x;
    Y[0] = y;
#pragma unroll
    for (int k = 0; k < SPEC; ++k) {
      inv_metric(F[k], lc, ihff, ihxx);
      F[k + 1] = sf + hdt * (af + pf * ihff);
      X[k + 1] = sx + hdt * (ax + px * ihxx);
      Y[k + 1] = sy + hdt * (ay + py * ihxx);
      const double a0 = fabs(F[k] - F[k + 1]), a1 = fabs(X[k] - X[k + 1]),
                   a2 = fabs(Y[k] - Y[k + 1]);
      const double sum = a0 + a1 + a2;
      d[k] = (sum != sum) ? sum : fmax(fmax(a0, a1), a2);  // np.max propagates NaN
    }
    bool stop = false;
    double sf_ = F[SPEC], sx_ = X[SPEC], sy_ = Y[SPEC], dsel = d[SPEC - 1];
    int take = SPEC;
#pragma unroll
    for (int k = SPEC - 1; k >= 0; --k) {
      if (!(d[k] > delta) || n + k + 1 >= cmax) {
        stop = true;
        take = k + 1;
        sf_ = F[k + 1];
        sx_ = X[k + 1];
        sy_ = Y[k + 1];
        dsel = d[k];
      }
    }
    f = sf_;
    x = sx_;
    y = sy_;
    n += take;
    if (stop) {
      last = dsel;
      return n;
    }
  }
}

// (H_ff'/H_ff + 2 H_xx'/H_xx)/2 with H_ff'/H_ff = -A/Bf^2 and
// H_xx'/H_xx = u^2 (1/g1 + 2 (B/g2) u)/s (0 when clamped) (:461-463)
__device__ __forceinline__ double metric_flux_term_lean(double f, const LeanConsts& l) {
  const double A = fma(f, l.inv_gff2, l.c0);
  const double ib = rcp_nr(f + l.c0);
  const double t1 = -A * (ib * ib);
  double t2 = 0.0;
  if (!(f < l.f_low)) {
    const double u = rcp_nr(f);
    const double s = u * fma(l.Bg2, u, l.inv_g1);
    t2 = (u * u) * fma(2.0 * l.Bg2, u, l.inv_g1) * rcp_nr(s);
  }
  return (t1 + 2.0 * t2) / 2.0;
}

// dphidq's metric term on the flux slot: (H_ff'/H_ff + 2 H_xx'/H_xx)/2 (:461-463)
__device__ __forceinline__ double metric_flux_term(double f, const Consts& c) {
  const double hff = H_ff(f, c), hffg = H_ff_grad(f, c);
  const double hxx = H_xx(f, c), hxxg = H_xx_grad(f, c);
  return ((hffg / hff) + (2.0 * hxxg / hxx)) / 2.0;
}

// dtaudq on the flux slot: (p_f^2 * (-H_ff'/H_ff^2))/2 — x, y slots are 0 (:479-481).
// `coef` = -H_ff'/H_ff^2 is constant while q is fixed (the whole p-loop).
__device__ __forceinline__ double dtaudq_coef(double f, const Consts& c) {
  const double h = H_ff(f, c);
  return -H_ff_grad(f, c) / (h * h);
}

// ------------------------------------------------------- DPP / permlane sums
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

// Sum over the 32 lanes of each half-wave; every lane of a half gets its
// half's sum (rows 0+1 and rows 2+3), bit-identical within the half.
__device__ __forceinline__ double half_sum_dpp(double v) {
  v += dpp_move<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_move<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_move<0x141>(v);  // row_half_mirror
  v += dpp_move<0x140>(v);  // row_mirror
  return swap_add<false>(v);
}

}  // namespace rhmc
