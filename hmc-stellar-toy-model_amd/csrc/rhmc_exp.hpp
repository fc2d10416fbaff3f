// rhmc_exp.hpp — exp(t) for t <= 0 in fp64 for the PSF factor tables.
//
// t = (64 N_hi + j) ln2/64 + r with |r| <= ln2/128, so
//   exp(t) = 2^N_hi * 2^(j/64) * e^r,
// 2^(j/64) from a 64-entry table kept in LDS (filled once per workgroup) and
// e^r - 1 from its degree-5 Taylor polynomial (truncation r^6/720 < 3.5e-17,
// a third of an ulp; the degree-6 one measured 0.6 % slower at C5, round 3).
// About 15 VALU instructions against ~30 for the general-purpose exp (no
// overflow handling is needed for t <= 0); the result agrees with it to ~1 ulp
// (tools/isa_bench.hip measures the difference).  NaN propagates; t < -1400
// underflows to 0 like exp.
#pragma once
#include <hip/hip_runtime.h>


namespace rhmc {

constexpr int kExpTab = 64;

__device__ static const double kExp2Tab64[kExpTab] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0};

// Copy the table into LDS (all threads of the block; call before the block
// barrier that precedes the first use).
__device__ __forceinline__ void exp_tab_fill(double* lds_tab) {
  for (int i = threadIdx.x; i < kExpTab; i += blockDim.x) lds_tab[i] = kExp2Tab64[i];
}

__device__ __forceinline__ double exp_neg(double t, const double* __restrict__ lds_tab) {
  constexpr double kInvLn2_64 = 0x1.71547652b82fep+6;   // 64/ln2
  constexpr double kLn2_64_hi = 0x1.62e42fee00000p-7;   // ln2/64, high part
  constexpr double kLn2_64_lo = 0x1.a39ef35793c76p-39;  // ln2/64 - high part
  t = (t < -1400.0) ? -1400.0 : t;                      // NaN compares false: kept
  const double nd = rint(t * kInvLn2_64);
  const int n = (int)nd;
  double r = fma(-nd, kLn2_64_hi, t);
  r = fma(-nd, kLn2_64_lo, r);
  const double tj = lds_tab[n & (kExpTab - 1)];
  double q = fma(r, 1.0 / 120.0, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  return ldexp(fma(tj, q * r, tj), n >> 6);  // arithmetic shift: floor(n / 64)
}

// ln(y) for finite y > 0 (the model image, y >= B > 0), branch-free: y = 2^e m
// with m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(s), s = (m - 1)/(m + 1),
// |s| <= 0.1716, the odd series to s^21 (truncation < 2^-55 relative), and
// e ln2 in two parts.  About 25 VALU instructions against ~100 for the
// general-purpose log (special operands, denormals); within ~2 ulp of it.
__device__ __forceinline__ double log_pos(double y) {
  constexpr double kLn2Hi = 0x1.62e42fefa3800p-1;       // ln2, 43 significant bits
  constexpr double kLn2Lo = 0x1.ef35793c76730p-45;      // ln2 - kLn2Hi
  double m = __builtin_amdgcn_frexp_mant(y);            // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(y);
  const bool lo = m < 0x1.6a09e667f3bcdp-1;            // sqrt(1/2)
  m = lo ? m + m : m;
  e = lo ? e - 1 : e;
  const double num = m - 1.0, den = m + 1.0;            // exact
  double r = __builtin_amdgcn_rcp(den);
  r = fma(r, fma(-den, r, 1.0), r);
  double s = num * r;
  s = fma(r, fma(-den, s, num), s);                     // s to ~0.5 ulp
  const double s2 = s * s;
  double p = fma(s2, 1.0 / 21.0, 1.0 / 19.0);
  p = fma(p, s2, 1.0 / 17.0);
  p = fma(p, s2, 1.0 / 15.0);
  p = fma(p, s2, 1.0 / 13.0);
  p = fma(p, s2, 1.0 / 11.0);
  p = fma(p, s2, 1.0 / 9.0);
  p = fma(p, s2, 1.0 / 7.0);
  p = fma(p, s2, 1.0 / 5.0);
  p = fma(p, s2, 1.0 / 3.0);
  const double ed = (double)e;
  const double ls = fma(2.0 * s, s2 * p, fma(ed, kLn2Lo, 2.0 * s));  // ln m + e ln2_lo
  return fma(ed, kLn2Hi, ls);
}

}  // namespace rhmc
