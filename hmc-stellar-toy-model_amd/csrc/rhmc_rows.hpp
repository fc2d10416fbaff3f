// rhmc_rows.hpp — ragged chain sets on the device, for the reversible-jump
// driver (librhmc_rj.so, include/rhmc_rj.h).  The driver keeps every chain's
// state in HBM for the whole run as rows of padded [n][ld] arrays (chain c's
// first 3 K[c] entries, zeros after), whatever its current star count:
//
//   rows_copy_kernel     dst[dst_rows[i]][0:width] = src[src_rows[i]][0:width]
//                        (either index list may be the identity): the phase
//                        gathers of one star count into a packed [n_K][3K]
//                        batch for the fixed-K kernels and the scatters back,
//                        the restore / commit of rejected / accepted rows
//   kinetic_rows_kernel  run_RHMC's momentum draw p = z sqrt(H(q))
//                        (sampler_RHMC.py:1021-1022, the z drawn on the host
//                        from each chain's NumPy stream) and the kinetic
//                        energy T(p, H(q)) = (sum p^2/H + sum ln|H|) / 2
//                        (:353-363) with NumPy's pairwise summation order, one
//                        wave per chain
//
// HBM-bound byte moves and O(K) per-chain arithmetic: no LDS, no MFMA.  The
// metric H_ff / H_xx follows the reference's operation order (:260-292) with
// FP contraction off, so p is the host replica's value bit for bit (IEEE
// division and sqrt); ln is the device's, within an ulp of C libm's.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rhmc {

struct RowsCopyArgs {
  const double* src;
  double* dst;
  const int64_t* src_rows;  // nullable: row i
  const int64_t* dst_rows;  // nullable: row i
  int64_t ld_src, ld_dst;
  int64_t n;
  int32_t width;
};

// one thread per copied double; rows of up to 768 doubles
__global__ void __launch_bounds__(256) rows_copy_kernel(RowsCopyArgs a) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = g / a.width;
  if (i >= a.n) return;
  const int32_t j = (int32_t)(g - i * a.width);
  const int64_t rs = a.src_rows ? a.src_rows[i] : i;
  const int64_t rd = a.dst_rows ? a.dst_rows[i] : i;
  a.dst[rd * a.ld_dst + j] = a.src[rs * a.ld_src + j];
}

struct KineticArgs {
  const double* q;       // [n][ld]
  double* p;             // [n][ld]
  const double* z;       // nullable: packed normals, chain c's at zoff[c]
  const int64_t* zoff;
  const int32_t* K;      // [n]
  double* T;             // [n]
  int64_t ld, n;
  double g_ff2, g_ff, g_xx, g0, g1, g2, B, f_low;
};

#pragma clang fp contract(off)
// H of one star's coordinate slot (0: flux, 1/2: position), sampler_RHMC.py:260-292
__device__ inline double rows_metric(const KineticArgs& a, double f, int slot) {
  if (slot == 0) return 1. / (f / a.g_ff2 + (a.B / a.g0) / a.g_ff);
  const double fl = f < a.f_low ? a.f_low : f;
  const double s = 1. / (a.g1 * fl) + a.B / (a.g2 * (fl * fl));
  return a.g_xx * (1. / s);
}

// NumPy's pairwise_sum_DOUBLE over a[0 .. n), n <= 128: eight accumulators,
// then the tail (host/np_legacy.hpp pairwise_sum)
__device__ __forceinline__ double rows_block_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
  int64_t i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 += a[i];
    r1 += a[i + 1];
    r2 += a[i + 2];
    r3 += a[i + 3];
    r4 += a[i + 4];
    r5 += a[i + 5];
    r6 += a[i + 6];
    r7 += a[i + 7];
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i];
  return res;
}

// the recursive halving above 128 terms, unrolled to the depth 3 K <= 768 needs
template <int DEPTH>
__device__ __forceinline__ double rows_pairwise(const double* a, int64_t n) {
  if constexpr (DEPTH == 0) {
    return rows_block_sum(a, n);
  } else {
    if (n <= 128) return rows_block_sum(a, n);
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return rows_pairwise<DEPTH - 1>(a, n2) + rows_pairwise<DEPTH - 1>(a + n2, n - n2);
  }
}

// One wave per chain (WAVES chains per block): lanes over the stars evaluate
// H once per star, draw p and write the two sums' terms into the wave's LDS
// rows in NumPy's array layout (p**2 / H and log(abs(H))); lane 0 and lane 1
// then sum them in NumPy's pairwise order.  Two shapes: 4 chains of up to 256
// stars per block (the reversible-jump driver's usual N_max), 1 chain of up
// to 1024 (rows wider than 768 doubles); DEPTH covers the pairwise halving
// (128 x 2^DEPTH >= MAXD).  A chain with more stars than MAXD / 3 gets T = NaN.
template <int WAVES, int MAXD, int DEPTH>
__global__ void __launch_bounds__(WAVES * 64) kinetic_rows_kernel(KineticArgs a) {
  __shared__ double terms[WAVES][2][MAXD];
  const int wv = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int64_t c = (int64_t)blockIdx.x * WAVES + wv;
  const bool live = c < a.n;
  const double* q = a.q + (live ? c : 0) * a.ld;
  double* p = a.p + (live ? c : 0) * a.ld;
  const int64_t d0 = live ? 3 * (int64_t)a.K[c] : 0;
  const bool over = d0 > MAXD;  // wave-uniform
  const int64_t d = over ? 0 : d0;
  double* t1 = terms[wv][0];
  double* t2 = terms[wv][1];
  for (int64_t i = 3 * lane; i < d; i += 3 * 64) {
    const double hf = rows_metric(a, q[i], 0), hx = rows_metric(a, q[i], 1);
    double pf, px, py;
    if (a.z) {  // p = randn(3K) * sqrt(H); H_y = H_x, one sqrt per star as on the host
      const double* z = a.z + a.zoff[c];
      const double sf = sqrt(hf), sx = sqrt(hx);
      pf = z[i] * sf;
      px = z[i + 1] * sx;
      py = z[i + 2] * sx;
      p[i] = pf;
      p[i + 1] = px;
      p[i + 2] = py;
    } else {
      pf = p[i];
      px = p[i + 1];
      py = p[i + 2];
    }
    t1[i] = (pf * pf) / hf;
    t1[i + 1] = (px * px) / hx;
    t1[i + 2] = (py * py) / hx;
    const double lf = log(fabs(hf)), lx = log(fabs(hx));  // a star's x and y share H
    t2[i] = lf;
    t2[i + 1] = lx;
    t2[i + 2] = lx;
  }
  if (live && a.z && !over)
    for (int64_t i = d + lane; i < a.ld; i += 64) p[i] = 0.;
  __syncthreads();
  if (!live || lane > 1) return;
  const double s = rows_pairwise<DEPTH>(lane == 0 ? t1 : t2, d);
  const double s2 = __shfl_down(s, 1, 64);  // lane 1's sum to lane 0
  if (lane == 0) a.T[c] = over ? __builtin_nan("") : (s + s2) / 2.;
}
#pragma clang fp contract(on)

}  // namespace rhmc
