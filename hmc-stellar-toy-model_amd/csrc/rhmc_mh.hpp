// rhmc_mh.hpp — device side of the Metropolis-Hastings outer loop
// (multi_gym.run_RHMC move-0 branch, sampler_RHMC.py:1018-1083), one thread
// per chain for the O(K) parts; the leapfrog and the potential V reuse the
// per-wave kernels.
//
// Per iteration l (all on one stream, no host round trip):
//   begin : p = z * sqrt(H(q))            (:1021-1022, z ~ N(0,1))
//           T0 = T(p, H(q)), E0 = V(q) + T0  (:1025-1027; V(q) is carried)
//           record q, V, T, E of the iteration start (:1038-1042)
//   leapfrog n_steps on (q', p')           (:1053-1054)
//   V(q')                                   (:1071)
//   end   : E1 = V(q') + T(p', H(q')), dE = E1 - E0; accept when dE < 0 or
//           ln u < -dE (:1072-1083); on accept q <- q', V(q) <- V(q').
// Randoms: host-supplied arrays (exact parity with the reference's NumPy
// stream) or Philox-4x32-10 on device, keyed by (seed, chain, iteration).
#pragma once
#include "rhmc_wave.hpp"

namespace rhmc {

// ------------------------------------------------------------ Philox-4x32-10
struct U4 {
  unsigned x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 ctr, unsigned k0, unsigned k1) {
  constexpr unsigned M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  constexpr unsigned W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    const unsigned hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = U4{hi1 ^ ctr.y ^ k0, lo1, hi0 ^ ctr.w ^ k1, lo0};
    k0 += W0;
    k1 += W1;
  }
  return ctr;
}

// 53-bit uniform in (0, 1] from two 32-bit words.
__device__ __forceinline__ double u01(unsigned a, unsigned b) {
  const unsigned long long m = ((unsigned long long)(a >> 5) << 26) | (b >> 6);  // 53 bits
  return ((double)m + 1.0) * (1.0 / 9007199254740992.0);
}

// Stream of the chain's iteration: counter = (index, iteration, chain lo, chain hi).
__device__ __forceinline__ U4 philox_block(unsigned long long seed, long long chain, int iter,
                                           unsigned index) {
  return philox4x32_10(U4{index, (unsigned)iter, (unsigned)chain, (unsigned)(chain >> 32)},
                       (unsigned)seed, (unsigned)(seed >> 32));
}

// Standard normal number `j` of (chain, iter): Box-Muller on one Philox block
// per pair of normals.
__device__ __forceinline__ double philox_normal(unsigned long long seed, long long chain,
                                                int iter, int j) {
  const U4 r = philox_block(seed, chain, iter, (unsigned)(j >> 1));
  const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
  const double rad = sqrt(-2.0 * log(u1));
  return (j & 1) ? rad * sin(6.283185307179586 * u2) : rad * cos(6.283185307179586 * u2);
}

// The acceptance uniform of (chain, iter): a separate block index.
__device__ __forceinline__ double philox_uniform(unsigned long long seed, long long chain,
                                                 int iter) {
  const U4 r = philox_block(seed, chain, iter, 0x80000000u);
  return u01(r.x, r.y);
}

struct MhArgs {
  double* q;        // [n][3K] current state (updated on accept)
  double* q_prop;   // [n][3K] proposal
  double* p;        // [n][3K] momentum
  double* V_cur;    // [n] V of the current state
  double* V_prop;   // [n] V of the proposal (written by the energy kernel)
  double* E0;       // [n] energy at the iteration start
  const double* z;  // nullable [n_iter][n][3K] standard normals
  const double* u;  // nullable [n_iter][n] uniforms
  double* q_chain;  // nullable [n_iter][n][3K]
  double* E_chain;  // nullable [n_iter][n]
  double* V_chain;  // nullable [n_iter][n]
  double* T_chain;  // nullable [n_iter][n]
  int32_t* accept;  // nullable [n_iter][n]
  int64_t n;
  int K, iter;
  unsigned long long seed;
  Consts c;
};

__device__ __forceinline__ void metric_pair(double f, const Consts& c, double& hff, double& hxx) {
  hff = H_ff(f, c);
  hxx = H_xx(f, c);
}

// T(p, H) = (sum p^2/H + sum log|H|)/2 with the reference's two separate sums (:353-363).
__device__ __forceinline__ double kinetic(const double* q, const double* p, int K,
                                          const Consts& c) {
  double t1 = 0.0, t2 = 0.0;
  for (int k = 0; k < K; ++k) {
    double hff, hxx;
    metric_pair(q[3 * k], c, hff, hxx);
    t1 += p[3 * k] * p[3 * k] / hff;
    t1 += p[3 * k + 1] * p[3 * k + 1] / hxx;
    t1 += p[3 * k + 2] * p[3 * k + 2] / hxx;
  }
  for (int k = 0; k < K; ++k) {
    double hff, hxx;
    metric_pair(q[3 * k], c, hff, hxx);
    t2 += log(fabs(hff));
    t2 += log(fabs(hxx));
    t2 += log(fabs(hxx));
  }
  return (t1 + t2) / 2.0;
}

__global__ void __launch_bounds__(256) mh_begin_kernel(MhArgs a) {
  const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= a.n) return;
  const int d = 3 * a.K;
  const double* q = a.q + ch * d;
  double* p = a.p + ch * d;
  double* qp = a.q_prop + ch * d;
  for (int k = 0; k < a.K; ++k) {
    double hff, hxx;
    metric_pair(q[3 * k], a.c, hff, hxx);
    const double h[3] = {hff, hxx, hxx};
    for (int j = 0; j < 3; ++j) {
      const int idx = 3 * k + j;
      const double zz = a.z ? a.z[((int64_t)a.iter * a.n + ch) * d + idx]
                            : philox_normal(a.seed, ch, a.iter, idx);
      p[idx] = zz * sqrt(h[j]);                  // u_sample(d) * np.sqrt(H_diag) (:1022)
      qp[idx] = q[idx];
    }
  }
  const double T0 = kinetic(q, p, a.K, a.c);
  const double V0 = a.V_cur[ch];
  const double E0 = V0 + T0;
  a.E0[ch] = E0;
  const int64_t r = (int64_t)a.iter * a.n + ch;
  if (a.q_chain)
    for (int i = 0; i < d; ++i) a.q_chain[r * d + i] = q[i];
  if (a.V_chain) a.V_chain[r] = V0;
  if (a.T_chain) a.T_chain[r] = T0;
  if (a.E_chain) a.E_chain[r] = E0;
}

__global__ void __launch_bounds__(256) mh_end_kernel(MhArgs a) {
  const int64_t ch = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= a.n) return;
  const int d = 3 * a.K;
  const double* qp = a.q_prop + ch * d;
  const double V1 = a.V_prop[ch];
  const double E1 = V1 + kinetic(qp, a.p + ch * d, a.K, a.c);
  const double dE = E1 - a.E0[ch];
  const double uu = a.u ? a.u[(int64_t)a.iter * a.n + ch] : philox_uniform(a.seed, ch, a.iter);
  const double lnu = log(uu);
  const bool acc = (dE < 0.0) || (lnu < -dE);   // :1076
  if (acc) {
    double* q = a.q + ch * d;
    for (int i = 0; i < d; ++i) q[i] = qp[i];
    a.V_cur[ch] = V1;
  }
  if (a.accept) a.accept[(int64_t)a.iter * a.n + ch] = acc ? 1 : 0;
}

// The same two steps with one wave per chain, lanes over the 3K coordinates
// (many stars: one thread per chain would leave most of the GPU idle, e.g.
// 4096 chains of K = 51 = 64 busy SIMDs).  T's two sums are wave sums
// (numpy's np.sum is pairwise: no order is the reference's exactly).
__global__ void __launch_bounds__(256) mh_begin_wave_kernel(MhArgs a) {
  const int64_t ch = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (ch >= a.n) return;
  const int lane = lane_id();
  const int d = 3 * a.K;
  const double* q = a.q + ch * d;
  double* p = a.p + ch * d;
  double* qp = a.q_prop + ch * d;
  const int64_t r = (int64_t)a.iter * a.n + ch;
  double t1 = 0.0, t2 = 0.0;
  for (int idx = lane; idx < d; idx += kWave) {
    double hff, hxx;
    metric_pair(q[idx - idx % 3], a.c, hff, hxx);
    const double h = (idx % 3 == 0) ? hff : hxx;
    const double zz = a.z ? a.z[((int64_t)a.iter * a.n + ch) * d + idx]
                          : philox_normal(a.seed, ch, a.iter, idx);
    const double pv = zz * sqrt(h);                 // u_sample(d) * np.sqrt(H_diag) (:1022)
    p[idx] = pv;
    qp[idx] = q[idx];
    if (a.q_chain) a.q_chain[r * d + idx] = q[idx];
    t1 += pv * pv / h;
    t2 += log(fabs(h));
  }
  const double T0 = (wave_sum(t1) + wave_sum(t2)) / 2.0;  // (:353-363)
  if (lane == 0) {
    const double V0 = a.V_cur[ch];
    const double E0 = V0 + T0;
    a.E0[ch] = E0;
    if (a.V_chain) a.V_chain[r] = V0;
    if (a.T_chain) a.T_chain[r] = T0;
    if (a.E_chain) a.E_chain[r] = E0;
  }
}

__global__ void __launch_bounds__(256) mh_end_wave_kernel(MhArgs a) {
  const int64_t ch = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
  if (ch >= a.n) return;
  const int lane = lane_id();
  const int d = 3 * a.K;
  const double* qp = a.q_prop + ch * d;
  const double* p = a.p + ch * d;
  double t1 = 0.0, t2 = 0.0;
  for (int idx = lane; idx < d; idx += kWave) {
    double hff, hxx;
    metric_pair(qp[idx - idx % 3], a.c, hff, hxx);
    const double h = (idx % 3 == 0) ? hff : hxx;
    t1 += p[idx] * p[idx] / h;
    t2 += log(fabs(h));
  }
  const double V1 = a.V_prop[ch];
  const double E1 = V1 + (wave_sum(t1) + wave_sum(t2)) / 2.0;
  const double dE = E1 - a.E0[ch];
  const double uu = a.u ? a.u[(int64_t)a.iter * a.n + ch] : philox_uniform(a.seed, ch, a.iter);
  const bool acc = (dE < 0.0) || (log(uu) < -dE);   // :1076 (wave-uniform)
  if (acc) {
    double* q = a.q + ch * d;
    for (int idx = lane; idx < d; idx += kWave) q[idx] = qp[idx];
  }
  if (lane == 0) {
    if (acc) a.V_cur[ch] = V1;
    if (a.accept) a.accept[(int64_t)a.iter * a.n + ch] = acc ? 1 : 0;
  }
}

}  // namespace rhmc
