// rhmc_mhpk.hpp — the whole MH outer loop (multi_gym.run_RHMC move-0 branch,
// sampler_RHMC.py:1018-1083) for 2 <= K <= 10 stars in ONE launch on the
// pixel-major kernel (rhmc_pixk.hpp): 32 lanes per chain, two chains per
// wave64, lane m < K owns star m.
//
// Per iteration, the arithmetic of mh_begin_kernel / leapfrog / energy /
// mh_end_kernel (rhmc_mh.hpp) without their launches and HBM round trips:
//   p = z sqrt(H(q))                      (:1021-1022; z of index 3m + j)
//   T0 = T(p, H(q)), E0 = V(q) + T0       (:1025-1027; V(q) carried)
//   n_steps x RHMC_single_step            (:1053-1054, km_steps)
//   V(q'): infinite outside the support (:303-317), else the image sum of
//          Lambda - D ln Lambda (pixel-major, as the gradient) + the prior
//   accept when dE < 0 or ln u < -dE      (:1072-1083)
// T is summed star by star in the reference's order (one lane reads the
// chain's terms), exactly as rhmc_mh.hpp's kinetic().  One launch per
// iteration (mh_pk_iter) after one for the starting V (mh_pk_v0); the chain's
// state and carried V(q) stay in HBM between launches (40 B per star).
#pragma once
#include "rhmc_mh.hpp"
#include "rhmc_pixk.hpp"

namespace rhmc {

struct MhKArgs {
  double* q;              // [n][3K] current state, updated in place
  const float* Df;        // D in fp32 (the pixel-major kernel needs an exact image)
  const double* z;        // nullable [n_iter][n][3K]
  const double* u;        // nullable [n_iter][n]
  double* q_chain;        // nullable [n_iter][n][3K]
  double* E_chain;        // nullable [n_iter][n]
  double* V_chain;        // nullable [n_iter][n]
  double* T_chain;        // nullable [n_iter][n]
  int32_t* accept;        // nullable [n_iter][n]
  int64_t n;
  int K, n_iter, n_steps, f_pos;
  unsigned long long seed;
  Consts c;
};

template <int IMG, int KMAX>
struct MhPK {
  using PK = PixK<IMG, KMAX, RHMC_PK_CT>;
  // LDS: the pixel-major kernel's (exp table, star tables, factor tables,
  // image).
  static __host__ __device__ constexpr size_t lds_bytes(int waves) {
    return PK::lds_bytes(waves);
  }

  // V of the chain whose star table holds q (sampler_RHMC.py:294-330): the
  // image sum of Lambda - D ln Lambda over the lane's pixels (Lambda as in
  // the gradient: B + the stars in ascending order), the prior per star, and
  // infinity outside the support.  Every lane of the chain gets it.
  static __device__ __forceinline__ double potential(const double* __restrict__ etab,
                                                  const float* __restrict__ simg,
                                                  const KRStar* tab, double* rtab, int K,
                                                  int f_pos, const Consts& c,
                                                  const LeanConsts& lc) {
    // lane id by a volatile read: the pixel addresses below are not hoisted
    // out of the MH loop (live across the step loop they would spill)
    int lid;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
    const int m = lid & (PK::LPC - 1);
    const int cg = m & 15, rh = m >> 4;
    double* ctab = rtab + (size_t)IMG * KMAX;
    wave_lds_sync();
    PK::tables(etab, tab, rtab, ctab, K, lc);
    wave_lds_sync();
    double v = 0.0;
#pragma unroll 1
    for (int ci = 0; ci < PK::NC; ++ci) {
      double fey[KMAX];
#pragma unroll
      for (int k = 0; k < KMAX; ++k) fey[k] = ctab[(cg + 16 * ci) * KMAX + k];
      const double* rt = rtab + (size_t)(rh * PK::NR) * KMAX;
#pragma unroll 2
      for (int r = 0; r < PK::NR; ++r) {
        double l = c.B;  // Lambda (:373-376)
#pragma unroll
        for (int k = 0; k < KMAX; ++k) l = fma(rt[r * KMAX + k], fey[k], l);
        const double d = (double)simg[PK::img_index(rh * PK::NR + r, cg + 16 * ci)];
        v += l - d * log_pos(l);  // :322-328
      }
    }
    v = half_sum_dpp(v);
    const KRStar st = tab[m < K ? m : 0];
    if (c.use_prior)  // V_prior per star, added after the image sum (:326, :329-330)
      v += half_sum_dpp(m < K ? c.alpha * log(st.f) + c.vprior : 0.0);
    const bool bad = m < K && (((f_pos & RHMC_V_FLUX_WALL) && st.f < c.f_lim) ||
                               (!(f_pos & RHMC_V_NO_POSCHECK) &&
                                (st.x < -1.0 || st.x > (double)(IMG + 1) || st.y < -1.0 ||
                                 st.y > (double)(IMG + 1))));  // :303-317
    return half_any(bad) ? INFINITY : v;
  }

  // T(p, H(q)) = (sum p^2/H + sum log|H|)/2 with the reference's two
  // star-ordered sums (:353-363; rhmc_mh.hpp kinetic()): every lane forms its
  // star's terms, the chain's sums read them in star order.
  static __device__ __forceinline__ double kinetic(double f, double pf, double px, double py,
                                                   bool own, int K, const Consts& c) {
    double hff, hxx;
    metric_pair(own ? f : 1.0, c, hff, hxx);
    const double a0 = pf * pf / hff, a1 = px * px / hxx, a2 = py * py / hxx;
    const double b0 = log(fabs(hff)), b1 = log(fabs(hxx));
    const int base = lane_id() & 32;
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < K; ++k) {  // K is wave-uniform
      t1 += __shfl(a0, base + k, kWave);
      t1 += __shfl(a1, base + k, kWave);
      t1 += __shfl(a2, base + k, kWave);
    }
    for (int k = 0; k < K; ++k) {
      const double l0 = __shfl(b0, base + k, kWave), l1 = __shfl(b1, base + k, kWave);
      t2 += l0;
      t2 += l1;
      t2 += l1;
    }
    return (t1 + t2) / 2.0;
  }
};

// A chain's lane bookkeeping, recomputed from a volatile lane id wherever it
// is needed: held across the step loop it would spill (leapfrog_pk does the
// same for its output index).
struct MhPkIds {
  int m;          // lane in the chain's half
  int slot;       // the chain's LDS slot in the workgroup
  int64_t chr;    // the chain (ragged tail: the wave's first chain)
  bool real;      // a chain of the batch (not a ragged-tail mirror)
};
template <int CPW, int LPC>
__device__ __forceinline__ MhPkIds mh_ids(int64_t n) {
  int lid;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
  const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / kWave) + wib;
  const int h = lid / LPC;
  MhPkIds r;
  r.m = lid % LPC;
  r.slot = wib * CPW + h;
  const int64_t ch = CPW * wave + h;
  r.real = ch < n;
  r.chr = r.real ? ch : CPW * wave;
  return r;
}

// The chain's star table from q [n][3K] (lanes without a star: 1, 0, 0).
template <class PK>
__device__ __forceinline__ void mh_pk_load(const double* q, const MhPkIds& id, int K,
                                           KRStar* tab) {
  const bool own = id.m < K;
  const int64_t e = id.chr * 3 * K + 3 * (own ? id.m : 0);
  KRStar s;
  s.f = own ? q[e] : 1.0;
  s.x = own ? q[e + 1] : 0.0;
  s.y = own ? q[e + 2] : 0.0;
  s.pad = flux_fold(s.f);
  // the table holds PK::NSTAR < 32 entries: lanes K .. NSTAR - 2 write the
  // placeholder, lanes past them read entry NSTAR - 2 (the last is E0's)
  if (id.m < PK::NSTAR - 1) tab[id.m] = s;
}

// Workgroup prologue shared by the two kernels: exp table, image; returns the
// image and sets the chain's LDS star table / factor tables.
template <class PK, int IMG>
__device__ __forceinline__ float* mh_pk_stage(double* lds, const float* Df) {
  const int W = blockDim.x / kWave;
  exp_tab_fill(lds);
  float* simg = reinterpret_cast<float*>(lds + kExpTab + PK::star_doubles(W) +
                                         (size_t)W * PK::CPW * PK::tab_doubles());
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x)
    simg[PK::img_index(e / IMG, e % IMG)] = Df[e];
  __syncthreads();
  return simg;
}

// V(q) of every chain (the MH loop's starting V, carried from then on).
template <int IMG, int KMAX>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
mh_pk_v0(MhKArgs a, double* V) {
  using MP = MhPK<IMG, KMAX>;
  using PK = typename MP::PK;
  extern __shared__ double lds[];
  const float* simg = mh_pk_stage<PK, IMG>(lds, a.Df);
  const int W = blockDim.x / kWave;
  const int64_t wave =
      (int64_t)blockIdx.x * W + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  if (PK::CPW * wave >= a.n) return;
  const MhPkIds id = mh_ids<PK::CPW, PK::LPC>(a.n);
  KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + id.slot * PK::NSTAR;
  double* rtab = lds + kExpTab + PK::star_doubles(W) +
                 (size_t)id.slot * PK::tab_doubles();
  mh_pk_load<PK>(a.q, id, a.K, tab);
  const LeanConsts lc = lean_consts(a.c);
  const double v = MP::potential(lds, simg, tab, rtab, a.K, a.f_pos, a.c, lc);
  if (id.real && id.m == 0) V[id.chr] = v;
}

// A kernel argument read at its use (a volatile load from the kernarg
// segment), so that the values needed after the step loop are not held in
// SGPRs across it (its SGPR pressure spills into VGPR lanes).
template <class T>
__device__ __forceinline__ T karg(const T& field) {
  return *(const volatile T*)&field;
}

// One MH iteration `it` of every chain in one launch: momentum draw, T0 / E0
// and the start-of-iteration records, n_steps steps, V(q') from the star
// table the step loop leaves, T(q', p'), the accept test; q and V (the
// carried V(q)) updated in place on accept.  One launch per iteration: a
// loop over iterations inside the kernel would hoist the draw's and the
// potential's constants into registers that stay live across the step loop
// (which already runs at the VGPR limit) and spill it.
template <int IMG, int KMAX>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
mh_pk_iter(MhKArgs a, int it, double* V) {
  using MP = MhPK<IMG, KMAX>;
  using PK = typename MP::PK;
  extern __shared__ double lds[];
  const float* simg = mh_pk_stage<PK, IMG>(lds, a.Df);
  const int W = blockDim.x / kWave;
  const int64_t wave =
      (int64_t)blockIdx.x * W + __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
  if (PK::CPW * wave >= a.n) return;
  const Consts& c = a.c;
  const LeanConsts lc = lean_consts(c);
  const int K = a.K;
  const int d = 3 * K;
  double f[1], x[1], y[1], pf[1], px[1], py[1];
  {
    const MhPkIds id = mh_ids<PK::CPW, PK::LPC>(a.n);
    KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + id.slot * PK::NSTAR;
    const bool own = id.m < K;
    mh_pk_load<PK>(a.q, id, K, tab);
    wave_lds_sync();
    const KRStar s0 = tab[id.m < PK::NSTAR - 2 ? id.m : PK::NSTAR - 2];
    f[0] = s0.f;
    x[0] = s0.x;
    y[0] = s0.y;
    const int64_t r = (int64_t)it * a.n + id.chr;
    double hff, hxx;
    metric_pair(f[0], c, hff, hxx);
    double z0 = 0.0, z1 = 0.0, z2 = 0.0;
    if (own) {
      const int idx = 3 * id.m;
      if (a.z) {
        z0 = a.z[r * d + idx];
        z1 = a.z[r * d + idx + 1];
        z2 = a.z[r * d + idx + 2];
      } else {
        z0 = philox_normal(a.seed, id.chr, it, idx);
        z1 = philox_normal(a.seed, id.chr, it, idx + 1);
        z2 = philox_normal(a.seed, id.chr, it, idx + 2);
      }
    }
    pf[0] = z0 * sqrt(hff);  // u_sample(d) * np.sqrt(H_diag) (:1022)
    px[0] = z1 * sqrt(hxx);
    py[0] = z2 * sqrt(hxx);
    const double V0 = V[id.chr];
    const double T0 = MP::kinetic(f[0], pf[0], px[0], py[0], own, K, c);
    const double E0 = V0 + T0;
    if (id.m == PK::LPC - 1) tab[PK::NSTAR - 1].pad = E0;  // the last entry: never a star (K <= KMAX)
    if (id.real) {
      if (a.q_chain && own) {
        a.q_chain[r * d + 3 * id.m] = f[0];
        a.q_chain[r * d + 3 * id.m + 1] = x[0];
        a.q_chain[r * d + 3 * id.m + 2] = y[0];
      }
      if (id.m == 0) {
        if (a.V_chain) a.V_chain[r] = V0;
        if (a.T_chain) a.T_chain[r] = T0;
        if (a.E_chain) a.E_chain[r] = E0;
      }
    }
  }
  {
    const MhPkIds id = mh_ids<PK::CPW, PK::LPC>(a.n);
    KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + id.slot * PK::NSTAR;
    double* rtab = lds + kExpTab + PK::star_doubles(W) +
                   (size_t)id.slot * PK::tab_doubles();
    bool own[1];
    own[0] = id.m < K;
    int it_p = 0, it_q = 0;
    unsigned st = 0u;
    auto grad = [&](const double (&)[1], const double (&)[1], double (&gf)[1], double (&gx)[1],
                    double (&gy)[1]) {
      PK::gradient(lds, simg, tab, rtab, K, c, lc, gf[0], gx[0], gy[0]);
    };
    km_steps<1, decltype(grad), true>(f, x, y, pf, px, py, own, tab, a.n_steps,
                                      (double)(IMG - 1), c, lc, grad, it_p, it_q, st);
  }
  const int64_t n = karg(a.n);
  const MhPkIds id = mh_ids<PK::CPW, PK::LPC>(n);
  KRStar* tab = reinterpret_cast<KRStar*>(lds + kExpTab) + id.slot * PK::NSTAR;
  double* rtab = lds + kExpTab + PK::star_doubles(W) +
                 (size_t)id.slot * PK::tab_doubles();
  const bool own = id.m < K;
  const double E0 = tab[PK::NSTAR - 1].pad;
  const double V1 = MP::potential(lds, simg, tab, rtab, K, karg(a.f_pos), c, lc);  // tab: q'
  const KRStar s1 = tab[own ? id.m : 0];
  const double dE = (V1 + MP::kinetic(s1.f, pf[0], px[0], py[0], own, K, c)) - E0;
  const int64_t r = (int64_t)it * n + id.chr;
  const double* u = karg(a.u);
  const double uu = u ? u[r] : philox_uniform(karg(a.seed), id.chr, it);
  const bool acc = (dE < 0.0) || (log(uu) < -dE);  // :1076
  if (id.real) {
    if (acc && own) {
      double* q = karg(a.q);
      const int64_t e = id.chr * d + 3 * id.m;
      q[e] = s1.f;
      q[e + 1] = s1.x;
      q[e + 2] = s1.y;
    }
    if (id.m == 0) {
      if (acc) V[id.chr] = V1;
      int32_t* accept = karg(a.accept);
      if (accept) accept[r] = acc ? 1 : 0;
    }
  }
}

}  // namespace rhmc
