// rhmc_mhk1.hpp — the whole MH outer loop (multi_gym.run_RHMC move-0 branch,
// sampler_RHMC.py:1018-1083) for one star in ONE launch on the register-window
// kernel (rhmc_tiledr.hpp): 16 lanes per chain, 4 chains per wave64, the
// chain's state, its window pixels and V(q) in registers across iterations.
//
// Per iteration (the same arithmetic as mh_begin_kernel / leapfrog /
// energy / mh_end_kernel of rhmc_mh.hpp, without their launches and HBM round
// trips):
//   p = z sqrt(H(q))                      (:1021-1022)
//   T0 = T(p, H(q)), E0 = V(q) + T0       (:1025-1027; V(q) carried)
//   n_steps x RHMC_single_step            (:1053-1054, rhmc_k1step.hpp)
//   V(q'): infinite outside the support (:303-317), else
//          sum_image (B - D ln B) + the window's (Lambda - B) - D (ln Lambda - ln B)
//          (TiledR::potential_window; outside the window Lambda == B) + prior
//   accept when dE < 0 or ln u < -dE      (:1072-1083)
// Randoms: host arrays z / u (exact parity with the reference's NumPy stream)
// or Philox keyed by (seed, chain, iteration) as in rhmc_mh.hpp.
#pragma once
#include "rhmc_mh.hpp"
#include "rhmc_tiledr.hpp"

namespace rhmc {

struct MhK1Args {
  double* q;              // [n][3] current state, updated in place
  const double* D;
  const float* Df;        // D in fp32 when exact, else nullptr
  const double* z;        // nullable [n_iter][n][3]
  const double* u;        // nullable [n_iter][n]
  double* q_chain;        // nullable [n_iter][n][3]
  double* E_chain;        // nullable [n_iter][n]
  double* V_chain;        // nullable [n_iter][n]
  double* T_chain;        // nullable [n_iter][n]
  int32_t* accept;        // nullable [n_iter][n]
  int64_t n;
  int n_iter, n_steps, f_pos;
  int it0;                // index of the launch's first iteration (RNG keys, record rows)
  unsigned long long seed;
  Consts c;
};

// Workgroup prologue of the one-star register-window kernels: the image into
// LDS (row pitch TL::P) and the exp table.
template <class TL, typename DT>
__device__ __forceinline__ DT* k1_stage_image(double* lds, const DT* gimg) {
  constexpr int IMG = TL::P - 1;
  DT* simg = reinterpret_cast<DT*>(lds + kExpTab);
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    simg[r * TL::P + cc] = gimg[e];
  }
  exp_tab_fill(lds);
  __syncthreads();
  return simg;
}

// sum over the image of B - D ln B = IMG^2 B - ln B sum D (the V of a
// star-free image; the window sum corrects it), lnB = log_pos(B).  Wave-wide.
template <class TL, typename DT>
__device__ __forceinline__ double k1_background_V(const DT* simg, double B, double lnB) {
  constexpr int IMG = TL::P - 1;
  double sd = 0.0;
  for (int e = lane_id(); e < IMG * IMG; e += kWave) sd += (double)simg[(e / IMG) * TL::P + e % IMG];
  return (double)(IMG * IMG) * B - lnB * wave_sum(sd);
}

// V(q) of one star (sampler_RHMC.py:294-330): the background V plus the
// window's correction plus the prior, infinite outside the support (f_pos:
// RHMC_V_FLUX_WALL / RHMC_V_NO_POSCHECK).  The window sum is evaluated either
// way (no divergence inside a chain's lane group).
template <class TL, typename DT>
__device__ __forceinline__ double k1_potential(const double* lds, const DT* simg,
                                               typename TL::Cache& cache, double f, double x,
                                               double y, int f_pos, double sum_B, double lnB,
                                               const Consts& c, const LeanConsts& lc) {
  constexpr int IMG = TL::P - 1;
  double v = sum_B + TL::potential_window(lds, simg, cache, f, x, y, c, lc, lnB);
  if (c.use_prior) v += c.alpha * log(f) + c.vprior;     // :326, :329-330
  if (((f_pos & RHMC_V_FLUX_WALL) && f < c.f_lim) ||
      (!(f_pos & RHMC_V_NO_POSCHECK) &&
       (x < -1.0 || x > (double)(IMG + 1) || y < -1.0 || y > (double)(IMG + 1))))
    v = INFINITY;
  return v;
}

template <int IMG, int WIN, typename DT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
mh_k1_tiledr(MhK1Args a) {
  using TL = TiledR<IMG, WIN, DT>;
  extern __shared__ double lds[];
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const DT* simg = k1_stage_image<TL>(lds, gimg);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n) return;
  const int lane = lane_id();
  const int64_t ch = TL::CPW * wave + lane / TL::LPC;
  const bool real = ch < a.n;                      // ragged tail: mirror the wave's first chain
  const int64_t chr = real ? ch : TL::CPW * wave;
  const bool writer = real && (lane % TL::LPC) == 0;

  const double lnB = log_pos(c.B);
  const double sum_B = k1_background_V<TL>(simg, c.B, lnB);
  double f = a.q[3 * chr], x = a.q[3 * chr + 1], y = a.q[3 * chr + 2];
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  auto potential = [&](double f_, double x_, double y_) {
    return k1_potential<TL>(lds, simg, cache, f_, x_, y_, a.f_pos, sum_B, lnB, c, lc);
  };
  // One potential evaluation in the code (it is the bulk of the kernel's
  // code): pass it = -1 evaluates V(q) of the starting state, pass it >= 0
  // evaluates V(q') of iteration it's proposal and decides it, then the next
  // iteration is drawn and integrated.
  double V0 = 0.0, E0 = 0.0;
  double f1 = f, x1 = x, y1 = y, pf = 0.0, px = 0.0, py = 0.0;
  for (int it = -1; it < a.n_iter; ++it) {
    const double V1 = potential(f1, x1, y1);
    if (it < 0) {
      V0 = V1;
    } else {
      const int gi = a.it0 + it;                   // the run's iteration index
      const int64_t r = (int64_t)gi * a.n + chr;
      const double q3p[3] = {f1, x1, y1};
      const double p3p[3] = {pf, px, py};
      const double dE = (V1 + kinetic(q3p, p3p, 1, c)) - E0;
      const double uu = a.u ? a.u[r] : philox_uniform(a.seed, chr, gi);
      const bool acc = (dE < 0.0) || (log(uu) < -dE);  // :1076
      if (acc) {
        f = f1;
        x = x1;
        y = y1;
        V0 = V1;
      }
      if (writer && a.accept) a.accept[r] = acc ? 1 : 0;
    }
    const int nx = it + 1;
    if (nx == a.n_iter) break;
    const int gn = a.it0 + nx;                     // the run's iteration index
    const int64_t r = (int64_t)gn * a.n + chr;
    double hff, hxx;
    metric_pair(f, c, hff, hxx);
    double z0, z1, z2;
    if (a.z) {
      z0 = a.z[3 * r];
      z1 = a.z[3 * r + 1];
      z2 = a.z[3 * r + 2];
    } else {
      z0 = philox_normal(a.seed, chr, gn, 0);
      z1 = philox_normal(a.seed, chr, gn, 1);
      z2 = philox_normal(a.seed, chr, gn, 2);
    }
    pf = z0 * sqrt(hff);                           // :1022
    px = z1 * sqrt(hxx);
    py = z2 * sqrt(hxx);
    const double q3[3] = {f, x, y};
    const double p3[3] = {pf, px, py};
    const double T0 = kinetic(q3, p3, 1, c);
    E0 = V0 + T0;
    if (writer) {
      if (a.q_chain) {
        a.q_chain[3 * r] = f;
        a.q_chain[3 * r + 1] = x;
        a.q_chain[3 * r + 2] = y;
      }
      if (a.V_chain) a.V_chain[r] = V0;
      if (a.T_chain) a.T_chain[r] = T0;
      if (a.E_chain) a.E_chain[r] = E0;
    }
    f1 = f;
    x1 = x;
    y1 = y;
    int it_p = 0, it_q = 0;
    unsigned st = 0u;
    k1_steps<false, TL::LPC>(f1, x1, y1, pf, px, py, a.n_steps, (double)(IMG - 1), c, lc,
             [&](double f_, double x_, double y_, double& gf, double& gx, double& gy) {
               TL::gradient(lds, simg, cache, f_, x_, y_, c, lc, gf, gx, gy);
             },
             it_p, it_q, st);
  }
  if (writer) {
    a.q[3 * ch] = f;
    a.q[3 * ch + 1] = x;
    a.q[3 * ch + 2] = y;
  }
}

// V and T of one-star chains (the energy kernel's job, sampler_RHMC.py
// :294-363) on the register-window layout: 16 lanes per chain, V from the
// window correction (784 logs per chain instead of the image's 2304).
struct EnergyK1Args {
  const double* q;
  const double* p;   // nullable: no T
  double* V;         // nullable: no V
  double* T;
  const double* D;
  const float* Df;
  int64_t n;
  int f_pos, pad;
  Consts c;
};

template <int IMG, typename DT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
energy_k1_tiledr(EnergyK1Args a) {
  using TL = TiledR<IMG, 28, DT>;
  extern __shared__ double lds[];
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const DT* simg = k1_stage_image<TL>(lds, gimg);
  const Consts& c = a.c;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n) return;
  const int lane = lane_id();
  const int64_t ch = TL::CPW * wave + lane / TL::LPC;
  const bool real = ch < a.n;                      // ragged tail: mirror the wave's first chain
  const int64_t chr = real ? ch : TL::CPW * wave;
  const bool writer = real && (lane % TL::LPC) == 0;
  const double f = a.q[3 * chr], x = a.q[3 * chr + 1], y = a.q[3 * chr + 2];
  if (a.T) {  // T(p, H(q)) (:353-363), the energy kernel's expression
    const double pf = a.p[3 * chr], px = a.p[3 * chr + 1], py = a.p[3 * chr + 2];
    double hff, hxx;
    metric_pair(f, c, hff, hxx);
    const double t1 = pf * pf / hff + px * px / hxx + py * py / hxx;
    const double t2 = log(fabs(hff)) + log(fabs(hxx)) + log(fabs(hxx));
    if (writer) a.T[ch] = (t1 + t2) / 2.0;
  }
  if (!a.V) return;
  const double lnB = log_pos(c.B);
  const double sum_B = k1_background_V<TL>(simg, c.B, lnB);
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  const double v = k1_potential<TL>(lds, simg, cache, f, x, y, a.f_pos, sum_B, lnB, c, lc);
  if (writer) a.V[ch] = v;
}

}  // namespace rhmc
