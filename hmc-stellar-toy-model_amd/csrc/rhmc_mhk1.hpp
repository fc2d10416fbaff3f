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
  int n_iter, n_steps, f_pos, pad;
  unsigned long long seed;
  Consts c;
};

template <int IMG, int WIN, typename DT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
mh_k1_tiledr(MhK1Args a) {
  using TL = TiledR<IMG, WIN, DT>;
  extern __shared__ double lds[];
  DT* simg = reinterpret_cast<DT*>(lds + kExpTab);
  const DT* gimg;
  if constexpr (sizeof(DT) == sizeof(float)) gimg = reinterpret_cast<const DT*>(a.Df);
  else gimg = reinterpret_cast<const DT*>(a.D);
  const Consts& c = a.c;
  const int W = blockDim.x / kWave;
  for (int e = threadIdx.x; e < IMG * IMG; e += blockDim.x) {
    const int r = e / IMG, cc = e - (e / IMG) * IMG;
    simg[r * TL::P + cc] = gimg[e];
  }
  exp_tab_fill(lds);
  __syncthreads();
  const int64_t wave = (int64_t)blockIdx.x * W + (threadIdx.x / kWave);
  if (TL::CPW * wave >= a.n) return;
  const int lane = lane_id();
  const int64_t ch = TL::CPW * wave + lane / TL::LPC;
  const bool real = ch < a.n;                      // ragged tail: mirror the wave's first chain
  const int64_t chr = real ? ch : TL::CPW * wave;
  const bool writer = real && (lane % TL::LPC) == 0;

  // sum over the image of B - D ln B = IMG^2 B - ln B sum D (the V of a
  // star-free image; the window sum corrects it)
  double sd = 0.0;
  for (int e = lane; e < IMG * IMG; e += kWave) sd += (double)simg[(e / IMG) * TL::P + e % IMG];
  const double lnB = log_pos(c.B);
  const double sum_B = (double)(IMG * IMG) * c.B - lnB * wave_sum(sd);
  double f = a.q[3 * chr], x = a.q[3 * chr + 1], y = a.q[3 * chr + 2];
  const LeanConsts lc = lean_consts(c);
  typename TL::Cache cache;
  TL::init(cache);
  // V(q) (:294-330): infinite outside the support, else window sum + prior
  // (the window sum is evaluated either way: no divergence inside a wave)
  auto potential = [&](double f_, double x_, double y_) {
    double v = sum_B + TL::potential_window(lds, simg, cache, f_, x_, y_, c, lc, lnB);
    if (c.use_prior) v += c.alpha * log(f_) + c.vprior;   // :326, :329-330
    if (((a.f_pos & RHMC_V_FLUX_WALL) && f_ < c.f_lim) ||
        (!(a.f_pos & RHMC_V_NO_POSCHECK) &&
         (x_ < -1.0 || x_ > (double)(IMG + 1) || y_ < -1.0 || y_ > (double)(IMG + 1))))
      v = INFINITY;
    return v;
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
      const int64_t r = (int64_t)it * a.n + chr;
      const double q3p[3] = {f1, x1, y1};
      const double p3p[3] = {pf, px, py};
      const double dE = (V1 + kinetic(q3p, p3p, 1, c)) - E0;
      const double uu = a.u ? a.u[r] : philox_uniform(a.seed, chr, it);
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
    const int64_t r = (int64_t)nx * a.n + chr;
    double hff, hxx;
    metric_pair(f, c, hff, hxx);
    double z0, z1, z2;
    if (a.z) {
      z0 = a.z[3 * r];
      z1 = a.z[3 * r + 1];
      z2 = a.z[3 * r + 2];
    } else {
      z0 = philox_normal(a.seed, chr, nx, 0);
      z1 = philox_normal(a.seed, chr, nx, 1);
      z2 = philox_normal(a.seed, chr, nx, 2);
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
    k1_steps(f1, x1, y1, pf, px, py, a.n_steps, (double)(IMG - 1), c, lc,
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

}  // namespace rhmc
