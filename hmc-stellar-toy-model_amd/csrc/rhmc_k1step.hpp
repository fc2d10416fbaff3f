// rhmc_k1step.hpp — the step loop of RHMC_single_step (sampler_RHMC.py:522-566)
// for one star, shared by the single-star kernels: every lane of a chain's
// lane group holds the same (q, p) and runs the same scalar code; only the
// gradient's pixel sum is spread over the group (the GRAD functor).
//
// The flux f changes only inside the q-loop, so every metric quantity a step
// needs at its current f — 1/H_ff, H_xx's s, dtaudq's coefficient, the dphidq
// metric term and the prior term — is computed once per distinct f
// (FluxMetric) and reused by the gradient, the next p-loop and the q-loop's
// q_tmp_s evaluation: three reciprocals per step plus one per q iteration,
// instead of six plus one.
#pragma once
#include "rhmc.h"
#include "rhmc_wave.hpp"

#ifdef RHMC_MARKS
#define RHMC_MARK(n) asm volatile("s_setprio " #n ::: "memory")
#else
#define RHMC_MARK(n)
#endif
namespace rhmc {

// Fixed-point iterations evaluated per pass (one branch per pass).
#ifndef RHMC_SPEC_P
#define RHMC_SPEC_P 2
#endif
#ifndef RHMC_SPEC_Q
#define RHMC_SPEC_Q 2
#endif
// RHMC_STATUS_NEAR_WALL in the one-star step loop: 2 = flux wall and image
// edges, 1 = flux wall only, 0 = off.
#ifndef RHMC_NEAR_WALL
#define RHMC_NEAR_WALL 2
#endif
constexpr int kSpecP = RHMC_SPEC_P;
constexpr int kSpecQ = RHMC_SPEC_Q;

// 1/d to within ~11 ulp (v_rcp_f64 is accurate to ~2^-24; one Newton step).
__device__ __forceinline__ double rcp_nr1(double d) {
  const double r = __builtin_amdgcn_rcp(d);
  return fma(r, fma(-d, r, 1.0), r);
}

struct FluxMetric {
  double A;      // f/g_ff2 + (B/g0)/g_ff = 1/H_ff                       (:290)
  double s;      // u/g1 + (B/g2) u^2, u = 1/max(f, f_low); H_xx = g_xx/s (:267-273)
  double coef;   // -H_ff'/H_ff^2 = (A/(f + (B/g0)/g_ff))^2               (:479)
  double mterm;  // (H_ff'/H_ff + 2 H_xx'/H_xx)/2                        (:459-463)
  double prior;  // alpha/f (use_prior)                                    (:408-409)
};

// Arguments of the single-star kernels (register-window, lane-group).
struct LeapArgsK1 {
  double* q;
  double* p;
  int32_t* fp_iters;
  int32_t* status;
  const double* D;
  const float* Df;   // D in fp32 when exact (ctx->img_f32), else nullptr
  int64_t n_chains;
  int n_steps, rows, cols, pad;
  Consts c;
};

__device__ __forceinline__ FluxMetric flux_metric(double f, const Consts& c,
                                                  const LeanConsts& l) {
  FluxMetric m;
  m.A = fma(f, l.inv_gff2, l.c0);
  const double ib = rcp_nr(f + l.c0);
  const double t = m.A * ib;
  m.coef = t * t;
  const bool low = f < l.f_low;
  const double fl = low ? l.f_low : f;
  const double u = rcp_nr(fl);
  m.s = u * fma(l.Bg2, u, l.inv_g1);
  const double t2 = low ? 0.0 : (u * u) * fma(l.two_Bg2, u, l.inv_g1) * rcp_nr(m.s);
  const double t1 = -m.A * (ib * ib);
  m.mterm = (t1 + 2.0 * t2) / 2.0;
  m.prior = c.use_prior ? c.alpha * (low ? rcp_nr(f) : u) : 0.0;
  return m;
}

// Lane-parallel q-loop passes (QL = 16 lanes per chain, one DPP row).
#ifndef RHMC_QPAR
#define RHMC_QPAR 1
#endif
constexpr bool kQPar = RHMC_QPAR;

__device__ __forceinline__ double row_shr1(double v) {  // lane l of a 16-lane row gets lane l - 1
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, 0x111, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0x111, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The q-loop (:538-545) with the chain's 16 lanes evaluating 8 iterations at
// once.  The flux iterates are an affine recurrence F' = bf F + cf, so lane j
// (j = lane % 8; lanes j and j + 8 duplicate) gets F_j = T^j(F_0) by binary
// powering of T (three conditional FMAs; rounding differs from the sequential
// chain by a few ulp, like the affine form itself), then F_{j+1} = T(F_j) and
// the position iterates X_{j+1}, Y_{j+1} = b g(F_j) + c; X_j, Y_j come from
// lane j - 1 by a DPP row shift.  The reference's test for iteration j
// (np.max |q_j - q_{j+1}| > delta, NaN stops, counter_max) is evaluated in lane
// j; a ballot gives the first stopping iteration k of each chain, whose state
// q_{k+1} is read from lane k (ds_bpermute).  A chain with no stop among the 8
// takes q_8 and runs another pass.  The iterates agree with the sequential
// loop's (and the reference's divide-form ones) to a few ulp, so the counts and
// cap status are the reference's except where an iterate's max |dq| lies
// within those few ulp of delta: there the loop can stop one iteration
// earlier or later (tests/test_gpu_delta_edge.py bounds that case).  One rcp
// chain per 8 iterations instead of per iteration.
__device__ __forceinline__ void q_loop_lanes16(double& f, double& x, double& y, double bf,
                                               double cf, double bx, double cx, double by,
                                               double cy, const Consts& c, const LeanConsts& lc,
                                               int& it_q, unsigned& st) {
  const int lane = lane_id();
  const int j = lane & 7;
  const int gsh = lane & 48;  // first lane of the chain's row
  // T^2, T^4 (wave-uniform per chain)
  const double b2 = bf * bf, c2 = fma(bf, cf, cf);
  const double b4 = b2 * b2, c4 = fma(b2, c2, c2);
  int n = 0;
  bool done = false, more = false;
  do {
    double Fj = f;
    if (j & 1) Fj = fma(bf, Fj, cf);
    if (j & 2) Fj = fma(b2, Fj, c2);
    if (j & 4) Fj = fma(b4, Fj, c4);
    const double Fj1 = fma(bf, Fj, cf);
    const double fl = (Fj < lc.f_low) ? lc.f_low : Fj;
    const double u = rcp_nr1(fl);
    const double g = u * fma(lc.Bg2, u, lc.inv_g1);
    const double Xj1 = fma(bx, g, cx), Yj1 = fma(by, g, cy);
    double Xj = row_shr1(Xj1), Yj = row_shr1(Yj1);
    if (j == 0) {
      Xj = x;
      Yj = y;
    }
    const double a0 = fabs(Fj - Fj1), a1 = fabs(Xj - Xj1), a2 = fabs(Yj - Yj1);
    const double sum = a0 + a1 + a2;
    const bool go = (fmax(fmax(a0, a1), a2) > c.delta) && (sum == sum);
    const bool stop = !go || (n + j + 1 >= c.counter_max);
    const unsigned long long bal = __builtin_amdgcn_ballot_w64(stop);
    const unsigned bits = (unsigned)(bal >> gsh) & 0xFFu;
    const int k = bits ? (int)__builtin_ctz(bits) : 7;
    const int src = gsh + k;
    const double nf = __shfl(Fj1, src, kWave), nx = __shfl(Xj1, src, kWave),
                 ny = __shfl(Yj1, src, kWave);
    const int ngo = __shfl((int)go, src, kWave);
    if (!done) {
      f = nf;
      x = nx;
      y = ny;
      n += k + 1;
      more = ngo != 0;
      done = bits != 0u;
    }
  } while (__builtin_amdgcn_ballot_w64(!done) != 0);
  it_q += n;
  if (more) st |= RHMC_STATUS_QLOOP_CAP;
}

// n_steps steps on (f, x, y, pf, px, py).  grad(f, x, y, gf, gx, gy) returns
// the pixel part of dphidq: gf = -sum psf (D/L - 1), gx, gy (:404-406).
// PROF (tools only): per-phase cycle sums, prof[0] gradient, prof[1] kicks +
// reflection + p-loop, prof[2] q-loop, prof[3] flux metric + closing update.
// QL: lanes per chain (16: the q-loop runs 8 iterations per pass across them).
template <bool PROF = false, int QL = 1, class GRAD>
__device__ __forceinline__ void k1_steps(double& f, double& x, double& y, double& pf,
                                         double& px, double& py, int n_steps, double edge,
                                         const Consts& c, const LeanConsts& lc, GRAD grad,
                                         int& it_p, int& it_q, unsigned& st,
                                         long long* prof = nullptr) {
  const double hdt = c.hdt;
  FluxMetric fm = flux_metric(f, c, lc);
  long long t0 = 0;
  // phase boundary: fenced clock read; the cycles since the last boundary go
  // to bucket `close` (a constant at every call site)
  auto mark = [&](int close) {
    if constexpr (PROF) {
      __builtin_amdgcn_sched_barrier(0);
      const long long t1 = clock64();
      if (t0) prof[close] += t1 - t0;
      t0 = t1;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int s = 0;; ++s) {
    double gf, gx, gy;
    mark(3);
    RHMC_MARK(1);
    grad(f, x, y, gf, gx, gy);
    RHMC_MARK(2);
    mark(0);
    if (c.use_prior) gf += fm.prior;               // :408-409
    gf += fm.mterm;                                // :459-463
    if (s > 0) {
      pf = pf - hdt * gf;                          // :551
      px = px - hdt * gx;
      py = py - hdt * gy;
      if (f < c.f_lim) {                           // :554-564
        pf = -pf;
        st |= RHMC_STATUS_REFLECT_F;
        if (RHMC_NEAR_WALL >= 1 && f >= c.near_f) st |= RHMC_STATUS_NEAR_WALL;
      }
      if (x < 0.0 || x > edge) {
        px = -px;
        st |= RHMC_STATUS_REFLECT_XY;
        if (RHMC_NEAR_WALL >= 2 && near_edge(x, edge)) st |= RHMC_STATUS_NEAR_WALL;
      }
      if (y < 0.0 || y > edge) {
        py = -py;
        st |= RHMC_STATUS_REFLECT_XY;
        if (RHMC_NEAR_WALL >= 2 && near_edge(y, edge)) st |= RHMC_STATUS_NEAR_WALL;
      }
    }
    if (s == n_steps) {
      mark(1);
      break;
    }
    pf = pf - hdt * gf;                            // :525
    px = px - hdt * gx;
    py = py - hdt * gy;
    {                                              // :528-535 (dtaudq is 0 on x, y)
      // SPEC_P iterations per pass; the state and count kept are those of the
      // first iteration whose test stops the reference's loop.
      const double rho = pf, hc = hdt * (fm.coef * 0.5);
      int n = 0;
      bool more;
      do {
        double P[kSpecP + 1];
        bool go[kSpecP];
        P[0] = pf;
#pragma unroll
        for (int k = 0; k < kSpecP; ++k) {
          P[k + 1] = fma(-hc, P[k] * P[k], rho);
          go[k] = fabs(P[k] - P[k + 1]) > c.delta;
        }
        int take = kSpecP;
        double sel = P[kSpecP];
        more = go[kSpecP - 1];
#pragma unroll
        for (int k = kSpecP - 1; k >= 0; --k) {
          if (!go[k] || n + k + 1 >= c.counter_max) {
            take = k + 1;
            sel = P[k + 1];
            more = go[k];
          }
        }
        pf = sel;
        n += take;
      } while (more && n < c.counter_max);
      it_p += n;
      if (more) st |= RHMC_STATUS_PLOOP_CAP;
      RHMC_MARK(3);
    }
    mark(1);
    {                                              // :538-545
      // q_{n+1} = q_s + hdt (p/H(q_s) + p/H(q_n)) with 1/H_ff(f) = f/g_ff2 + c0
      // and 1/H_xx(f) = g(f)/g_xx, g = u/g1 + (B/g2) u^2: affine in f and g.
      // The flux iterates are an affine recurrence, so SPEC_Q iterations per
      // pass cost one dependent chain (their reciprocals overlap) and one branch.
      const double ihxx_s = fm.s * lc.inv_gxx;
      const double bf = hdt * (pf * lc.inv_gff2), cf = f + hdt * (pf * fm.A + pf * lc.c0);
      const double bx = hdt * (px * lc.inv_gxx), cx = x + hdt * (px * ihxx_s);
      const double by = hdt * (py * lc.inv_gxx), cy = y + hdt * (py * ihxx_s);
      if constexpr (QL == 16 && kQPar) {
        q_loop_lanes16(f, x, y, bf, cf, bx, cx, by, cy, c, lc, it_q, st);
      } else {
      bool more;
      int n = 0;
      do {
        double F[kSpecQ + 1], X[kSpecQ + 1], Y[kSpecQ + 1];
        bool go[kSpecQ];
        F[0] = f;
        X[0] = x;
        Y[0] = y;
#pragma unroll
        for (int k = 0; k < kSpecQ; ++k) F[k + 1] = fma(bf, F[k], cf);
#pragma unroll
        for (int k = 0; k < kSpecQ; ++k) {
          const double fl = (F[k] < lc.f_low) ? lc.f_low : F[k];
          const double u = rcp_nr1(fl);
          const double g = u * fma(lc.Bg2, u, lc.inv_g1);
          X[k + 1] = fma(bx, g, cx);
          Y[k + 1] = fma(by, g, cy);
          const double a0 = fabs(F[k] - F[k + 1]), a1 = fabs(X[k] - X[k + 1]),
                       a2 = fabs(Y[k] - Y[k + 1]);
          const double sum = a0 + a1 + a2;
          // dq = np.max(...) > delta, NaN stops the loop
          go[k] = (fmax(fmax(a0, a1), a2) > c.delta) && (sum == sum);
        }
        int take = kSpecQ;
        double sf = F[kSpecQ], sx = X[kSpecQ], sy = Y[kSpecQ];
        more = go[kSpecQ - 1];
#pragma unroll
        for (int k = kSpecQ - 1; k >= 0; --k) {
          if (!go[k] || n + k + 1 >= c.counter_max) {
            take = k + 1;
            sf = F[k + 1];
            sx = X[k + 1];
            sy = Y[k + 1];
            more = go[k];
          }
        }
        f = sf;
        x = sx;
        y = sy;
        n += take;
      } while (more && n < c.counter_max);
      it_q += n;
      if (more) st |= RHMC_STATUS_QLOOP_CAP;
      }
      RHMC_MARK(4);
    }
    mark(2);
    fm = flux_metric(f, c, lc);
    pf = pf - hdt * ((pf * pf) * fm.coef / 2.0);   // :548
    RHMC_MARK(5);
  }
}

}  // namespace rhmc
