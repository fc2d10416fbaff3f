// rhmc_rj.cpp — librhmc_rj.so: multi_gym.run_RHMC's reversible-jump sampler
// (sampler_RHMC.py:937-1198, moves :1200-1445) for many chains at once, native
// host code around the engine's C-ABI (include/rhmc_rj.h).
//
// One iteration l (every chain c has its own RandomState replica and star
// count K_c):
//   1. host, per chain, in parallel: g_ff2 / beta from the schedules
//      (:1010-1016), H(q) (:229-258), p = randn(3K) sqrt(H) (:1021-1022),
//      T0 (:1026), the move type (:1045) and grow / shrink (:1094, :1140)
//   2. engine: V(q) of every chain, grouped by K                  (:1025)
//   3. engine: Nsteps steps on every chain, grouped by K     (:1053, :1098)
//   4. host, jumping chains: p = -p, the proposal and its ln-acceptance
//      factor (:1099-1102; birth_death_move / split_merge_move)
//   5. engine: Nsteps steps on the jumping chains at their new K   (:1109)
//   6. engine: V(q') of every chain                          (:1069, :1117)
//   7. host: E1 = V' + T(p', H(q')), the accept uniform, accept / restore
//      (:1072-1083, :1120-1131)
// The host expressions follow the reference's operation order
// (rhmc_amd/sampler.py's _H_vec / T / moves, which tests pin to it).
#include "rhmc_rj.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cmath>
#include <cstring>
#include <exception>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "np_legacy.hpp"

namespace {

constexpr int kMaxPipes = 4;  // rhmc_rj_config::n_pipes

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

constexpr double kPi = 3.141592653589793;  // np.pi

// ------------------------------------------------------------ model helpers
// H(q) of one star (sampler.py _H_vec, sampler_RHMC.py:260-292): Hd = (H_ff,
// H_xx, H_xx).
struct Metric {
  double g_ff2, g_ff, g_xx, g0, g1, g2, B, f_low;
  void star(double f, double* Hd) const {
    const double Hf = 1. / (f / g_ff2 + (B / g0) / g_ff);
    const double fl = f < f_low ? f_low : f;
    const double s = 1. / (g1 * fl) + B / (g2 * (fl * fl));
    const double Hx = g_xx * (1. / s);
    Hd[0] = Hf;
    Hd[1] = Hx;
    Hd[2] = Hx;
  }
  void all(const double* q, int64_t d, double* Hd) const {
    for (int64_t i = 0; i < d; i += 3) star(q[i], Hd + i);
  }
};

// T(p, H) = (sum p^2 / H + sum ln|H|) / 2 with NumPy's pairwise sums (:353-363)
double kinetic(const double* p, const double* H, int64_t d, std::vector<double>& tmp) {
  tmp.resize((size_t)d);
  for (int64_t i = 0; i < d; ++i) tmp[i] = (p[i] * p[i]) / H[i];
  const double s1 = rhmc_np::pairwise_sum(tmp.data(), d);
  for (int64_t i = 0; i < d; ++i)  // a star's two position entries share H: one log
    tmp[i] = (i % 3 == 2 && H[i] == H[i - 1]) ? tmp[i - 1] : std::log(std::fabs(H[i]));
  const double s2 = rhmc_np::pairwise_sum(tmp.data(), d);
  return (s1 + s2) / 2.;
}

// RandomState.choice(k, p=w) for one value: cdf = cumsum(w) / cdf[-1], one
// uniform, searchsorted(side='right')
int64_t choice(rhmc_np::Legacy& r, const double* w, int64_t k, std::vector<double>& cdf) {
  cdf.resize((size_t)k);
  double acc = 0.;
  for (int64_t i = 0; i < k; ++i) cdf[i] = acc = acc + w[i];
  const double last = cdf[k - 1];
  for (int64_t i = 0; i < k; ++i) cdf[i] /= last;
  const double u = r.random_sample();
  return std::upper_bound(cdf.begin(), cdf.end(), u) - cdf.begin();
}

// scipy.stats.beta.logpdf / pdf: xlog1py(b-1, -x) + xlogy(a-1, x) - betaln(a, b);
// the pdf with integer exponents as products (the merge evaluates it on every
// star pair: beta_a = beta_b = 2 by default, 6 x (1 - x))
struct BetaDist {
  double a = 2., b = 2., lb = 0., inv_b = 0.;
  int ia = -1, ib = -1;  // a - 1, b - 1 when small non-negative integers
  void set(double a_, double b_) {
    a = a_;
    b = b_;
    lb = std::lgamma(a) + std::lgamma(b) - std::lgamma(a + b);
    inv_b = std::exp(-lb);
    ia = (a - 1 >= 0 && a - 1 <= 8 && a == std::floor(a)) ? (int)(a - 1) : -1;
    ib = (b - 1 >= 0 && b - 1 <= 8 && b == std::floor(b)) ? (int)(b - 1) : -1;
  }
  double logpdf(double x) const {
    const double t1 = (b - 1.0 == 0.0) ? 0.0 : (b - 1.0) * std::log1p(-x);
    const double t2 = (a - 1.0 == 0.0) ? 0.0 : (a - 1.0) * std::log(x);
    return t1 + t2 - lb;
  }
  double pdf(double x) const {
    if (!(x >= 0.0 && x <= 1.0)) return 0.0;
    if (ia >= 0 && ib >= 0) {
      double v = inv_b;
      for (int k = 0; k < ia; ++k) v *= x;
      const double y = 1.0 - x;
      for (int k = 0; k < ib; ++k) v *= y;
      return v;
    }
    return std::exp(logpdf(x));
  }
};

// ------------------------------------------------------------- thread pool
// Fork-join pool that lives for one run: the workers sleep between phases
// (spawning threads per phase cost ~3 ms per iteration at 16 threads).
class Pool {
 public:
  explicit Pool(int n) {
    try {
      for (int t = 1; t < n; ++t) th_.emplace_back([this] { worker(); });
    } catch (...) {  // a thread could not start: stop and join the ones that did
      shutdown();
      throw;
    }
  }
  ~Pool() { shutdown(); }
  int size() const { return (int)th_.size() + 1; }
  // body(i) for i in [0, n), chunks of 16, the caller works too.  An exception
  // from body (any thread) is rethrown here once every thread has left it.
  void run(int64_t n, const std::function<void(int64_t)>& body) {
    {
      std::lock_guard<std::mutex> l(mu_);
      body_ = &body;
      n_ = n;
      next_.store(0);
      busy_ = (int)th_.size();
      exc_ = nullptr;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(mu_);
    done_.wait(l, [this] { return busy_ == 0; });
    body_ = nullptr;
    if (exc_) {
      std::exception_ptr e = exc_;
      exc_ = nullptr;
      std::rethrow_exception(e);
    }
  }

 private:
  void shutdown() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
    th_.clear();
  }
  void work() {
    try {
      for (;;) {
        const int64_t b = next_.fetch_add(16);
        if (b >= n_) return;
        const int64_t e = std::min(n_, b + 16);
        for (int64_t i = b; i < e; ++i) (*body_)(i);
      }
    } catch (...) {  // keep the first; the other chunks still drain
      std::lock_guard<std::mutex> l(mu_);
      if (!exc_) exc_ = std::current_exception();
      next_.store(n_);
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> l(mu_);
      if (--busy_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int64_t)>* body_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
  std::exception_ptr exc_;
};

// ------------------------------------------------------------------- chains
struct Chain {
  rhmc_np::Legacy rng;
  std::vector<double> q, p, q0;  // state, momentum, the iteration's starting q
  int32_t K = 0, K0 = 0;
  int move = 0;                  // 0 within, 1 birth/death, 2 split/merge
  bool grow = false, dead = false;
  double E0 = 0., factor = 0.;
  std::vector<double> H, tmp, cdf;
};

struct Run {
  const rhmc_rj_physics* phys;
  rhmc_params P;
  const rhmc_rj_config* cfg;
  std::vector<Chain> ch;
  int nt;
  int Kmax;
  BetaDist beta;

  Pool* pool = nullptr;

  template <class F>
  void parallel(const std::vector<int64_t>& idx, F f) {
    const int64_t n = (int64_t)idx.size();
    if (!pool || pool->size() <= 1 || n < 32) {
      for (int64_t i = 0; i < n; ++i) f(idx[i]);
      return;
    }
    const std::function<void(int64_t)> body = [&](int64_t i) { f(idx[i]); };
    pool->run(n, body);
  }

  // chains grouped by star count in order of first appearance
  std::vector<std::pair<int32_t, std::vector<int64_t>>> groups(const std::vector<int64_t>& idx) {
    std::vector<std::pair<int32_t, std::vector<int64_t>>> g;
    std::map<int32_t, size_t> where;
    for (int64_t c : idx) {
      const int32_t K = ch[c].K;
      auto it = where.find(K);
      if (it == where.end()) {
        where[K] = g.size();
        g.push_back({K, {c}});
      } else {
        g[it->second].second.push_back(c);
      }
    }
    return g;
  }

  int energies(const std::vector<int64_t>& idx, std::vector<double>& V) {
    if (staged.energy) return energies_staged(idx, V);
    std::vector<double> qb, vb;
    for (auto& grp : groups(idx)) {
      const int32_t K = grp.first;
      const auto& cs = grp.second;
      const size_t d = 3 * (size_t)K;
      qb.resize(cs.size() * d);
      vb.assign(cs.size(), 0.);
      for (size_t i = 0; i < cs.size(); ++i) std::memcpy(&qb[i * d], ch[cs[i]].q.data(), d * 8);
      const int rc = phys->energy(phys->user, &P, qb.data(), (int64_t)cs.size(), K, cfg->f_pos,
                                  vb.data());
      if (rc != 0) return engine_fail(rc, "energy");
      for (size_t i = 0; i < cs.size(); ++i) V[cs[i]] = vb[i];
    }
    return 0;
  }

  // optional (the context path): a phase's groups staged in one pinned buffer
  // and run concurrently on several HIP streams.  buffer(user, doubles)
  // returns the staging area; launch(...) runs group g from q at off[g] and
  // p at off[g] + n[g] 3 K[g], in place.
  struct Staged {
    void* user = nullptr;
    double* (*buffer)(void* user, size_t doubles) = nullptr;
    int (*launch)(void* user, const rhmc_params* P, int32_t G, const int32_t* K,
                  const int64_t* n, const size_t* off, int32_t n_steps) = nullptr;
    // V of group g: q at off[g], V written at off[g] + n[g] 3 K[g]
    int (*energy)(void* user, const rhmc_params* P, int32_t G, const int32_t* K,
                  const int64_t* n, const size_t* off, int32_t f_pos) = nullptr;
  };
  Staged staged;

  int energies_staged(const std::vector<int64_t>& idx, std::vector<double>& V) {
    const auto gs = groups(idx);
    if (gs.empty()) return 0;
    const int32_t G = (int32_t)gs.size();
    std::vector<int32_t> Ks((size_t)G);
    std::vector<int64_t> ns((size_t)G);
    std::vector<size_t> off((size_t)G);
    size_t total = 0;
    for (int32_t g = 0; g < G; ++g) {
      Ks[g] = gs[g].first;
      ns[g] = (int64_t)gs[g].second.size();
      off[g] = total;
      total += (size_t)ns[g] * (3 * (size_t)Ks[g] + 1);
    }
    double* h = staged.buffer(staged.user, total);
    if (!h) return fail(RHMC_ERR_NOMEM, "staging buffer: " + g_err);
    std::vector<int64_t> slots, slot_c;
    std::vector<double*> slot_q, slot_v;
    for (int32_t g = 0; g < G; ++g) {
      const size_t d = 3 * (size_t)Ks[g];
      for (size_t i = 0; i < gs[g].second.size(); ++i) {
        slots.push_back((int64_t)slots.size());
        slot_c.push_back(gs[g].second[i]);
        slot_q.push_back(h + off[g] + i * d);
        slot_v.push_back(h + off[g] + (size_t)ns[g] * d + i);
      }
    }
    parallel(slots, [&](int64_t j) {
      const Chain& c = ch[slot_c[j]];
      std::memcpy(slot_q[j], c.q.data(), c.q.size() * 8);
    });
    const int rc = staged.energy(staged.user, &P, G, Ks.data(), ns.data(), off.data(), cfg->f_pos);
    if (rc != 0) return engine_fail(rc, "energy");
    for (size_t j = 0; j < slots.size(); ++j) V[slot_c[j]] = *slot_v[j];
    return 0;
  }

  int trajectories(const std::vector<int64_t>& idx) {
    if (staged.launch) return trajectories_staged(idx);
    std::vector<double> qb, pb;
    for (auto& grp : groups(idx)) {
      const int32_t K = grp.first;
      const auto& cs = grp.second;
      const size_t d = 3 * (size_t)K;
      qb.resize(cs.size() * d);
      pb.resize(cs.size() * d);
      for (size_t i = 0; i < cs.size(); ++i) {
        std::memcpy(&qb[i * d], ch[cs[i]].q.data(), d * 8);
        std::memcpy(&pb[i * d], ch[cs[i]].p.data(), d * 8);
      }
      const int rc = phys->steps(phys->user, &P, qb.data(), pb.data(), (int64_t)cs.size(), K,
                                 cfg->n_steps);
      if (rc != 0) return engine_fail(rc, "steps");
      for (size_t i = 0; i < cs.size(); ++i) {
        std::memcpy(ch[cs[i]].q.data(), &qb[i * d], d * 8);
        std::memcpy(ch[cs[i]].p.data(), &pb[i * d], d * 8);
      }
    }
    return 0;
  }

  int trajectories_staged(const std::vector<int64_t>& idx) {
    const auto gs = groups(idx);
    if (gs.empty()) return 0;
    const int32_t G = (int32_t)gs.size();
    std::vector<int32_t> Ks((size_t)G);
    std::vector<int64_t> ns((size_t)G);
    std::vector<size_t> off((size_t)G);
    size_t total = 0;
    for (int32_t g = 0; g < G; ++g) {
      Ks[g] = gs[g].first;
      ns[g] = (int64_t)gs[g].second.size();
      off[g] = total;
      total += 2 * (size_t)ns[g] * 3 * (size_t)Ks[g];
    }
    double* h = staged.buffer(staged.user, total);
    if (!h) return fail(RHMC_ERR_NOMEM, "staging buffer: " + g_err);
    // slot j of the phase: its chain, its q row and the offset of its p row
    // (group g's p block follows its q block) in the staging buffer
    std::vector<int64_t> slots, slot_c;
    std::vector<double*> slot_q;
    std::vector<size_t> pofs;
    for (int32_t g = 0; g < G; ++g) {
      const size_t d = 3 * (size_t)Ks[g];
      for (size_t i = 0; i < gs[g].second.size(); ++i) {
        slots.push_back((int64_t)slots.size());
        slot_c.push_back(gs[g].second[i]);
        slot_q.push_back(h + off[g] + i * d);
        pofs.push_back((size_t)ns[g] * d);
      }
    }
    parallel(slots, [&](int64_t j) {
      const Chain& c = ch[slot_c[j]];
      std::memcpy(slot_q[j], c.q.data(), c.q.size() * 8);
      std::memcpy(slot_q[j] + pofs[j], c.p.data(), c.p.size() * 8);
    });
    const int rc = staged.launch(staged.user, &P, G, Ks.data(), ns.data(), off.data(),
                                 cfg->n_steps);
    if (rc != 0) return engine_fail(rc, "steps");
    parallel(slots, [&](int64_t j) {
      Chain& c = ch[slot_c[j]];
      std::memcpy(c.q.data(), slot_q[j], c.q.size() * 8);
      std::memcpy(c.p.data(), slot_q[j] + pofs[j], c.p.size() * 8);
    });
    return 0;
  }

  int engine_fail(int rc, const char* what) {
    const char* m = rhmc_last_error();
    return fail(rc, std::string("engine ") + what + " failed: " + (m ? m : ""));
  }

  Metric metric() const {
    return Metric{P.g_ff2, P.g_ff, P.g_xx, P.g0, P.g1, P.g2, P.B_count, P.f_low};
  }

  // --------------------------------------------------------------- moves
  // birth_death_move (sampler_RHMC.py:1200-1270) on (q, -p); false = dead end
  bool birth_death(Chain& c, const Metric& M) {
    const double alpha = P.alpha;
    if (c.grow) {
      if (c.K + 1 > Kmax) return false;
      const double x = c.rng.random_sample() * (cfg->rows - 2.) + 1.;    // :1219
      const double y = c.rng.random_sample() * (cfg->cols - 2.) + 1.;    // :1220
      const double u = c.rng.random_sample();                             // :1221
      const double e = 1 - alpha;                                         // utils.py:469-471
      const double lm = std::pow(cfg->fmin, e) + u * (std::pow(cfg->fmax, e) - std::pow(cfg->fmin, e));
      const double f = std::exp(std::log(lm) / e);
      const double qn[3] = {f, x, y};
      double H3[3], pn[3];
      M.star(f, H3);
      for (int i = 0; i < 3; ++i) pn[i] = c.rng.gauss() * std::sqrt(H3[i]);   // :1231
      c.factor = alpha * std::log(f) - 3 / 2. + kinetic(pn, H3, 3, c.tmp) + P.V_prior_const;
      c.q.insert(c.q.end(), qn, qn + 3);
      c.p.insert(c.p.end(), pn, pn + 3);
      c.K += 1;
    } else {
      if (c.K - 1 < 1) return false;
      const int64_t k = c.rng.randint(0, c.K);                            // :1249
      double H3[3];
      M.star(c.q[3 * k], H3);
      const double Tk = kinetic(&c.p[3 * k], H3, 3, c.tmp);
      c.factor = -alpha * std::log(c.q[3 * k]) + 3 / 2. - Tk - P.V_prior_const;
      c.q.erase(c.q.begin() + 3 * k, c.q.begin() + 3 * k + 3);
      c.p.erase(c.p.begin() + 3 * k, c.p.begin() + 3 * k + 3);
      c.K -= 1;
    }
    return true;
  }

  // split_merge_move (sampler_RHMC.py:1273-1445) on (q, -p); false = dead end
  bool split_merge(Chain& c, const Metric& M) {
    const double a = cfg->beta_a, b = cfg->beta_b, Ks = cfg->K_split;
    const double two_pi_ks2 = 2 * kPi * std::pow(Ks, 2);
    const double ln_q_dxdy = std::log(two_pi_ks2);
    const double two_ks2 = 2 * std::pow(Ks, 2);
    if (c.grow) {
      if (c.K + 1 > Kmax) return false;
      const int64_t i = c.rng.randint(0, c.K);                            // :1291
      const double fs = c.q[3 * i], xs = c.q[3 * i + 1], ys = c.q[3 * i + 2];
      const double qs[3] = {fs, xs, ys}, ps[3] = {c.p[3 * i], c.p[3 * i + 1], c.p[3 * i + 2]};
      const double g1 = c.rng.gauss(), g2 = c.rng.gauss();                // :1300
      const double dx = g1 * Ks, dy = g2 * Ks;
      const double dr_sq = std::pow(dx, 2) + std::pow(dy, 2);
      const double F = c.rng.beta(a, b);                                  // :1302
      const double q1[3] = {F * fs, xs + (1 - F) * dx, ys + (1 - F) * dy};
      const double q2[3] = {(1 - F) * fs, xs - F * dx, ys - F * dy};
      double H1[3], H2[3], Hs[3], p1[3], p2[3];
      M.star(q1[0], H1);
      for (int t = 0; t < 3; ++t) p1[t] = c.rng.gauss() * std::sqrt(H1[t]);   // :1328
      M.star(q2[0], H2);
      for (int t = 0; t < 3; ++t) p2[t] = c.rng.gauss() * std::sqrt(H2[t]);   // :1333
      M.star(qs[0], Hs);
      const double Ts = kinetic(ps, Hs, 3, c.tmp);
      const double T1 = kinetic(p1, H1, 3, c.tmp), T2 = kinetic(p2, H2, 3, c.tmp);
      c.factor = (-3 / 2.) + std::log(fs) - beta.logpdf(F) + ln_q_dxdy + (dr_sq / two_ks2) +
                 T1 + T2 - Ts;
      for (int t = 0; t < 3; ++t) {
        c.q[3 * i + t] = q1[t];
        c.p[3 * i + t] = p1[t];
      }
      c.q.insert(c.q.end(), q2, q2 + 3);
      c.p.insert(c.p.end(), p2, p2 + 3);
      c.K += 1;
      return true;
    }
    const int64_t n = c.K;
    if (n - 1 < 1) return false;
    // pair probabilities ~ Beta(F_ij) N(r_ij), self pairs excluded (:1366-1378)
    std::vector<double> P2((size_t)(n * n));
    for (int64_t r = 0; r < n; ++r)
      for (int64_t s = 0; s < n; ++s) {
        const double fr = c.q[3 * r], fc = c.q[3 * s];
        const double Fm = fc / (fr + fc);
        double v = beta.pdf(Fm);
        if (std::fabs(Fm - 0.5) < 1e-6) v = 0.;
        const double ddx = c.q[3 * r + 1] - c.q[3 * s + 1], ddy = c.q[3 * r + 2] - c.q[3 * s + 2];
        const double Rsq = std::pow(ddx, 2) + std::pow(ddy, 2);
        P2[r * n + s] = v * (std::exp(-Rsq / two_ks2) / two_pi_ks2);
      }
    const double tot = rhmc_np::pairwise_sum(P2.data(), n * n);
    if (!(tot > 0.0) || !std::isfinite(tot)) return false;  // the reference raises here
    for (auto& v : P2) v /= tot;
    const int64_t pair = choice(c.rng, P2.data(), n * n, c.cdf);          // :1381
    if (pair >= n * n) return false;
    const int64_t i1 = pair / n, i2 = pair % n;
    const double q1[3] = {c.q[3 * i1], c.q[3 * i1 + 1], c.q[3 * i1 + 2]};
    const double p1[3] = {c.p[3 * i1], c.p[3 * i1 + 1], c.p[3 * i1 + 2]};
    const double q2[3] = {c.q[3 * i2], c.q[3 * i2 + 1], c.q[3 * i2 + 2]};
    const double p2[3] = {c.p[3 * i2], c.p[3 * i2 + 1], c.p[3 * i2 + 2]};
    const double F = q1[0] / (q1[0] + q2[0]);
    const double dx = q1[1] - q2[1], dy = q1[2] - q2[2];
    const double dr_sq = std::pow(dx, 2) + std::pow(dy, 2);
    const double qs[3] = {q1[0] + q2[0], F * q1[1] + (1 - F) * q2[1], F * q1[2] + (1 - F) * q2[2]};
    double H1[3], H2[3], Hs[3], ps[3];
    M.star(q1[0], H1);
    const double T1 = kinetic(p1, H1, 3, c.tmp);
    M.star(q2[0], H2);
    const double T2 = kinetic(p2, H2, 3, c.tmp);
    M.star(qs[0], Hs);
    for (int t = 0; t < 3; ++t) ps[t] = c.rng.gauss() * std::sqrt(Hs[t]);      // :1415
    const double Ts = kinetic(ps, Hs, 3, c.tmp);
    const int64_t lo = std::min(i1, i2), hi = std::max(i1, i2);
    std::vector<double> nq, np_;
    nq.reserve((size_t)(3 * (n - 1)));
    np_.reserve((size_t)(3 * (n - 1)));
    for (int64_t s = 0; s < n; ++s) {
      if (s == lo || s == hi) continue;
      nq.insert(nq.end(), &c.q[3 * s], &c.q[3 * s] + 3);
      np_.insert(np_.end(), &c.p[3 * s], &c.p[3 * s] + 3);
    }
    nq.insert(nq.end(), qs, qs + 3);
    np_.insert(np_.end(), ps, ps + 3);
    c.factor = (3 / 2.) - std::log(qs[0]) + beta.logpdf(F) - ln_q_dxdy - (dr_sq / two_ks2) -
               T1 - T2 + Ts;
    c.q.swap(nq);
    c.p.swap(np_);
    c.K -= 1;
    return true;
  }
};

int check(const rhmc_params* P, const rhmc_rj_config* cfg, const double* q, const int32_t* K,
          const uint32_t* seeds, int64_t n) {
  if (!P || !cfg) return fail(RHMC_ERR_ARG, "params or config is NULL");
  if (cfg->reserved != 0) return fail(RHMC_ERR_ARG, "config.reserved must be 0");
  if (cfg->n_pipes < 0 || cfg->n_pipes > kMaxPipes)
    return fail(RHMC_ERR_ARG, "n_pipes must be in [0, 4]");
  if (n < 0) return fail(RHMC_ERR_ARG, "n < 0");
  if (n > 0 && (!q || !K)) return fail(RHMC_ERR_ARG, "q or K is NULL");
  if (cfg->use_states != 0 && cfg->use_states != 1)
    return fail(RHMC_ERR_ARG, "use_states must be 0 or 1");
  if (n > 0 && cfg->use_states && !cfg->states)
    return fail(RHMC_ERR_ARG, "use_states without states");
  if (n > 0 && !cfg->use_states && !seeds) return fail(RHMC_ERR_ARG, "seeds is NULL");
  for (int64_t c = 0; cfg->use_states && c < n; ++c)
    if (cfg->states[c].pos < 0 || cfg->states[c].pos > 624)
      return fail(RHMC_ERR_ARG, "states[c].pos must be in [0, 624]");
  if (cfg->n_iter < 0 || cfg->n_steps < 0) return fail(RHMC_ERR_ARG, "n_iter or n_steps < 0");
  if (cfg->N_max < 1 || cfg->N_max > 256) return fail(RHMC_ERR_ARG, "N_max must be in [1, 256]");
  if (cfg->rows < 3 || cfg->cols < 3) return fail(RHMC_ERR_ARG, "rows / cols < 3");
  if ((cfg->n_g_ff2 > 0 && !cfg->schedule_g_ff2) || (cfg->n_beta > 0 && !cfg->schedule_beta) ||
      cfg->n_g_ff2 < 0 || cfg->n_beta < 0)
    return fail(RHMC_ERR_ARG, "schedule array missing");
  double ps = 0.;
  for (int i = 0; i < 3; ++i) {
    if (!(cfg->P_move[i] >= 0.0)) return fail(RHMC_ERR_ARG, "P_move entries must be >= 0");
    ps += cfg->P_move[i];
  }
  if (!(std::fabs(ps - 1.0) <= 1.4901161193847656e-08))  // choice(): sqrt(eps) tolerance
    return fail(RHMC_ERR_ARG, "P_move must sum to 1");
  if ((cfg->P_move[1] > 0 || cfg->P_move[2] > 0) &&
      !(cfg->fmin > 0 && cfg->fmax > 0 && cfg->K_split > 0 && cfg->beta_a > 0 && cfg->beta_b > 0))
    return fail(RHMC_ERR_ARG, "jumps need fmin, fmax, K_split, beta_a, beta_b > 0");
  for (int64_t c = 0; c < n; ++c)
    if (K[c] < 1 || K[c] > cfg->N_max) return fail(RHMC_ERR_ARG, "K[c] must be in [1, N_max]");
  return 0;
}

int host_threads(const rhmc_rj_config* cfg) {
  const int nt = cfg->n_threads;
  if (nt > 0) return nt;
  return (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
}

// n chains (a contiguous slice of the caller's: q, K, seeds point at its
// first chain); record row l of chain c is l * rec_stride + rec_off + c; nt
// host threads; the phase times are added to phase_out[7].
int run(const rhmc_rj_physics* phys, const Run::Staged* staged, const rhmc_params* P0,
        const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds, int64_t n,
        const rhmc_rj_record* rec, int64_t rec_stride, int64_t rec_off, int nt,
        double* phase_out) {
  if (!phys || !phys->energy || !phys->steps) return fail(RHMC_ERR_ARG, "physics is NULL");
  Run R;
  R.phys = phys;
  if (staged) R.staged = *staged;
  R.P = *P0;
  R.cfg = cfg;
  R.Kmax = cfg->N_max;
  R.beta.set(cfg->beta_a, cfg->beta_b);
  R.nt = nt;
  Pool pool(nt);
  R.pool = &pool;
  R.ch.resize((size_t)n);
  const int64_t W = 3 * (int64_t)cfg->N_max;
  std::vector<int64_t> all((size_t)n);
  for (int64_t c = 0; c < n; ++c) {
    all[c] = c;
    Chain& h = R.ch[c];
    if (cfg->use_states) {
      const rhmc_np_state& st = cfg->states[rec_off + c];
      h.rng.set_state(st.key, st.pos, st.has_gauss, st.gauss);
    } else {
      h.rng.seed(seeds[c]);
    }
    h.K = K[c];
    h.q.assign(q + c * W, q + c * W + 3 * (int64_t)K[c]);
  }
  const int64_t rows_n = (int64_t)cfg->n_iter + 1;
  std::vector<double> V0((size_t)n), V1((size_t)n), T0((size_t)n);
  // V of every chain's q at the end of the previous iteration (V(q') if it
  // accepted, else its V(q)) and the prior parameters it was computed with:
  // while a schedule leaves them unchanged, an iteration's V(q) is that value
  // (the engine's V of a chain does not depend on the batch it is in:
  // tests/test_gpu_rj_native.py recomputes every recorded V), saving one
  // engine phase per iteration
  std::vector<double> V_end((size_t)n);
  double V_end_g_ff2 = 0., V_end_beta = 0.;
  bool V_end_ok = false;
  double phase[7] = {0, 0, 0, 0, 0, 0, 0};
  auto clk = std::chrono::steady_clock::now();
  auto lap = [&](int i) {  // the time since the last lap goes to phase i
    const auto t = std::chrono::steady_clock::now();
    phase[i] += std::chrono::duration<double>(t - clk).count();
    clk = t;
  };
  for (int64_t l = 0; l < rows_n; ++l) {
    if (cfg->n_g_ff2 > 0) R.P.g_ff2 = cfg->schedule_g_ff2[std::min<int64_t>(l, cfg->n_g_ff2 - 1)];
    if (cfg->n_beta > 0) R.P.beta = cfg->schedule_beta[std::min<int64_t>(l, cfg->n_beta - 1)];
    const Metric M = R.metric();
    // 1. momentum, T0, move type, grow / shrink
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      const int64_t d = 3 * (int64_t)h.K;
      h.H.resize((size_t)d);
      M.all(h.q.data(), d, h.H.data());
      h.p.resize((size_t)d);
      for (int64_t i = 0; i < d; i += 3) {  // p = randn(3K) * sqrt(H); H_y = H_x
        const double sf = std::sqrt(h.H[i]), sx = std::sqrt(h.H[i + 1]);
        h.p[i] = h.rng.gauss() * sf;
        h.p[i + 1] = h.rng.gauss() * sx;
        h.p[i + 2] = h.rng.gauss() * (h.H[i + 2] == h.H[i + 1] ? sx : std::sqrt(h.H[i + 2]));
      }
      h.move = (int)choice(h.rng, cfg->P_move, 3, h.cdf);
      h.grow = false;
      if (h.move != 0) {
        const double half[2] = {0.5, 0.5};
        h.grow = choice(h.rng, half, 2, h.cdf) == 0;   // [True, False]
      }
      T0[c] = kinetic(h.p.data(), h.H.data(), d, h.tmp);
      h.q0 = h.q;
      h.K0 = h.K;
      h.dead = false;
    });
    lap(0);
    // 2. V(q)
    if (V_end_ok && R.P.g_ff2 == V_end_g_ff2 && R.P.beta == V_end_beta) {
      V0 = V_end;
    } else if (int rc = R.energies(all, V0)) {
      return rc;
    }
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      h.E0 = V0[c] + T0[c];
      const int64_t r = l * rec_stride + rec_off + c;
      if (rec) {
        if (rec->q_chain) {  // the state, zero-padded to 3 N_max
          double* row = rec->q_chain + r * W;
          std::fill(std::copy(h.q.begin(), h.q.end(), row), row + W, 0.);
        }
        if (rec->p_chain) {
          double* row = rec->p_chain + r * W;
          std::fill(std::copy(h.p.begin(), h.p.end(), row), row + W, 0.);
        }
        if (rec->V_chain) rec->V_chain[r] = V0[c];
        if (rec->T_chain) rec->T_chain[r] = T0[c];
        if (rec->E_chain) rec->E_chain[r] = h.E0;
        if (rec->n_stars) rec->n_stars[r] = h.K;
        if (rec->move)
          rec->move[r] = h.move == 0 ? 0 : h.move == 1 ? (h.grow ? 1 : 2) : (h.grow ? 3 : 4);
      }
    });
    lap(1);
    // 3. the trajectory of every chain
    if (int rc = R.trajectories(all)) return rc;
    lap(2);
    // 4. the proposals
    std::vector<int64_t> jump;
    for (int64_t c = 0; c < n; ++c)
      if (R.ch[c].move != 0) jump.push_back(c);
    R.parallel(jump, [&](int64_t c) {
      Chain& h = R.ch[c];
      for (auto& v : h.p) v = -v;
      const bool ok = h.move == 1 ? R.birth_death(h, M) : R.split_merge(h, M);
      if (!ok) {
        h.dead = true;
        h.q = h.q0;
        h.K = h.K0;
      }
    });
    std::vector<int64_t> live;
    for (int64_t c : jump)
      if (!R.ch[c].dead) live.push_back(c);
    lap(3);
    // 5. the trajectory after the jump
    if (int rc = R.trajectories(live)) return rc;
    lap(4);
    for (int64_t c : live)
      for (auto& v : R.ch[c].p) v = -v;
    // 6. V(q')
    std::vector<int64_t> scored;
    for (int64_t c = 0; c < n; ++c)
      if (!R.ch[c].dead) scored.push_back(c);
    if (int rc = R.energies(scored, V1)) return rc;
    lap(5);
    // 7. accept / reject
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      const int64_t r = l * rec_stride + rec_off + c;
      bool acc = false;
      if (!h.dead) {
        const int64_t d = 3 * (int64_t)h.K;
        h.H.resize((size_t)d);
        M.all(h.q.data(), d, h.H.data());
        const double E1 = V1[c] + kinetic(h.p.data(), h.H.data(), d, h.tmp);
        const double u = std::log(h.rng.random_sample());
        if (h.move == 0) {
          const double dE = E1 - h.E0;
          acc = (dE < 0) || (u < -dE);
        } else {
          const double ln_alpha0 = -(E1 - h.E0) + h.factor;
          acc = (ln_alpha0 > 0) || (u < ln_alpha0);
        }
        if (!acc) {
          h.q = h.q0;
          h.K = h.K0;
        }
      }
      V_end[c] = acc ? V1[c] : V0[c];
      if (rec) {
        if (rec->accept) rec->accept[r] = acc ? 1 : 0;
        if (rec->flags) rec->flags[r] = h.dead ? (int32_t)RHMC_RJ_DEAD_END : 0;
      }
    });
    lap(6);
    V_end_g_ff2 = R.P.g_ff2;
    V_end_beta = R.P.beta;
    V_end_ok = true;
  }
  if (phase_out)
    for (int i = 0; i < 7; ++i) phase_out[i] += phase[i];
  for (int64_t c = 0; c < n; ++c) {
    const Chain& h = R.ch[c];
    std::fill(q + c * W, q + (c + 1) * W, 0.);
    std::copy(h.q.begin(), h.q.end(), q + c * W);
    K[c] = h.K;
    if (cfg->states) {
      rhmc_np_state& st = cfg->states[rec_off + c];
      h.rng.get_state(st.key, &st.pos, &st.has_gauss, &st.gauss);
    }
  }
  return 0;
}

// the engine as physics: V by rhmc_energy; the trajectories of all star-count
// groups of a phase at once, each group on one of kStreams HIP streams
// (rhmc_leapfrog_device), so that small groups fill the GPU together instead
// of one after the other
constexpr int kStreams = 4;
static_assert(kStreams >= kMaxPipes, "a stream per pipe at least");

// The streams live for the process, kStreams per device, created on first use
// and warmed by one small copy each: the first dispatch to a new HIP stream
// binds its hardware queue, which cost 6-11 ms per stream when it happened
// inside a run (profiles/r04_rj/).
struct DeviceStreams {
  hipStream_t s[kStreams] = {};
  double* warm = nullptr;
};

std::mutex g_streams_mu;
std::map<int, DeviceStreams> g_streams;

struct CtxEngine {
  rhmc_ctx* ctx = nullptr;
  hipStream_t s[kStreams] = {};
  int ns = kStreams;             // streams in use: s[0 .. ns)
  int dev = 0;
  double* d = nullptr;
  size_t d_bytes = 0;
  double* h = nullptr;
  size_t h_bytes = 0;
  ~CtxEngine() {  // nothing may still be copying into the buffers (error paths)
    for (int i = 0; i < ns; ++i)
      if (s[i]) (void)hipStreamSynchronize(s[i]);
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
  }
};

#define RJ_HIP(expr)                                                                   \
  do {                                                                                 \
    const hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) return fail(RHMC_ERR_HIP, std::string(#expr) + ": " +        \
                                                        hipGetErrorString(e_));        \
  } while (0)

int engine_init(CtxEngine& E) {
  const double* dimg = nullptr;
  if (int rc = rhmc_ctx_image_device(E.ctx, &dimg)) return rc;
  if (!dimg) return fail(RHMC_ERR_ARG, "context has no image");
  hipPointerAttribute_t at;
  RJ_HIP(hipPointerGetAttributes(&at, dimg));
  RJ_HIP(hipSetDevice(at.device));
  E.dev = at.device;
  std::lock_guard<std::mutex> lock(g_streams_mu);
  DeviceStreams& ds = g_streams[at.device];
  if (!ds.warm) {
    RJ_HIP(hipMalloc(&ds.warm, kStreams * sizeof(double)));
    for (int i = 0; i < kStreams; ++i) {
      RJ_HIP(hipStreamCreateWithFlags(&ds.s[i], hipStreamNonBlocking));
      RJ_HIP(hipMemsetAsync(ds.warm + i, 0, sizeof(double), ds.s[i]));
    }
    for (int i = 0; i < kStreams; ++i) RJ_HIP(hipStreamSynchronize(ds.s[i]));
  }
  for (int i = 0; i < kStreams; ++i) E.s[i] = ds.s[i];
  return 0;
}

// One 1-chain, 0-step trajectory of the run's first star count on each stream
// the first time the process meets that (device, kernel): the first dispatch
// of a kernel on a hardware queue set up its scratch and cost 6-8 ms inside a
// run (profiles/r04_rj/trace).
std::map<std::pair<int, int>, bool> g_warm;  // (device, K) under g_streams_mu

int engine_warm(CtxEngine& E, const rhmc_params* P, int32_t K) {
  int dev = 0;
  RJ_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(g_streams_mu);
  bool& done = g_warm[{dev, K}];
  if (done) return 0;
  double* d = nullptr;
  std::vector<double> h(6 * (size_t)K, 0.0);  // q: stars of 1000 counts at (1 + k/2, 2), p = 0
  for (int32_t k = 0; k < K; ++k) {
    h[3 * k] = 1000.0;
    h[3 * k + 1] = 1.0 + 0.5 * k;
    h[3 * k + 2] = 2.0;
  }
  RJ_HIP(hipMalloc(&d, h.size() * sizeof(double)));
  RJ_HIP(hipMemcpy(d, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
  int rc = 0;
  for (int i = 0; i < kStreams && rc == 0; ++i)
    rc = rhmc_leapfrog_device(E.ctx, P, d, d + 3 * K, 1, K, 0, nullptr, nullptr, E.s[i]);
  for (int i = 0; i < kStreams; ++i) (void)hipStreamSynchronize(E.s[i]);
  (void)hipFree(d);
  if (rc) return rc;
  done = true;
  return 0;
}

int ctx_energy(void* user, const rhmc_params* P, const double* q, int64_t n, int32_t K,
               int32_t f_pos, double* V) {
  return rhmc_energy(static_cast<CtxEngine*>(user)->ctx, P, q, nullptr, V, nullptr, n, K, f_pos);
}
int ctx_steps(void* user, const rhmc_params* P, double* q, double* p, int64_t n, int32_t K,
              int32_t n_steps) {
  return rhmc_leapfrog(static_cast<CtxEngine*>(user)->ctx, P, q, p, n, K, n_steps, nullptr,
                       nullptr);
}
double* ctx_buffer(void* user, size_t doubles) {
  CtxEngine& E = *static_cast<CtxEngine*>(user);
  const size_t bytes = doubles * 8;
  if (bytes > E.d_bytes) {
    if (E.d) (void)hipFree(E.d);
    E.d = nullptr;
    E.d_bytes = 0;
    if (hipMalloc(&E.d, bytes) != hipSuccess) {
      g_err = "hipMalloc failed";
      return nullptr;
    }
    E.d_bytes = bytes;
  }
  if (bytes > E.h_bytes) {
    if (E.h) (void)hipHostFree(E.h);
    E.h = nullptr;
    E.h_bytes = 0;
    if (hipHostMalloc(&E.h, bytes, hipHostMallocDefault) != hipSuccess) {
      g_err = "hipHostMalloc failed";
      return nullptr;
    }
    E.h_bytes = bytes;
  }
  return E.h;
}

int ctx_launch(void* user, const rhmc_params* P, int32_t G, const int32_t* K, const int64_t* n,
               const size_t* off, int32_t n_steps) {
  CtxEngine& E = *static_cast<CtxEngine*>(user);
  std::vector<int32_t> order((size_t)G);
  for (int32_t g = 0; g < G; ++g) order[g] = g;
  std::stable_sort(order.begin(), order.end(),
                   [&](int32_t a, int32_t b) { return n[a] * K[a] > n[b] * K[b]; });
  int rc = 0;
  for (int32_t i = 0; i < G && rc == 0; ++i) {  // largest groups first
    const int32_t g = order[i];
    const size_t sb = (size_t)n[g] * 3 * (size_t)K[g];
    hipStream_t st = E.s[i % E.ns];
    double* hq = E.h + off[g];
    double* dq = E.d + off[g];
    hipError_t e = hipMemcpyAsync(dq, hq, 2 * sb * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      rc = rhmc_leapfrog_device(E.ctx, P, dq, dq + sb, n[g], K[g], n_steps, nullptr, nullptr, st);
      if (rc == 0) e = hipMemcpyAsync(hq, dq, 2 * sb * 8, hipMemcpyDeviceToHost, st);
    }
    if (e != hipSuccess) rc = fail(RHMC_ERR_HIP, std::string("staging copy: ") + hipGetErrorString(e));
  }
  for (int i = 0; i < E.ns; ++i) RJ_HIP(hipStreamSynchronize(E.s[i]));
  return rc;
}

int ctx_energy_staged(void* user, const rhmc_params* P, int32_t G, const int32_t* K,
                      const int64_t* n, const size_t* off, int32_t f_pos) {
  CtxEngine& E = *static_cast<CtxEngine*>(user);
  int rc = 0;
  for (int32_t g = 0; g < G && rc == 0; ++g) {
    const size_t sb = (size_t)n[g] * 3 * (size_t)K[g];
    hipStream_t st = E.s[g % E.ns];
    double* hq = E.h + off[g];
    double* dq = E.d + off[g];
    hipError_t e = hipMemcpyAsync(dq, hq, sb * 8, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
      rc = rhmc_energy_device(E.ctx, P, dq, nullptr, dq + sb, nullptr, n[g], K[g], f_pos, st);
      if (rc == 0) e = hipMemcpyAsync(hq + sb, dq + sb, (size_t)n[g] * 8, hipMemcpyDeviceToHost, st);
    }
    if (e != hipSuccess) rc = fail(RHMC_ERR_HIP, std::string("staging copy: ") + hipGetErrorString(e));
  }
  for (int i = 0; i < E.ns; ++i) RJ_HIP(hipStreamSynchronize(E.s[i]));
  return rc;
}

// Split n chains into `pipes` contiguous parts run concurrently, part i on
// its own host thread (part 0 on the caller's) with its share of the nt pool
// threads: body(i, first chain, count, threads, phase[7]) -> rc.  The first
// failing part's error is the one reported.
template <class Body>
int run_pipes(int pipes, int64_t n, int nt, double* phase, Body body) {
  // one part's body on this thread; an exception becomes an error code (no
  // C++ exception may cross the ABI, and none may leave a std::thread)
  auto guarded = [&](int i, int64_t f, int64_t m, int t, double* ph, std::string& err) {
    try {
      const int rc = body(i, f, m, t, ph);
      if (rc) err = g_err;
      return rc;
    } catch (const std::exception& e) {
      err = std::string("host exception: ") + e.what();
    } catch (...) {
      err = "host exception";
    }
    return (int)RHMC_ERR_NOMEM;
  };
  if (pipes <= 1) {
    std::string err;
    const int rc = guarded(0, 0, n, nt, phase, err);
    if (rc) g_err = err;
    return rc;
  }
  std::vector<int64_t> first((size_t)pipes + 1);
  for (int i = 0; i <= pipes; ++i) first[i] = n * i / pipes;
  std::vector<int> threads((size_t)pipes);
  for (int i = 0; i < pipes; ++i) threads[i] = std::max(1, nt * (i + 1) / pipes - nt * i / pipes);
  std::vector<std::array<double, 7>> ph((size_t)pipes);
  std::vector<int> rcs((size_t)pipes, 0);
  std::vector<std::string> errs((size_t)pipes);
  std::vector<std::thread> ts;
  ts.reserve((size_t)pipes);
  for (int i = 1; i < pipes; ++i) {
    ph[i].fill(0.);
    try {
      ts.emplace_back([&, i] {
        rcs[i] = guarded(i, first[i], first[i + 1] - first[i], threads[i], ph[i].data(), errs[i]);
      });
    } catch (const std::exception& e) {  // this part does not run: report it
      rcs[i] = RHMC_ERR_NOMEM;
      errs[i] = std::string("cannot start a pipe thread: ") + e.what();
    }
  }
  ph[0].fill(0.);
  rcs[0] = guarded(0, first[0], first[1] - first[0], threads[0], ph[0].data(), errs[0]);
  for (auto& t : ts) t.join();
  for (int i = 0; i < pipes; ++i)
    for (int k = 0; k < 7; ++k) phase[k] += ph[i][k];
  for (int i = 0; i < pipes; ++i)
    if (rcs[i]) {
      g_err = errs[i];
      return rcs[i];
    }
  return 0;
}

int pipes_for(const rhmc_rj_config* cfg, int64_t n) {
  // default: measured at big-sim4 geometry (profiles/r04_pipes2/): 2 pipes
  // from 1,024 chains (1.11x one at 4,096; 3 and 4 lose there), 3 from 16,384
  // (1.54x one, 1.16x two or four)
  int pipes = cfg->n_pipes > 0 ? cfg->n_pipes : (n >= 16384 ? 3 : n >= 1024 ? 2 : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>(pipes, n));
}

}  // namespace

extern "C" {

int rhmc_rj_run_physics(const rhmc_rj_physics* phys, const rhmc_params* P,
                        const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds,
                        int64_t n, const rhmc_rj_record* rec) {
  try {
    if (int rc = check(P, cfg, q, K, seeds, n)) return rc;
    double phase[7] = {0, 0, 0, 0, 0, 0, 0};
    const int nt = host_threads(cfg);
    // with pipes > 1 the callbacks are called from that many threads at once
    const int64_t W = 3 * (int64_t)cfg->N_max;
    int rc = run_pipes(cfg->n_pipes > 1 ? pipes_for(cfg, n) : 1, n, nt, phase,
                       [&](int, int64_t f, int64_t m, int t, double* ph) {
                         return run(phys, nullptr, P, cfg, q + f * W, K + f,
                                    seeds ? seeds + f : nullptr, m, rec, n, f, t, ph);
                       });
    if (rc == 0 && rec && rec->phase_s) std::copy(phase, phase + 7, rec->phase_s);
    return rc;
  } catch (const std::exception& e) {
    return fail(RHMC_ERR_NOMEM, std::string("host exception: ") + e.what());
  }
}

int rhmc_rj_run(rhmc_ctx* ctx, const rhmc_params* P, const rhmc_rj_config* cfg, double* q,
                int32_t* K, const uint32_t* seeds, int64_t n, const rhmc_rj_record* rec) {
  if (!ctx) return fail(RHMC_ERR_ARG, "ctx is NULL");
  try {
    if (int rc = check(P, cfg, q, K, seeds, n)) return rc;
    CtxEngine E[kMaxPipes];
    for (auto& e : E) e.ctx = ctx;
    if (int rc = engine_init(E[0])) return rc;
    if (n > 0)
      if (int rc = engine_warm(E[0], P, K[0])) return rc;
    const int pipes = pipes_for(cfg, n);
    const int nt = host_threads(cfg);
    // pipe i takes streams i, i + pipes, ... (the HIP calls of the *_device
    // entry points touch no shared context state)
    hipStream_t all_s[kStreams];
    std::copy(E[0].s, E[0].s + kStreams, all_s);
    for (int i = 0; i < pipes; ++i) {
      E[i].dev = E[0].dev;
      E[i].ns = 0;
      for (int j = i; j < kStreams; j += pipes) E[i].s[E[i].ns++] = all_s[j];
    }
    const int64_t W = 3 * (int64_t)cfg->N_max;
    double phase[7] = {0, 0, 0, 0, 0, 0, 0};
    const int rc = run_pipes(pipes, n, nt, phase, [&](int i, int64_t f, int64_t m, int t,
                                                      double* ph) {
      if (i > 0 && hipSetDevice(E[i].dev) != hipSuccess) return fail(RHMC_ERR_HIP, "hipSetDevice failed");
      rhmc_rj_physics phys{&E[i], ctx_energy, ctx_steps};
      Run::Staged st;
      st.user = &E[i];
      st.buffer = ctx_buffer;
      st.launch = ctx_launch;
      st.energy = ctx_energy_staged;
      return run(&phys, &st, P, cfg, q + f * W, K + f, seeds ? seeds + f : nullptr, m, rec, n, f,
                 t, ph);
    });
    if (rc == 0 && rec && rec->phase_s) std::copy(phase, phase + 7, rec->phase_s);
    return rc;
  } catch (const std::exception& e) {
    return fail(RHMC_ERR_NOMEM, std::string("host exception: ") + e.what());
  }
}

int rhmc_np_draws(uint32_t seed, int32_t kind, double a, double b, int64_t n, double* out) {
  if (n < 0 || (n > 0 && !out)) return fail(RHMC_ERR_ARG, "bad n or out");
  rhmc_np::Legacy r(seed);
  for (int64_t i = 0; i < n; ++i) {
    switch (kind) {
      case 0: out[i] = r.random_sample(); break;
      case 1: out[i] = r.gauss(); break;
      case 2:
        if (!(a >= 1.0)) return fail(RHMC_ERR_ARG, "randint needs a >= 1");
        out[i] = (double)r.randint(0, (int64_t)a);
        break;
      case 3: out[i] = r.beta(a, b); break;
      case 4: out[i] = r.standard_gamma(a); break;
      case 5: out[i] = r.standard_exponential(); break;
      default: return fail(RHMC_ERR_ARG, "unknown kind");
    }
  }
  return 0;
}

int rhmc_rj_beta_eval(double a, double b, const double* x, int64_t n, double* pdf, double* logpdf) {
  if (!(a > 0) || !(b > 0)) return fail(RHMC_ERR_ARG, "beta_a and beta_b must be > 0");
  if (n < 0 || (n > 0 && !x)) return fail(RHMC_ERR_ARG, "bad n or x");
  BetaDist d;
  d.set(a, b);
  for (int64_t i = 0; i < n; ++i) {
    if (pdf) pdf[i] = d.pdf(x[i]);
    if (logpdf) logpdf[i] = d.logpdf(x[i]);
  }
  return 0;
}

const char* rhmc_rj_last_error(void) { return g_err.c_str(); }

}  // extern "C"
