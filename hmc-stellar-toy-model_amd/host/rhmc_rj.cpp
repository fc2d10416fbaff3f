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
#include <cstdio>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <emmintrin.h>
#include <hip/hip_runtime_api.h>

#include "np_legacy.hpp"

namespace {

constexpr int kMaxPipes = 8;  // rhmc_rj_config::n_pipes

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

constexpr double kPi = 3.141592653589793;  // np.pi

// ------------------------------------------------------------ record rows
// One [3 N_max] row of a record or of the final states: src[0, d) then zeros
// to `zero_to` (W, or less where the caller's row is known to be zero past it:
// rhmc_rj_config::records_zero_padded).  A full row goes out with
// non-temporal stores: the q_chain / p_chain records are 2 x 3 N_max doubles
// per chain and iteration (24 MB per iteration at 4,096 chains and N_max 120,
// most of it the zero padding), written once and not read back by the run;
// plain stores first pull every destination line into the cache, which
// halved the host's record bandwidth (tools/rec_write_bench.cpp).  The
// caller issues _mm_sfence() before the rows are handed on.
void put_row(double* dst, const double* src, int64_t d, int64_t zero_to, int64_t W) {
  if (zero_to < W) {
    std::fill(std::copy(src, src + d, dst), dst + zero_to, 0.);
    return;
  }
  int64_t i = 0;
  if (reinterpret_cast<uintptr_t>(dst) & 15) {  // to a 16-byte boundary
    dst[0] = d > 0 ? src[0] : 0.;
    i = 1;
  }
  for (; i + 2 <= d; i += 2) _mm_stream_pd(dst + i, _mm_loadu_pd(src + i));
  if (i < d) {  // one live value left
    if (i + 2 <= W) {
      _mm_stream_pd(dst + i, _mm_set_pd(0., src[i]));
      i += 2;
    } else {
      dst[i] = src[i];
      ++i;
    }
  }
  const __m128d z = _mm_setzero_pd();
  for (; i + 2 <= W; i += 2) _mm_stream_pd(dst + i, z);
  if (i < W) dst[i] = 0.;
}

// The zero fill's end for record row r: with records_zero_padded the row
// holds zeros past 3 n_stars[r] (the previous run's count), so the fill stops
// at the larger of that and the new width d; else the whole row
int64_t zero_end(const rhmc_rj_config* cfg, const rhmc_rj_record* rec, int64_t r, int64_t d,
                 int64_t W) {
  if (!(cfg->records_zero_padded & RHMC_RJ_ZP_RECORDS)) return W;
  const int32_t old = rec->n_stars[r];
  if (old < 1 || old > cfg->N_max) return W;
  return std::max(d, 3 * (int64_t)old);
}

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
// Fork-join pool shared by every pipe of a run (and kept between runs: spawning
// threads per phase cost ~3 ms per iteration at 16 threads, per run ~1 ms).
// Several callers may run jobs at once: a worker takes chunks of whichever job
// has some left, so while one pipe waits for its GPU phase its share of the
// host threads works on the other pipes' host phases (round 5's per-pipe
// pools left them idle), and a pipe thread waiting for its stream takes chunks
// too (help()).  Each chain's work is its own, so results do not depend on
// which thread runs it.
class Pool {
 public:
  explicit Pool(int workers) {
    try {
      for (int t = 0; t < workers; ++t) th_.emplace_back([this] { worker(); });
    } catch (...) {  // a thread could not start: stop and join the ones that did
      shutdown();
      throw;
    }
  }
  ~Pool() { shutdown(); }
  int size() const { return (int)th_.size() + 1; }
  // body(i) for i in [0, n), in chunks, the caller works too.  An exception
  // from body (any thread) is rethrown here once no thread is left in it.
  void run(int64_t n, const std::function<void(int64_t)>& body) {
    Job j;
    j.body = &body;
    j.n = n;
    {
      std::lock_guard<std::mutex> l(mu_);
      jobs_.push_back(&j);
      pending_.fetch_add(1);
    }
    cv_.notify_all();
    while (take(j)) {
    }
    {
      std::lock_guard<std::mutex> l(mu_);
      jobs_.erase(std::find(jobs_.begin(), jobs_.end(), &j));
      pending_.fetch_sub(1);
    }
    // every chunk is taken; wait for the ones still running elsewhere (no
    // worker picks the job up once it is off the list)
    while (j.done.load() != n || j.users.load() != 0) std::this_thread::yield();
    if (j.exc) std::rethrow_exception(j.exc);
  }
  // one chunk of any caller's job, if one is left: false if none
  bool help() {
    Job* j = nullptr;
    {
      std::lock_guard<std::mutex> l(mu_);
      j = pick();
      if (j) j->users.fetch_add(1);
    }
    if (!j) return false;
    const bool did = take(*j);
    j->users.fetch_sub(1);
    return did;
  }

 private:
  static constexpr int64_t kChunk = 16;
  struct Job {
    const std::function<void(int64_t)>* body = nullptr;
    int64_t n = 0;
    std::atomic<int64_t> next{0}, done{0};
    std::atomic<int> users{0};
    std::atomic<bool> failed{false};
    std::mutex emu;
    std::exception_ptr exc;
  };
  Job* pick() {  // mu_ held
    for (Job* j : jobs_)
      if (j->next.load() < j->n) return j;
    return nullptr;
  }
  // one chunk of j; false when none was left.  After a failure the remaining
  // chunks are counted without running (the first exception is kept)
  bool take(Job& j) {
    const int64_t b = j.next.fetch_add(kChunk);
    if (b >= j.n) return false;
    const int64_t e = std::min(j.n, b + kChunk);
    if (!j.failed.load()) {
      try {
        for (int64_t i = b; i < e; ++i) (*j.body)(i);
      } catch (...) {
        std::lock_guard<std::mutex> l(j.emu);
        if (!j.exc) j.exc = std::current_exception();
        j.failed.store(true);
      }
    }
    j.done.fetch_add(e - b);
    return true;
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
      stop_flag_.store(true);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
    th_.clear();
  }
  void worker() {
    for (;;) {
      Job* j = nullptr;
      // spin a little before sleeping: the pipes' phases follow each other
      // within tens of microseconds, and a futex wake-up costs about that
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; pending_.load(std::memory_order_relaxed) == 0 && !stop_flag_.load(); ++k) {
        _mm_pause();
        if ((k & 255) == 255 &&
            std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(kSpinUs))
          break;
      }
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || (j = pick()) != nullptr; });
        if (stop_) return;
        j->users.fetch_add(1);
      }
      while (take(*j)) {
      }
      j->users.fetch_sub(1);
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Job*> jobs_;
  bool stop_ = false;
  std::atomic<bool> stop_flag_{false};
  std::atomic<int> pending_{0};  // jobs on the list (the spin's hint)
  static constexpr int kSpinUs = 50;
};

// The process's pools by worker count, kept for its lifetime (a run takes the
// one of its size; runs on other threads may share it)
std::shared_ptr<Pool> shared_pool(int workers) {
  static std::mutex mu;
  static std::map<int, std::shared_ptr<Pool>> pools;
  std::lock_guard<std::mutex> l(mu);
  auto& p = pools[workers];
  if (!p) p = std::make_shared<Pool>(workers);
  return p;
}

// ------------------------------------------------------------------- chains
struct Chain {
  rhmc_np::Legacy rng;
  std::vector<double> q, p, q0;  // state, momentum, the iteration's starting q
  int32_t K = 0, K0 = 0;
  int move = 0;                  // 0 within, 1 birth/death, 2 split/merge
  bool grow = false, dead = false;
  double E0 = 0., factor = 0.;
  std::vector<double> H, tmp, cdf;
  // the device driver's draws made ahead, while the GPU runs: the accept
  // uniform, and the next iteration's normals / move / grow of a chain whose
  // star count cannot change (move 0 or a dead end) — the stream's order is
  // unchanged, only the time of the draws moves
  double u = 0.;
  bool pre = false, grow_next = false;
  int move_next = 0;
  std::vector<double> znext;
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

  int trajectories(const std::vector<int64_t>& idx) {
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
    // pair probabilities ~ Beta(F_ij) N(r_ij), self pairs excluded (:1366-1378).
    // R_sq is symmetric bit for bit ((a - b)^2 == (b - a)^2), so each pair's
    // Gaussian factor is evaluated once for both orders
    std::vector<double> P2((size_t)(n * n));
    for (int64_t r = 0; r < n; ++r)
      for (int64_t s = r; s < n; ++s) {
        const double ddx = c.q[3 * r + 1] - c.q[3 * s + 1], ddy = c.q[3 * r + 2] - c.q[3 * s + 2];
        const double Rsq = std::pow(ddx, 2) + std::pow(ddy, 2);
        const double g = std::exp(-Rsq / two_ks2) / two_pi_ks2;
        const double fr = c.q[3 * r], fc = c.q[3 * s];
        const double F1 = fc / (fr + fc);
        double v1 = beta.pdf(F1);
        if (std::fabs(F1 - 0.5) < 1e-6) v1 = 0.;
        P2[r * n + s] = v1 * g;
        if (s == r) continue;
        const double F2 = fr / (fc + fr);
        double v2 = beta.pdf(F2);
        if (std::fabs(F2 - 0.5) < 1e-6) v2 = 0.;
        P2[s * n + r] = v2 * g;
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
  if (cfg->records_zero_padded < 0 || cfg->records_zero_padded > 3)
    return fail(RHMC_ERR_ARG, "records_zero_padded must be in [0, 3]");
  if (cfg->n_pipes < 0 || cfg->n_pipes > kMaxPipes)
    return fail(RHMC_ERR_ARG, "n_pipes must be in [0, 8]");
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
  if (cfg->N_max < 1 || cfg->N_max > 1024)
    return fail(RHMC_ERR_ARG, "N_max must be in [1, 1024]");
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

int check_records(const rhmc_rj_config* cfg, const rhmc_rj_record* rec) {
  if ((cfg->records_zero_padded & RHMC_RJ_ZP_RECORDS) && !(rec && rec->n_stars))
    return fail(RHMC_ERR_ARG, "records_zero_padded needs the n_stars record");
  return 0;
}

int host_threads(const rhmc_rj_config* cfg) {
  const int nt = cfg->n_threads;
  if (nt > 0) return nt;
  return (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
}

// n chains (a contiguous slice of the caller's: q, K, seeds point at its
// first chain); record row l of chain c is l * rec_stride + rec_off + c; the
// host work on `pool`; the phase times are added to phase_out[7].
int run(const rhmc_rj_physics* phys, const rhmc_params* P0,
        const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds, int64_t n,
        const rhmc_rj_record* rec, int64_t rec_stride, int64_t rec_off, Pool* pool,
        double* phase_out) {
  if (!phys || !phys->energy || !phys->steps) return fail(RHMC_ERR_ARG, "physics is NULL");
  Run R;
  R.phys = phys;
  R.P = *P0;
  R.cfg = cfg;
  R.Kmax = cfg->N_max;
  R.beta.set(cfg->beta_a, cfg->beta_b);
  R.nt = pool->size();
  R.pool = pool;
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
        // the state, zero-padded to 3 N_max (read n_stars[r] before it is rewritten)
        const int64_t d = 3 * (int64_t)h.K, zt = zero_end(cfg, rec, r, d, W);
        if (rec->q_chain) put_row(rec->q_chain + r * W, h.q.data(), d, zt, W);
        if (rec->p_chain) put_row(rec->p_chain + r * W, h.p.data(), d, zt, W);
        _mm_sfence();
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
    put_row(q + c * W, h.q.data(), 3 * (int64_t)h.K, W, W);
    _mm_sfence();
    K[c] = h.K;
    if (cfg->states) {
      rhmc_np_state& st = cfg->states[rec_off + c];
      h.rng.get_state(st.key, &st.pos, &st.has_gauss, &st.gauss);
    }
  }
  return 0;
}

// ===================================================================== device
// rhmc_rj_run: the chains live in HBM for the whole run (librhmc.so's
// ragged-set entry points, rhmc.h ABI 4).  Per pipe: padded [n][W] rows
// (W = 3 N_max, zeros past a chain's 3 K) of
//   Q0   the chains' states (the iteration's starting point; the q_chain rows)
//   Q, P the working trajectory state
// and per iteration only these cross PCIe:
//   H2D  the host-drawn normals z (3 K per chain: the NumPy-stream draws stay
//        on the host, bit for bit), the star counts, index lists, and the
//        jumping chains' proposed rows
//   D2H  T0, V / T at the end (one double each per chain), the jumping chains'
//        rows before their proposal, and — when the caller records them — the
//        q_chain / p_chain rows (on a second stream, overlapping the trajectory)
// The momentum p = z sqrt(H(q)) and both kinetic energies run on the device
// (rhmc_kinetic_rows_device, the reference's operation order); every phase is
// one ragged launch for the star counts the slotted kernels serve (dense /
// windowed, rhmc_ragged_ok) plus one packed launch per remaining star count
// (the one-star, pixel-major and multi-star register-window kernels), the
// packed ones spread over the pipe's two streams.
constexpr int kStreamsPerPipe = 2;  // main (in order) + aux (records, packed groups)

#define RJ_HIP(expr)                                                                   \
  do {                                                                                 \
    const hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) return fail(RHMC_ERR_HIP, std::string(#expr) + ": " +        \
                                                        hipGetErrorString(e_));        \
  } while (0)

#define RJ_TRY(expr)                        \
  do {                                      \
    if (int rc_ = (expr)) return rc_;       \
  } while (0)

// Index lists of an iteration, one region each (the launches read them from
// mapped host memory when they execute, so no region is rewritten before a
// wait on its readers).
enum { kIdxV0, kIdxSteps1, kIdxJump, kIdxSteps2, kIdxV1, kIdxCommit, kIdxRegions };

// One pipe's buffers: device rows and pinned staging, grown as needed and kept
// until rhmc_rj_release (a run of 4,096 chains at N_max 120 holds ~90 MB of HBM
// and ~60 MB of pinned memory per pipe).  `mu` is held for a whole run, so two
// concurrent rhmc_rj_run calls on one device serialise pipe by pipe.
struct Work {
  std::mutex mu;
  int dev = -1;
  // the pipe's per-chain host state, kept between runs with its vectors'
  // capacity (freeing and reallocating it per run cost ~2 ms at 1,024 chains)
  std::vector<Chain> chains;
  hipStream_t s[kStreamsPerPipe] = {};
  hipEvent_t ev[4] = {};

  int64_t cap_n = 0, cap_W = 0;
  // Device rows: Q, P (the trajectories' state), Q0 (each iteration's start),
  // pack (the fixed-K launches' gathered batches).
  double *Q = nullptr, *P = nullptr, *Q0 = nullptr, *pack = nullptr;
  // Everything that crosses PCIe lives in coherent pinned host memory mapped
  // into the device's address space, and the kernels read or write it there
  // (their *_d addresses): the iteration's draws `up` = [zoff (N int64) | K
  // (N int32, in N int64 slots) | Z (M doubles)], the index lists, T0 | V(q),
  // V(q') | T', the record rows' live columns and the jumping rows.  No copy
  // engine and no copy call: SDMA copies stalled a pipe 7-8 ms at its first
  // large copy of a direction (profiles/r06_rj/, RHMC_RJ_TIMING build), and
  // each one added a queue hand-off to the iteration's critical path.
  void *up_h = nullptr, *vt_h = nullptr;
  double *Zh = nullptr, *Jh = nullptr, *recq = nullptr, *recp = nullptr;
  double *T0h = nullptr, *T1h = nullptr, *Vh = nullptr;
  int32_t* Kh = nullptr;
  int64_t *zoffh = nullptr, *idxh = nullptr;
  // their device addresses
  double *Zd = nullptr, *Jd = nullptr, *recqd = nullptr, *recpd = nullptr;
  double *T0d = nullptr, *T1d = nullptr, *Vd = nullptr;
  int32_t* Kd = nullptr;
  int64_t *zoffd = nullptr, *idxd = nullptr;

  void release() {
    for (double* d : {Q, P, Q0, pack}) (void)hipFree(d);
    for (double* h : {Jh, recq, recp, T0h}) (void)hipHostFree(h);
    for (void* h : {up_h, vt_h}) (void)hipHostFree(h);
    (void)hipHostFree(idxh);
    Q = P = Q0 = pack = nullptr;
    up_h = vt_h = nullptr;
    Zh = Jh = recq = recp = T0h = T1h = Vh = nullptr;
    Zd = Jd = recqd = recpd = T0d = T1d = Vd = nullptr;
    Kh = Kd = nullptr;
    zoffh = idxh = zoffd = idxd = nullptr;
    cap_n = cap_W = 0;
  }

  // everything, streams and events included (rhmc_rj_release; `mu` held)
  void destroy() {
    std::vector<Chain>().swap(chains);
    if (dev < 0) return;
    (void)hipSetDevice(dev);
    for (auto& st : s)
      if (st) (void)hipStreamSynchronize(st);
    release();
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);

    for (auto& st : s)
      if (st) (void)hipStreamDestroy(st);
    for (auto& e : ev) e = nullptr;
    for (auto& st : s) st = nullptr;
    dev = -1;
  }

  // streams and events on `device` once; buffers for n chains of W doubles
  int ensure(int device, int64_t n, int64_t W) {
    if (dev < 0) {
      dev = device;
      for (auto& st : s) RJ_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
      for (auto& e : ev) RJ_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));

    }
    if (n <= cap_n && W <= cap_W) return 0;
    for (auto& st : s) RJ_HIP(hipStreamSynchronize(st));
    release();
    const int64_t N = std::max<int64_t>(n, 1), M = N * W;
    auto dmal = [](auto** p, size_t count) {
      return hipMalloc((void**)p, count * sizeof(**p)) == hipSuccess;
    };
    // coherent, mapped: the kernels read / write it at its device address
    auto hmap = [](auto** p, auto** d, size_t count) {
      return hipHostMalloc((void**)p, count * sizeof(**p),
                           hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
             hipHostGetDevicePointer((void**)d, *p, 0) == hipSuccess;
    };
    double *uph = nullptr, *upd = nullptr, *vth = nullptr, *vtd = nullptr;
    const bool ok = dmal(&Q, M) && dmal(&P, M) && dmal(&Q0, M) && dmal(&pack, 4 * M) &&
                    hmap(&uph, &upd, 2 * N + M) && hmap(&Jh, &Jd, 2 * M) &&
                    hmap(&recq, &recqd, M) && hmap(&recp, &recpd, M) &&
                    hmap(&T0h, &T0d, 2 * N) && hmap(&vth, &vtd, 2 * N) &&
                    hmap(&idxh, &idxd, kIdxRegions * N);
    up_h = uph;
    vt_h = vth;
    if (ok) {
      zoffh = (int64_t*)uph;
      Kh = (int32_t*)(uph + N);
      Zh = uph + 2 * N;
      zoffd = (int64_t*)upd;
      Kd = (int32_t*)(upd + N);
      Zd = upd + 2 * N;
      Vh = vth;
      T1h = vth + N;
      Vd = vtd;
      T1d = vtd + N;
    }
    if (!ok) {
      release();
      return fail(RHMC_ERR_NOMEM, "reversible-jump device buffers: allocation failed");
    }
    cap_n = N;
    cap_W = W;
    return 0;
  }
};

std::mutex g_work_mu;
std::map<std::pair<int, int>, Work*> g_work;  // (device, pipe), process lifetime

Work* work_for(int dev, int pipe) {
  std::lock_guard<std::mutex> lock(g_work_mu);
  Work*& w = g_work[{dev, pipe}];
  if (!w) w = new Work();
  return w;
}

// The caller's current device, restored when a run returns.
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// One phase's launch plan over chains `idx` (star counts K): the chains of the
// slotted kernels' star counts grouped by register slots (one ragged launch
// each), then one packed launch per other star count (first appearance).
struct Call {
  bool ragged;
  int32_t Kmin, Kmax;
  int64_t off, n;  // the call's chains: order[off .. off + n)
};
struct Plan {
  std::vector<int64_t> order;
  std::vector<Call> calls;
};

Plan make_plan(const std::vector<int64_t>& idx, const std::vector<int32_t>& K,
               const std::vector<char>& ragged_ok) {
  Plan pl;
  // the engine's ragged launch classes: one kernel family and one register-slot
  // count each (2-10 stars: the pixel-major kernel on 32/48-px images; then the
  // slot counts of the dense / windowed kernels)
  std::vector<int64_t> cls[6];
  std::vector<std::pair<int32_t, std::vector<int64_t>>> groups;
  std::map<int32_t, size_t> where;
  for (int64_t c : idx) {
    const int32_t k = K[c];
    if (ragged_ok[k]) {
      cls[k <= 10 ? 0 : k <= 64 ? 1 : k <= 128 ? 2 : k <= 256 ? 3 : k <= 512 ? 4 : 5].push_back(c);
      continue;
    }
    auto it = where.find(k);
    if (it == where.end()) {
      where[k] = groups.size();
      groups.push_back({k, {c}});
    } else {
      groups[it->second].second.push_back(c);
    }
  }
  for (auto& v : cls) {
    if (v.empty()) continue;
    int32_t lo = 1024, hi = 1;
    for (int64_t c : v) {
      lo = std::min(lo, K[c]);
      hi = std::max(hi, K[c]);
    }
    pl.calls.push_back({true, lo, hi, (int64_t)pl.order.size(), (int64_t)v.size()});
    pl.order.insert(pl.order.end(), v.begin(), v.end());
  }
  for (auto& g : groups) {
    pl.calls.push_back({false, g.first, g.first, (int64_t)pl.order.size(),
                        (int64_t)g.second.size()});
    pl.order.insert(pl.order.end(), g.second.begin(), g.second.end());
  }
  return pl;
}

struct DevRun {
  rhmc_ctx* ctx;
  Work* w;
  int64_t n, W;
  std::vector<int32_t>& K;  // host star counts (what the kernels read: set_K)
  const std::vector<char>& ragged_ok;

  int engine_fail(int rc, const char* what) {
    const char* m = rhmc_last_error();
    return fail(rc, std::string("engine ") + what + " failed: " + (m ? m : ""));
  }
  // the star counts as the kernels read them (mapped host memory; no kernel
  // reading them is in flight when the host rewrites them)
  void set_K() { std::copy(K.begin(), K.end(), w->Kh); }
  int64_t* idx_h(int region) { return w->idxh + region * w->cap_n; }
  int64_t* idx_d(int region) { return w->idxd + region * w->cap_n; }
  // the plan's chain order as the launches' index list.  Each region is
  // rewritten only after a wait on the launches that read it (or, for the
  // commit list, behind them in stream order)
  void set_order(const Plan& pl, int region) {
    std::copy(pl.order.begin(), pl.order.end(), idx_h(region));
  }
  // the host waits until stream i is done.  (A blocking-sync event instead of
  // the runtime's spinning wait measured 0.87-0.93x at B4: the wake-up latency
  // costs more than the CPU the spin takes from the pool threads.)
  // While the stream runs, the waiting pipe thread takes host chunks of the
  // other pipes' phases.
  Pool* pool;
  int wait(int i) {
    for (;;) {
      const hipError_t e = hipStreamQuery(w->s[i]);
      if (e == hipSuccess) return 0;
      if (e != hipErrorNotReady)
        return fail(RHMC_ERR_HIP, std::string("reversible-jump stream: ") + hipGetErrorString(e));
      if (!pool->help()) std::this_thread::yield();
    }
  }
  // the host waits for event e (recorded on a stream), taking pool chunks
  int wait_event(int e) {
    for (;;) {
      const hipError_t r = hipEventQuery(w->ev[e]);
      if (r == hipSuccess) return 0;
      if (r != hipErrorNotReady)
        return fail(RHMC_ERR_HIP, std::string("reversible-jump event: ") + hipGetErrorString(r));
      if (!pool->help()) std::this_thread::yield();
    }
  }
  // aux waits for main, or main for aux
  int join(int from, int to, int e) {
    RJ_HIP(hipEventRecord(w->ev[e], w->s[from]));
    RJ_HIP(hipStreamWaitEvent(w->s[to], w->ev[e], 0));
    return 0;
  }

  // n_steps steps on chains idx (rows of Q, P)
  int trajectories(const rhmc_params* P, const std::vector<int64_t>& idx, int32_t n_steps,
                   int region) {
    if (idx.empty()) return 0;
    const Plan pl = make_plan(idx, K, ragged_ok);
    set_order(pl, region);
    bool aux_used = false;
    int packed = 0;
    for (const Call& c : pl.calls) {
      const int64_t* rows = idx_d(region) + c.off;
      if (c.ragged) {
#ifdef RHMC_RJ_TIMING  // diagnostic build: a launch call that blocks
        const auto tl0 = std::chrono::steady_clock::now();
#endif
        if (int rc = rhmc_leapfrog_ragged_device(ctx, P, w->Q, w->P, W, rows, w->Kd, c.n, c.Kmin,
                                                 c.Kmax, n_steps, w->s[0]))
          return engine_fail(rc, "ragged steps");
#ifdef RHMC_RJ_TIMING
        const double tl = std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0)
                              .count() * 1e3;
        if (tl > 0.2)
          std::fprintf(stderr, "rj slow launch: steps K %d-%d n %lld %.3f ms\n", c.Kmin, c.Kmax,
                       (long long)c.n, tl);
#endif
        continue;
      }
      // packed: gather, fixed-K steps, scatter — alternate groups onto aux
      const int si = (packed++ % 2);
      if (si == 1 && !aux_used) {
        RJ_TRY(join(0, 1, 0));
        aux_used = true;
      }
      hipStream_t st = w->s[si];
      const int64_t d = 3 * (int64_t)c.Kmin;
      double* pq = w->pack + (si ? 2 * n * W : 0);
      double* pp = pq + c.n * d;
      if (int rc = rhmc_rows_copy_device(ctx, w->Q, W, rows, pq, d, nullptr, c.n, (int32_t)d, st))
        return engine_fail(rc, "gather");
      if (int rc = rhmc_rows_copy_device(ctx, w->P, W, rows, pp, d, nullptr, c.n, (int32_t)d, st))
        return engine_fail(rc, "gather");
      if (int rc = rhmc_leapfrog_device(ctx, P, pq, pp, c.n, c.Kmin, n_steps, nullptr, nullptr, st))
        return engine_fail(rc, "steps");
      if (int rc = rhmc_rows_copy_device(ctx, pq, d, nullptr, w->Q, W, rows, c.n, (int32_t)d, st))
        return engine_fail(rc, "scatter");
      if (int rc = rhmc_rows_copy_device(ctx, pp, d, nullptr, w->P, W, rows, c.n, (int32_t)d, st))
        return engine_fail(rc, "scatter");
    }
    if (aux_used) RJ_TRY(join(1, 0, 1));
    return 0;
  }

  // V of chains idx (rows of Q) -> V_out[j] for chain order[j] (a device
  // address: the mapped host buffer the host reads after a wait)
  int energies(const rhmc_params* P, const std::vector<int64_t>& idx, int32_t f_pos,
               std::vector<int64_t>& order, int region, double* V_out) {
    order.clear();
    if (idx.empty()) return 0;
    const Plan pl = make_plan(idx, K, ragged_ok);
    order = pl.order;
    set_order(pl, region);
    for (const Call& c : pl.calls) {
      const int64_t* rows = idx_d(region) + c.off;
      if (c.ragged) {
#ifdef RHMC_RJ_TIMING
        const auto tl0 = std::chrono::steady_clock::now();
#endif
        if (int rc = rhmc_energy_ragged_device(ctx, P, w->Q, W, rows, w->Kd, c.n, c.Kmin, c.Kmax,
                                               f_pos, V_out + c.off, w->s[0]))
          return engine_fail(rc, "ragged energy");
#ifdef RHMC_RJ_TIMING
        const double tl = std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0)
                              .count() * 1e3;
        if (tl > 0.2)
          std::fprintf(stderr, "rj slow launch: energy K %d-%d n %lld %.3f ms\n", c.Kmin, c.Kmax,
                       (long long)c.n, tl);
#endif
        continue;
      }
      const int64_t d = 3 * (int64_t)c.Kmin;
      if (int rc = rhmc_rows_copy_device(ctx, w->Q, W, rows, w->pack, d, nullptr, c.n, (int32_t)d,
                                         w->s[0]))
        return engine_fail(rc, "gather");
      if (int rc = rhmc_energy_device(ctx, P, w->pack, nullptr, V_out + c.off, nullptr, c.n, c.Kmin,
                                      f_pos, w->s[0]))
        return engine_fail(rc, "energy");
    }
    return 0;
  }
};

// The device-resident run of chains [0, n) of one pipe (q, K, seeds point at
// its first chain; record row l of chain c is l * rec_stride + rec_off + c).
int run_device(rhmc_ctx* ctx, int dev, Work* w, const rhmc_params* P0,
               const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds, int64_t n,
               const rhmc_rj_record* rec, int64_t rec_stride, int64_t rec_off, Pool* pool,
               double* phase_out) {
#ifdef RHMC_RJ_TIMING
  const auto t_setup0 = std::chrono::steady_clock::now();
#endif
  const int64_t W = 3 * (int64_t)cfg->N_max;
  RJ_TRY(w->ensure(dev, n, W));
  hipStream_t s0 = w->s[0];
  Run R;
  R.phys = nullptr;
  R.P = *P0;
  R.cfg = cfg;
  R.Kmax = cfg->N_max;
  R.beta.set(cfg->beta_a, cfg->beta_b);
  R.nt = pool->size();
  R.pool = pool;
  struct GiveBack {  // the chains' storage returns to the pipe on every exit
    std::vector<Chain>& from;
    std::vector<Chain>& to;
    ~GiveBack() { from.swap(to); }
  } give_back{R.ch, w->chains};
  R.ch.swap(w->chains);
  R.ch.resize((size_t)n);
  std::vector<int32_t> Kc((size_t)n);
  const std::vector<int32_t> K_in(K, K + n);  // the rows' widths on entry (ZP_STARTS)
  std::vector<int64_t> all((size_t)n);
  int32_t kin = 1;
  for (int64_t c = 0; c < n; ++c) {
    all[c] = c;
    kin = std::max(kin, K[c]);
  }
  // each chain's stream (MT19937 seeding: ~2 us a chain) and the caller's
  // rows' live columns (3 K_max, zeros past 3 K) -> Q0, on the pool; the
  // rest of Q0 is zeroed on the device
  const int64_t w0 = 3 * (int64_t)kin;
  R.parallel(all, [&](int64_t c) {
    Chain& h = R.ch[c];
    if (cfg->use_states) {
      const rhmc_np_state& st = cfg->states[rec_off + c];
      h.rng.set_state(st.key, st.pos, st.has_gauss, st.gauss);
    } else {
      h.rng.seed(seeds[c]);
    }
    h.K = K[c];
    Kc[c] = K[c];
    double* row = w->Zh + c * w0;
    std::copy(q + c * W, q + c * W + 3 * (int64_t)K[c], row);
    std::fill(row + 3 * (int64_t)K[c], row + w0, 0.);
  });
  RJ_HIP(hipMemsetAsync(w->Q0, 0, (size_t)(n * W) * 8, s0));
  if (int rc = rhmc_rows_copy_device(ctx, w->Zd, w0, nullptr, w->Q0, W, nullptr, n, (int32_t)w0, s0))
    return fail(rc, std::string("engine start rows failed: ") +
                        (rhmc_last_error() ? rhmc_last_error() : ""));
  RJ_HIP(hipStreamSynchronize(s0));  // Zh is the draws' staging next
  std::vector<char> ragged_ok((size_t)cfg->N_max + 1, 0);
  {
    int32_t ok = 0;
    for (int k = 1; k <= cfg->N_max; ++k) {
      if (int rc = rhmc_ragged_ok(ctx, P0, k, &ok)) return rc;
      ragged_ok[k] = (char)ok;
    }
  }
  DevRun D{ctx, w, n, W, Kc, ragged_ok, pool};
  const int64_t rows_n = (int64_t)cfg->n_iter + 1;
  std::vector<double> V0((size_t)n), V1((size_t)n), V_end((size_t)n);
  double V_end_g_ff2 = 0., V_end_beta = 0.;
  bool V_end_ok = false;
  const bool rec_q = rec && rec->q_chain, rec_p = rec && rec->p_chain;
  double phase[7] = {0, 0, 0, 0, 0, 0, 0};
  auto clk = std::chrono::steady_clock::now();
  int64_t l_now = 0;
  auto lap = [&](int i) {
    const auto t = std::chrono::steady_clock::now();
    const double dt = std::chrono::duration<double>(t - clk).count();
    phase[i] += dt;
    clk = t;
#ifdef RHMC_RJ_TIMING
    if (dt > 1e-3)
      std::fprintf(stderr, "rj slow phase %d: %.3f ms (l %lld)\n", i, dt * 1e3, (long long)l_now);
#else
    (void)l_now;
#endif
  };
  std::vector<int64_t> order, order0, jump, live, scored, acc_rows;
#ifdef RHMC_RJ_TIMING
  const auto t_loop0 = std::chrono::steady_clock::now();
#endif
  // an iteration's first draws (:1021-1022, :1031-1033): z = randn(3K), the
  // move type, grow / shrink
  auto draw_start = [&](Chain& h, double* z) {
    for (int64_t i = 0; i < 3 * (int64_t)h.K; ++i) z[i] = h.rng.gauss();
    h.move = (int)choice(h.rng, cfg->P_move, 3, h.cdf);
    h.grow = false;
    if (h.move != 0) {
      const double half[2] = {0.5, 0.5};
      h.grow = choice(h.rng, half, 2, h.cdf) == 0;  // [True, False]
    }
  };
  for (auto& h : R.ch) h.pre = false;
  for (int64_t l = 0; l < rows_n; ++l) {
    l_now = l;
    if (cfg->n_g_ff2 > 0) R.P.g_ff2 = cfg->schedule_g_ff2[std::min<int64_t>(l, cfg->n_g_ff2 - 1)];
    if (cfg->n_beta > 0) R.P.beta = cfg->schedule_beta[std::min<int64_t>(l, cfg->n_beta - 1)];
    const Metric M = R.metric();
    // 1. host draws: z = randn(3K) (the momentum, :1021-1022), move type, grow / shrink
    int64_t zt = 0;
    for (int64_t c = 0; c < n; ++c) {
      w->zoffh[c] = zt;
      zt += 3 * (int64_t)Kc[c];
    }
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      double* z = w->Zh + w->zoffh[c];
      if (h.pre) {  // drawn during the previous iteration's V(q') wait
        std::copy(h.znext.begin(), h.znext.end(), z);
        h.move = h.move_next;
        h.grow = h.grow_next;
        h.pre = false;
      } else {
        draw_start(h, z);
      }
      h.K0 = h.K;
      h.dead = false;
    });
    lap(0);
    // 2. device: Q = Q0, p = z sqrt(H(q)), T0; record rows; V(q) unless reused.
    // Rows are zero past 3 K in Q0; Q may hold a rejected birth's or split's
    // extra star past it (3 entries), so Q = Q0 covers 3 K_max + 3 columns and
    // every other copy only the columns a row can use (not the 3 N_max width)
    const int32_t kmax = *std::max_element(Kc.begin(), Kc.end());
    const int64_t wq = std::min<int64_t>(W, 3 * (int64_t)kmax + 3);
    const int64_t wr = 3 * (int64_t)kmax;  // the record rows' live columns
    D.set_K();  // [zoff | K | Z] are read by the kernels where the host wrote them
    RJ_HIP(hipMemcpy2DAsync(w->Q, (size_t)W * 8, w->Q0, (size_t)W * 8, (size_t)wq * 8, (size_t)n,
                            hipMemcpyDeviceToDevice, s0));
    if (int rc = rhmc_kinetic_rows_device(ctx, &R.P, w->Q, w->P, W, w->Kd, w->Zd, w->zoffd, n,
                                          w->T0d, s0))
      return D.engine_fail(rc, "momentum");
    // the record rows' live columns, before the trajectory moves P
    if (rec_q)
      if (int rc = rhmc_rows_copy_device(ctx, w->Q0, W, nullptr, w->recqd, W, nullptr, n,
                                         (int32_t)wr, s0))
        return D.engine_fail(rc, "record rows");
    if (rec_p)
      if (int rc = rhmc_rows_copy_device(ctx, w->P, W, nullptr, w->recpd, W, nullptr, n,
                                         (int32_t)wr, s0))
        return D.engine_fail(rc, "record rows");
    const bool reuse = V_end_ok && R.P.g_ff2 == V_end_g_ff2 && R.P.beta == V_end_beta;
    // V(q) when not reused, [T0 | V(q)] read at the accept step
    double* V0h = w->T0h + w->cap_n;
    if (!reuse) RJ_TRY(D.energies(&R.P, all, cfg->f_pos, order0, kIdxV0, w->T0d + w->cap_n));
    // the jumping chains (their rows go to the host after the trajectory)
    jump.clear();
    for (int64_t c = 0; c < n; ++c)
      if (R.ch[c].move != 0) jump.push_back(c);
    std::copy(jump.begin(), jump.end(), D.idx_h(kIdxJump));
    // 3. the trajectory of every chain (queued behind the above).  The host
    // needs T0, V(q) and the record rows only at the accept step: no wait here
    RJ_HIP(hipEventRecord(w->ev[2], s0));  // T0, V(q) and the record rows are in
                                           // (events 0 and 1: join())
    RJ_TRY(D.trajectories(&R.P, all, cfg->n_steps, kIdxSteps1));
    lap(1);
    // while the trajectories run: the iteration's record rows (row l: its
    // starting state; none of it depends on the accept step)
    RJ_TRY(D.wait_event(2));
    if (!reuse)
      for (size_t j = 0; j < order0.size(); ++j) V0[order0[j]] = V0h[j];
    else
      V0 = V_end;
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      const int64_t r = l * rec_stride + rec_off + c;
      h.E0 = V0[c] + w->T0h[c];
      if (!rec) return;
      // the rows are zero past 3 K0 on the device: copy the 3 K0, write the
      // zeros (read n_stars[r] before it is rewritten)
      const int64_t d = 3 * (int64_t)h.K0, zt = zero_end(cfg, rec, r, d, W);
      if (rec_q) put_row(rec->q_chain + r * W, w->recq + c * W, d, zt, W);
      if (rec_p) put_row(rec->p_chain + r * W, w->recp + c * W, d, zt, W);
      _mm_sfence();
      if (rec->V_chain) rec->V_chain[r] = V0[c];
      if (rec->T_chain) rec->T_chain[r] = w->T0h[c];
      if (rec->E_chain) rec->E_chain[r] = h.E0;
      if (rec->n_stars) rec->n_stars[r] = h.K0;
      if (rec->move)
        rec->move[r] = h.move == 0 ? 0 : h.move == 1 ? (h.grow ? 1 : 2) : (h.grow ? 3 : 4);
    });
    lap(6);
    // 4. the jumping chains' rows to the host, their proposals on (q, -p), back
    const int64_t nj = (int64_t)jump.size();
    // a jumping row's columns: its 3 K stars and the one a birth / split adds
    int32_t kj = 1;
    for (int64_t c : jump) kj = std::max(kj, Kc[c]);
    const int64_t dj = std::min<int64_t>(W, 3 * (int64_t)kj + 3);
    double* Jq = w->Jd;             // [nj][dj] q rows, then [nj][dj] p rows (host, mapped)
    double* Jp = w->Jd + nj * dj;
    int64_t* jd = D.idx_d(kIdxJump);
    if (nj > 0) {
      if (int rc = rhmc_rows_copy_device(ctx, w->Q, W, jd, Jq, dj, nullptr, nj, (int32_t)dj, s0))
        return D.engine_fail(rc, "gather");
      if (int rc = rhmc_rows_copy_device(ctx, w->P, W, jd, Jp, dj, nullptr, nj, (int32_t)dj, s0))
        return D.engine_fail(rc, "gather");
    }
    RJ_TRY(D.wait(0));
    lap(2);
    std::vector<int64_t> jpos(jump.size());
    for (int64_t j = 0; j < nj; ++j) jpos[j] = j;
    R.parallel(jpos, [&](int64_t j) {
      Chain& h = R.ch[jump[j]];
      double* rq = w->Jh + j * dj;
      double* rp = w->Jh + nj * dj + j * dj;
      const int64_t d = 3 * (int64_t)h.K;
      h.q.assign(rq, rq + d);
      h.p.resize((size_t)d);
      for (int64_t i = 0; i < d; ++i) h.p[i] = -rp[i];
      const bool ok = h.move == 1 ? R.birth_death(h, M) : R.split_merge(h, M);
      if (!ok) {
        h.dead = true;
        h.K = h.K0;
        return;  // its rows are restored from Q0 at the accept step
      }
      std::fill(std::copy(h.q.begin(), h.q.end(), rq), rq + dj, 0.);
      std::fill(std::copy(h.p.begin(), h.p.end(), rp), rp + dj, 0.);
    });
    live.clear();
    for (int64_t c : jump)
      if (!R.ch[c].dead) live.push_back(c);
    for (int64_t c : live) Kc[c] = R.ch[c].K;
    lap(3);
    if (nj > 0) {  // every jumping row back (a dead end's rows are restored later)
      if (int rc = rhmc_rows_copy_device(ctx, Jq, dj, nullptr, w->Q, W, jd, nj, (int32_t)dj, s0))
        return D.engine_fail(rc, "scatter");
      if (int rc = rhmc_rows_copy_device(ctx, Jp, dj, nullptr, w->P, W, jd, nj, (int32_t)dj, s0))
        return D.engine_fail(rc, "scatter");
      D.set_K();
    }
    // 5. the trajectory after the jump
    RJ_TRY(D.trajectories(&R.P, live, cfg->n_steps, kIdxSteps2));
    lap(4);
    // 6. V(q') and T(p', H(q')) of every chain that was not a dead end
    scored.clear();
    for (int64_t c = 0; c < n; ++c)
      if (!R.ch[c].dead) scored.push_back(c);
    RJ_TRY(D.energies(&R.P, scored, cfg->f_pos, order, kIdxV1, w->Vd));
    if (int rc = rhmc_kinetic_rows_device(ctx, &R.P, w->Q, w->P, W, w->Kd, nullptr, nullptr, n,
                                          w->T1d, s0))
      return D.engine_fail(rc, "kinetic");
    lap(4);
    // while they run: each scored chain's accept uniform (:1072, :1120), and
    // for a chain whose star count cannot change the next iteration's draws
    const bool next = l + 1 < rows_n;
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      if (h.dead) {
        h.K = h.K0;
      } else {
        h.u = std::log(h.rng.random_sample());
        if (h.move != 0) return;
      }
      if (!next) return;
      const int mv = h.move;  // this iteration's, for its accept step
      const bool gr = h.grow;
      h.znext.resize(3 * (size_t)h.K);
      draw_start(h, h.znext.data());
      h.move_next = h.move;
      h.grow_next = h.grow;
      h.move = mv;
      h.grow = gr;
      h.pre = true;
    });
    lap(0);
    RJ_TRY(D.wait(0));  // V(q') and T'
    for (size_t j = 0; j < order.size(); ++j) V1[order[j]] = w->Vh[j];
    lap(5);
    // 7. accept / reject (:1072-1083, :1120-1131); accepted rows become Q0
    std::vector<char> acc((size_t)n, 0);
    R.parallel(all, [&](int64_t c) {
      Chain& h = R.ch[c];
      const int64_t r = l * rec_stride + rec_off + c;
      bool a = false;
      if (!h.dead) {
        const double E1 = V1[c] + w->T1h[c];
        const double u = h.u;
        if (h.move == 0) {
          const double dE = E1 - h.E0;
          a = (dE < 0) || (u < -dE);
        } else {
          const double ln_alpha0 = -(E1 - h.E0) + h.factor;
          a = (ln_alpha0 > 0) || (u < ln_alpha0);
        }
        if (!a) h.K = h.K0;
      }
      acc[c] = a;
      V_end[c] = a ? V1[c] : V0[c];
      if (rec) {
        if (rec->accept) rec->accept[r] = a ? 1 : 0;
        if (rec->flags) rec->flags[r] = h.dead ? (int32_t)RHMC_RJ_DEAD_END : 0;
      }
    });
    acc_rows.clear();
    int32_t kacc = 1;  // an accepted row's columns: its old and new stars
    for (int64_t c = 0; c < n; ++c) {
      if (acc[c]) {
        acc_rows.push_back(c);
        kacc = std::max(kacc, std::max(R.ch[c].K0, R.ch[c].K));
      }
      Kc[c] = R.ch[c].K;
    }
    if (!acc_rows.empty()) {
      const int64_t dc = std::min<int64_t>(W, 3 * (int64_t)kacc);
      int64_t* cd = D.idx_d(kIdxCommit);
      std::copy(acc_rows.begin(), acc_rows.end(), D.idx_h(kIdxCommit));
      if (int rc = rhmc_rows_copy_device(ctx, w->Q, W, cd, w->Q0, W, cd,
                                         (int64_t)acc_rows.size(), (int32_t)dc, s0))
        return D.engine_fail(rc, "commit");
    }
    lap(6);
    V_end_g_ff2 = R.P.g_ff2;
    V_end_beta = R.P.beta;
    V_end_ok = true;
  }
#ifdef RHMC_RJ_TIMING
  const auto t_loop1 = std::chrono::steady_clock::now();
#endif
  // the final states: the live columns (3 K_max) back, zeros past 3 K
  int32_t kout = 1;
  for (int64_t c = 0; c < n; ++c) kout = std::max(kout, R.ch[c].K);
  const int64_t w1 = 3 * (int64_t)kout;
  if (int rc = rhmc_rows_copy_device(ctx, w->Q0, W, nullptr, w->Zd, w1, nullptr, n, (int32_t)w1,
                                     s0))
    return D.engine_fail(rc, "final rows");
  RJ_HIP(hipStreamSynchronize(s0));
  R.parallel(all, [&](int64_t c) {
    // ZP_STARTS: the caller's row is zero past 3 K_in, so the zeros stop there
    const int64_t d = 3 * (int64_t)R.ch[c].K;
    put_row(q + c * W, w->Zh + c * w1, d,
            (cfg->records_zero_padded & RHMC_RJ_ZP_STARTS) ? std::max(d, 3 * (int64_t)K_in[c]) : W,
            W);
    _mm_sfence();
    const Chain& h = R.ch[c];
    K[c] = h.K;
    if (cfg->states) {
      rhmc_np_state& st = cfg->states[rec_off + c];
      h.rng.get_state(st.key, &st.pos, &st.has_gauss, &st.gauss);
    }
  });
  if (phase_out)
    for (int i = 0; i < 7; ++i) phase_out[i] += phase[i];
#ifdef RHMC_RJ_TIMING  // diagnostic build: setup / iterations / teardown of a pipe
  const auto t_end = std::chrono::steady_clock::now();
  auto ms = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count() * 1e3; };
  std::fprintf(stderr, "rj pipe n=%lld setup %.3f ms iterations %.3f ms teardown %.3f ms\n",
               (long long)n, ms(t_setup0, t_loop0), ms(t_loop0, t_loop1), ms(t_loop1, t_end));
#endif
  return 0;
}

// Split n chains into `pipes` contiguous parts run concurrently, part i on
// its own host thread (part 0 on the caller's), all on one shared pool of
// nt - pipes workers: body(i, first chain, count, pool, phase[7]) -> rc.  The
// first failing part's error is the one reported.
template <class Body>
int run_pipes(int pipes, int64_t n, int nt, double* phase, Body body) {
  const std::shared_ptr<Pool> pool = shared_pool(std::max(0, nt - std::max(1, pipes)));
  // one part's body on this thread; an exception becomes an error code (no
  // C++ exception may cross the ABI, and none may leave a std::thread)
  auto guarded = [&](int i, int64_t f, int64_t m, double* ph, std::string& err) {
    try {
      const int rc = body(i, f, m, pool.get(), ph);
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
    const int rc = guarded(0, 0, n, phase, err);
    if (rc) g_err = err;
    return rc;
  }
  std::vector<int64_t> first((size_t)pipes + 1);
  for (int i = 0; i <= pipes; ++i) first[i] = n * i / pipes;
  std::vector<std::array<double, 7>> ph((size_t)pipes);
  std::vector<int> rcs((size_t)pipes, 0);
  std::vector<std::string> errs((size_t)pipes);
  std::vector<std::thread> ts;
  ts.reserve((size_t)pipes);
  for (int i = 1; i < pipes; ++i) {
    ph[i].fill(0.);
    try {
      ts.emplace_back([&, i] {
        rcs[i] = guarded(i, first[i], first[i + 1] - first[i], ph[i].data(), errs[i]);
      });
    } catch (const std::exception& e) {  // this part does not run: report it
      rcs[i] = RHMC_ERR_NOMEM;
      errs[i] = std::string("cannot start a pipe thread: ") + e.what();
    }
  }
  ph[0].fill(0.);
  rcs[0] = guarded(0, first[0], first[1] - first[0], ph[0].data(), errs[0]);
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
  // default for the device-resident driver, measured at big-sim4 geometry
  // (profiles/r05_pipes/, three repeats on one box, chain-steps/s): 4,096
  // chains 1.70e7 / 1.82e7 / 1.84e7 with 2 / 3 / 4 pipes; 16,384 chains
  // 1.80e7 / 2.06e7 / 2.12e7.  After the ragged pixel-major launches
  // (profiles/r05_pipes2/, r05_pipes3/, four repeats): 4,096 chains B4 2.62e7 /
  // 2.72e7 with 3 / 4 pipes, the flagship 2.64e7 / 2.78e7; 6 and 8 pipes
  // (more streams than the box's 4 hardware queues) 0.75-0.95x.  At 16,384
  // chains 8 pipes beat 4 (profiles/r05_pipes8/, two repeats): B4 3.28e7 /
  // 3.18e7 against 2.94e7 / 2.82e7 (4,096 chains: 0.6x)
  int pipes = cfg->n_pipes > 0
                  ? cfg->n_pipes
                  : (n >= 16384 ? 8 : n >= 4096 ? 4 : n >= 2048 ? 3 : n >= 1024 ? 2 : 1);
  return (int)std::max<int64_t>(1, std::min<int64_t>(pipes, n));
}

}  // namespace

extern "C" {

int rhmc_rj_run_physics(const rhmc_rj_physics* phys, const rhmc_params* P,
                        const rhmc_rj_config* cfg, double* q, int32_t* K, const uint32_t* seeds,
                        int64_t n, const rhmc_rj_record* rec) {
  try {
    if (int rc = check(P, cfg, q, K, seeds, n)) return rc;
    if (int rc = check_records(cfg, rec)) return rc;
    double phase[7] = {0, 0, 0, 0, 0, 0, 0};
    const int nt = host_threads(cfg);
    // with pipes > 1 the callbacks are called from that many threads at once
    const int64_t W = 3 * (int64_t)cfg->N_max;
    int rc = run_pipes(cfg->n_pipes > 1 ? pipes_for(cfg, n) : 1, n, nt, phase,
                       [&](int, int64_t f, int64_t m, Pool* pool, double* ph) {
                         return run(phys, P, cfg, q + f * W, K + f,
                                    seeds ? seeds + f : nullptr, m, rec, n, f, pool, ph);
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
#ifdef RHMC_RJ_TIMING
  const auto t_entry = std::chrono::steady_clock::now();
  auto ms_since = [&] {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_entry).count() * 1e3;
  };
#endif
  try {
    if (int rc = check(P, cfg, q, K, seeds, n)) return rc;
    if (int rc = check_records(cfg, rec)) return rc;
    const double* dimg = nullptr;
    if (int rc = rhmc_ctx_image_device(ctx, &dimg)) return rc;
    if (!dimg) return fail(RHMC_ERR_ARG, "context has no image");
    hipPointerAttribute_t at;
    RJ_HIP(hipPointerGetAttributes(&at, dimg));
    const int dev = at.device;
    DeviceGuard guard;  // the caller's device comes back on return
    RJ_HIP(hipSetDevice(dev));
    const int pipes = pipes_for(cfg, n);
    const int nt = host_threads(cfg);
    // each pipe on its own process-lifetime buffers and streams, held for the run
    Work* works[kMaxPipes] = {};
    std::unique_lock<std::mutex> locks[kMaxPipes];
    for (int i = 0; i < pipes; ++i) {
      works[i] = work_for(dev, i);
      locks[i] = std::unique_lock<std::mutex>(works[i]->mu);
    }
    const int64_t W = 3 * (int64_t)cfg->N_max;
    double phase[7] = {0, 0, 0, 0, 0, 0, 0};
#ifdef RHMC_RJ_TIMING
    std::fprintf(stderr, "rj run: pipes start at %.3f ms\n", ms_since());
#endif
    const int rc = run_pipes(pipes, n, nt, phase, [&](int i, int64_t f, int64_t m, Pool* pool,
                                                      double* ph) {
#ifdef RHMC_RJ_TIMING
      std::fprintf(stderr, "rj run: pipe %d starts at %.3f ms\n", i, ms_since());
#endif
      if (hipSetDevice(dev) != hipSuccess) return fail(RHMC_ERR_HIP, "hipSetDevice failed");
      const int rc_i = run_device(ctx, dev, works[i], P, cfg, q + f * W, K + f,
                                  seeds ? seeds + f : nullptr, m, rec, n, f, pool, ph);
#ifdef RHMC_RJ_TIMING
      std::fprintf(stderr, "rj run: pipe %d returns at %.3f ms\n", i, ms_since());
#endif
      return rc_i;
    });
#ifdef RHMC_RJ_TIMING
    std::fprintf(stderr, "rj run: pipes joined at %.3f ms\n", ms_since());
#endif
    if (rc == 0 && rec && rec->phase_s) std::copy(phase, phase + 7, rec->phase_s);
    return rc;
  } catch (const std::exception& e) {
    return fail(RHMC_ERR_NOMEM, std::string("host exception: ") + e.what());
  }
}

int rhmc_rj_release(int32_t device) {
  try {
    DeviceGuard guard;
    std::lock_guard<std::mutex> lock(g_work_mu);
    for (auto it = g_work.begin(); it != g_work.end();) {
      if (device >= 0 && it->first.first != device) {
        ++it;
        continue;
      }
      Work* w = it->second;
      {
        std::lock_guard<std::mutex> l(w->mu);  // a run using it finishes first
        w->destroy();
      }
      delete w;
      it = g_work.erase(it);
    }
    return 0;
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

int rhmc_rj_pack_starts(const double* rows, const int32_t* K, int64_t n, int32_t N_max,
                        double flux_to_count, double* q) {
  return rhmc_rj_pack_starts_padded(rows, K, n, N_max, flux_to_count, q, nullptr);
}

int rhmc_rj_pack_starts_padded(const double* rows, const int32_t* K, int64_t n, int32_t N_max,
                               double flux_to_count, double* q, const int32_t* K_prev) {
  if (n < 0 || N_max < 1) return fail(RHMC_ERR_ARG, "bad n or N_max");
  if (n > 0 && (!rows || !K || !q)) return fail(RHMC_ERR_ARG, "rows, K or q is NULL");
  const int64_t W = 3 * (int64_t)N_max;
  std::vector<int64_t> at;
  try {
    at.resize((size_t)n + 1);
  } catch (...) {
    return fail(RHMC_ERR_NOMEM, "pack_starts: out of host memory");
  }
  at[0] = 0;
  for (int64_t c = 0; c < n; ++c) {
    if (K[c] < 1 || K[c] > N_max) return fail(RHMC_ERR_ARG, "K[c] must be in [1, N_max]");
    at[c + 1] = at[c] + 3 * (int64_t)K[c];
  }
  auto pack = [&](int64_t c0, int64_t c1) {
    std::vector<double> tmp((size_t)W);
    // pow is a pure function: a small direct-mapped memo of magnitudes (the
    // flagship starts every chain from the same model stars)
    uint64_t memo_key[64];
    double memo_val[64];
    bool memo_ok[64] = {};
    for (int64_t c = c0; c < c1; ++c) {
      const double* src = rows + at[c];
      for (int32_t k = 0; k < K[c]; ++k) {
        const double v = src[3 * k];
        // mag2flux_converter (sampler_RHMC.py:147-152, utils.py:24-25): libm pow,
        // the function NumPy's and Python's float power call
        double f = v;
        if (flux_to_count > 0) {
          uint64_t bits;
          std::memcpy(&bits, &v, 8);
          const int slot = (int)((bits * 0x9E3779B97F4A7C15ull) >> 58);
          if (!memo_ok[slot] || memo_key[slot] != bits) {
            memo_key[slot] = bits;
            memo_val[slot] = std::pow(10.0, 0.4 * (22.5 - v));
            memo_ok[slot] = true;
          }
          f = memo_val[slot] * flux_to_count;
        }
        tmp[3 * k] = f;
        tmp[3 * k + 1] = src[3 * k + 1];
        tmp[3 * k + 2] = src[3 * k + 2];
      }
      // zero-padded (streamed), or only up to the row's old width
      const int64_t d = 3 * (int64_t)K[c];
      const int32_t kp = K_prev ? K_prev[c] : 0;
      put_row(q + c * W, tmp.data(), d, kp >= 1 && kp <= N_max ? std::max(d, 3 * (int64_t)kp) : W,
              W);
    }
    _mm_sfence();
  };
  // a few host threads for large batches (one pow per distinct magnitude, a
  // 3 N_max row of stores per chain); chains split in contiguous ranges, so
  // the result does not depend on the thread count
  const int64_t work = at[n];
  const int nt = (int)std::min<int64_t>(8, std::max<int64_t>(1, work / 60000));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) {
    const int64_t c0 = n * t / nt, c1 = n * (t + 1) / nt;
    try {
      th.emplace_back(pack, c0, c1);
    } catch (...) {  // no thread: this thread packs the range
      pack(c0, c1);
    }
  }
  pack(0, nt > 1 ? n / nt : n);
  for (auto& t : th) t.join();
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
