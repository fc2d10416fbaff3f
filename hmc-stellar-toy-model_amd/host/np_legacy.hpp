// np_legacy.hpp — a replica of numpy.random.RandomState (NumPy's legacy
// generator): MT19937 seeded like RandomState(int) (mt19937_seed), and the
// legacy algorithms of numpy/random/src/legacy/legacy-distributions.c and
// numpy/random/src/distributions that RandomState methods call:
//   random_sample  genrand_res53: (a >> 5, b >> 6) -> (a 2^26 + b) / 2^53
//   randn          legacy_gauss: Marsaglia polar method, the second value cached
//   randint        bounded masked rejection on 32-bit draws (use_masked=True)
//   standard_exponential  -log(1 - U)
//   standard_gamma legacy_standard_gamma (Marsaglia-Tsang for shape > 1)
//   beta           legacy_beta (Johnk for a, b <= 1, else a gamma ratio)
// Every draw is bit-identical to NumPy's when this file is compiled without
// floating-point contraction (-ffp-contract=off, as NumPy's own C code is):
// tests/test_rj_native_host.py compares long streams of every kind.
#pragma once
#include <cmath>
#include <cstdint>

namespace rhmc_np {

class Legacy {
 public:
  explicit Legacy(uint32_t seed = 0) { this->seed(seed); }

  void seed(uint32_t s) {  // mt19937_seed
    for (int i = 0; i < kN; ++i) {
      key_[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    pos_ = kN;
    has_gauss_ = false;
    gauss_ = 0.0;
  }

  // RandomState.get_state() / set_state() (key, pos, has_gauss, cached_gaussian)
  void get_state(uint32_t* key, int32_t* pos, int32_t* has_gauss, double* gauss) const {
    for (int i = 0; i < kN; ++i) key[i] = key_[i];
    *pos = pos_;
    *has_gauss = has_gauss_ ? 1 : 0;
    *gauss = gauss_;
  }
  bool set_state(const uint32_t* key, int32_t pos, int32_t has_gauss, double gauss) {
    if (pos < 0 || pos > kN) return false;
    for (int i = 0; i < kN; ++i) key_[i] = key[i];
    pos_ = pos;
    has_gauss_ = has_gauss != 0;
    gauss_ = has_gauss_ ? gauss : 0.0;
    return true;
  }

  uint32_t next32() {
    if (pos_ == kN) generate();
    uint32_t y = key_[pos_++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  double random_sample() {
    const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
  }

  double gauss() {
    if (has_gauss_) {
      has_gauss_ = false;
      const double t = gauss_;
      gauss_ = 0.0;
      return t;
    }
    double x1, x2, r2;
    do {
      x1 = 2.0 * random_sample() - 1.0;
      x2 = 2.0 * random_sample() - 1.0;
      r2 = x1 * x1 + x2 * x2;
    } while (r2 >= 1.0 || r2 == 0.0);
    const double f = std::sqrt(-2.0 * std::log(r2) / r2);
    gauss_ = f * x1;
    has_gauss_ = true;
    return f * x2;
  }

  // randint(low, high) for one value: rng = high - low - 1, masked rejection
  int64_t randint(int64_t low, int64_t high) {
    const uint64_t rng = (uint64_t)(high - low - 1);
    if (rng == 0) return low;
    if (rng <= 0xFFFFFFFFull) {
      if (rng == 0xFFFFFFFFull) return low + (int64_t)next32();
      uint32_t mask = (uint32_t)rng;
      mask |= mask >> 1;
      mask |= mask >> 2;
      mask |= mask >> 4;
      mask |= mask >> 8;
      mask |= mask >> 16;
      uint32_t v;
      while ((v = (next32() & mask)) > (uint32_t)rng) {
      }
      return low + (int64_t)v;
    }
    uint64_t mask = rng;  // 64-bit ranges (not used by the sampler)
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    mask |= mask >> 32;
    uint64_t v;
    do {
      v = ((uint64_t)next32() << 32) | next32();
      v &= mask;
    } while (v > rng);
    return low + (int64_t)v;
  }

  double standard_exponential() { return -std::log(1.0 - random_sample()); }

  double standard_gamma(double shape) {
    if (shape == 1.0) return standard_exponential();
    if (shape == 0.0) return 0.0;
    if (shape < 1.0) {
      for (;;) {
        const double U = random_sample();
        const double V = standard_exponential();
        if (U <= 1.0 - shape) {
          const double X = std::pow(U, 1. / shape);
          if (X <= V) return X;
        } else {
          const double Y = -std::log((1 - U) / shape);
          const double X = std::pow(1.0 - shape + shape * Y, 1. / shape);
          if (X <= (V + Y)) return X;
        }
      }
    }
    const double b = shape - 1. / 3.;
    const double c = 1. / std::sqrt(9 * b);
    for (;;) {
      double X, V;
      do {
        X = gauss();
        V = 1.0 + c * X;
      } while (V <= 0.0);
      V = V * V * V;
      const double U = random_sample();
      if (U < 1.0 - 0.0331 * (X * X) * (X * X)) return b * V;
      if (std::log(U) < 0.5 * X * X + b * (1. - V + std::log(V))) return b * V;
    }
  }

  double beta(double a, double b) {
    if (a <= 1.0 && b <= 1.0) {
      for (;;) {
        const double U = random_sample();
        const double V = random_sample();
        const double X = std::pow(U, 1.0 / a);
        const double Y = std::pow(V, 1.0 / b);
        if ((X + Y) <= 1.0) {
          if (X + Y > 0) return X / (X + Y);
          double logX = std::log(U) / a;
          double logY = std::log(V) / b;
          const double logM = logX > logY ? logX : logY;
          logX -= logM;
          logY -= logM;
          return std::exp(logX - std::log(std::exp(logX) + std::exp(logY)));
        }
      }
    }
    const double Ga = standard_gamma(a);
    const double Gb = standard_gamma(b);
    return Ga / (Ga + Gb);
  }

 private:
  static constexpr int kN = 624, kM = 397;
  void generate() {
    constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
    int i = 0;
    uint32_t y;
    for (; i < kN - kM; ++i) {
      y = (key_[i] & kUpper) | (key_[i + 1] & kLower);
      key_[i] = key_[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      y = (key_[i] & kUpper) | (key_[i + 1] & kLower);
      key_[i] = key_[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    y = (key_[kN - 1] & kUpper) | (key_[0] & kLower);
    key_[kN - 1] = key_[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    pos_ = 0;
  }

  uint32_t key_[kN];
  int pos_;
  bool has_gauss_;
  double gauss_;
};

// numpy's pairwise summation of a contiguous float64 array (np.sum over one
// axis: pairwise_sum_DOUBLE, blocks of 128, eight accumulators).
inline double pairwise_sum(const double* a, int64_t n) {
  if (n < 8) {
    double r = 0.;
    for (int64_t i = 0; i < n; ++i) r += a[i];
    return r;
  }
  if (n <= 128) {
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
      for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
  }
  int64_t n2 = n / 2;
  n2 -= n2 % 8;
  return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

}  // namespace rhmc_np
