// Host record-write bandwidth of the RJ driver's accept step (tools only):
// rows of W doubles, 3 K live columns copied from a staging row and the rest
// zero-filled, over n chains x rows_n iterations, split over T threads as the
// pipes split them.  Plain stores (std::copy / std::fill) against
// non-temporal SSE2 stores.  usage: rec_write_bench [n] [W] [K] [rows] [T]
#include <emmintrin.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
#include <algorithm>

static void row_plain(double* dst, const double* src, long d, long W) {
  std::fill(std::copy(src, src + d, dst), dst + W, 0.);
}

static void row_nt(double* dst, const double* src, long d, long W) {
  long i = 0;
  for (; i < W && (reinterpret_cast<uintptr_t>(dst + i) & 15); ++i) dst[i] = i < d ? src[i] : 0.;
  const __m128d z = _mm_setzero_pd();
  for (; i + 2 <= d; i += 2) _mm_stream_pd(dst + i, _mm_loadu_pd(src + i));
  if (i < d && i + 2 <= W) {
    _mm_stream_pd(dst + i, _mm_set_pd(0., src[i]));
    i += 2;
  }
  for (; i + 2 <= W; i += 2) _mm_stream_pd(dst + i, z);
  for (; i < W; ++i) dst[i] = i < d ? src[i] : 0.;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 4096, W = argc > 2 ? atol(argv[2]) : 360;
  const long K = argc > 3 ? atol(argv[3]) : 8, rows = argc > 4 ? atol(argv[4]) : 10;
  const int T = argc > 5 ? atoi(argv[5]) : 16;
  std::vector<double> q((size_t)rows * n * W), p((size_t)rows * n * W), st((size_t)n * W, 1.5);
  for (int mode = 0; mode < 2; ++mode)
    for (int rep = 0; rep < 4; ++rep) {
      const auto t0 = std::chrono::steady_clock::now();
      for (long l = 0; l < rows; ++l) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t] {
            for (long c = t; c < n; c += T) {
              double* dq = q.data() + ((size_t)l * n + c) * W;
              double* dp = p.data() + ((size_t)l * n + c) * W;
              const double* s = st.data() + (size_t)c * W;
              if (mode == 0) {
                row_plain(dq, s, 3 * K, W);
                row_plain(dp, s, 3 * K, W);
              } else {
                row_nt(dq, s, 3 * K, W);
                row_nt(dp, s, 3 * K, W);
              }
            }
            _mm_sfence();
          });
        for (auto& x : th) x.join();
      }
      const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      const double bytes = 2.0 * rows * n * W * 8;
      std::printf("%s rep %d: %.2f ms, %.1f GB/s (n %ld W %ld K %ld rows %ld threads %d)\n",
                  mode ? "non-temporal" : "plain", rep, s * 1e3, bytes / s / 1e9, n, W, K, rows, T);
    }
  return 0;
}
