// Host AddressSanitizer driver for the C-ABI (include/rhmc.h).  The library's
// host code (argument checks, staging, context lifetime, error strings) is
// built with -Xarch_host -fsanitize=address (device code unchanged) and linked
// into this program by `make -C hmc-stellar-toy-model_amd asan`.
//
//   capi_asan cpu   error paths that need no GPU (NULL / bad arguments, no device)
//   capi_asan gpu   every entry point on small batches (rhmc_energy_device too): ragged chain counts,
//                   image resize, K = 1 / 3 / 12, all solvers, MH with host and
//                   device randoms and records, data generation, context churn
//
// Exit status 0 = every check passed and ASan reported nothing (ASan aborts
// the process on the first heap error).  tests/test_asan_host.py runs it.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "rhmc.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                   \
      std::fprintf(stderr, " [%s]\n", rhmc_last_error());  \
      ++g_fail;                                            \
    }                                                      \
  } while (0)

// C2-like parameters (SURVEY §8(a) a7 constants, g_xx = g_ff = g_ff2 = 1).
static rhmc_params params() {
  rhmc_params P;
  std::memset(&P, 0, sizeof(P));
  P.dt = 0.1;
  P.delta = 1e-6;
  P.B_count = 24.98145266935892;
  P.f_lim = 24.98145266935892;
  P.f_low = 3.9592934273456466;
  P.fwhm_pix = 3.4999999999999996;
  P.g_xx = P.g_ff = P.g_ff2 = 1.0;
  P.g0 = 0.035997054345069765;
  P.g1 = 0.4523523265306124;
  P.g2 = 0.008141675878296745;
  P.alpha = 2.0;
  P.counter_max = 1000;
  return P;
}

struct Rng {  // deterministic normals / uniforms (xorshift64* + Box-Muller)
  uint64_t s = 0x9E3779B97F4A7C15ull;
  double uni() {
    s ^= s >> 12;
    s ^= s << 25;
    s ^= s >> 27;
    return ((s * 2685821657736338717ull) >> 11) * 0x1p-53 + 0x1p-54;
  }
  double normal() { return std::sqrt(-2.0 * std::log(uni())) * std::cos(6.283185307179586 * uni()); }
};

static bool all_finite(const std::vector<double>& v) {
  for (double x : v)
    if (!std::isfinite(x)) return false;
  return true;
}

static void cpu_checks() {
  CHECK(rhmc_abi_version() == RHMC_ABI_VERSION, "abi version");
  int n = -1;
  CHECK(rhmc_device_count(&n) == RHMC_OK && n >= 0, "device count");
  CHECK(rhmc_device_count(nullptr) == RHMC_ERR_ARG, "device count NULL");
  CHECK(std::strlen(rhmc_last_error()) > 0, "error message set");
  rhmc_ctx* ctx = nullptr;
  std::vector<double> D(48 * 48, 25.0);
  CHECK(rhmc_ctx_create(0, D.data(), 48, 48, nullptr) == RHMC_ERR_ARG, "create NULL out");
  if (n == 0) {
    CHECK(rhmc_ctx_create(0, D.data(), 48, 48, &ctx) == RHMC_ERR_HIP && !ctx, "create, no GPU");
  }
  const rhmc_params P = params();
  std::vector<double> q(3), p(3);
  CHECK(rhmc_leapfrog(nullptr, &P, q.data(), p.data(), 1, 1, 1, nullptr, nullptr) == RHMC_ERR_ARG,
        "leapfrog NULL ctx");
  CHECK(rhmc_gradient(nullptr, &P, q.data(), p.data(), 1, 1, 0) == RHMC_ERR_ARG, "gradient");
  CHECK(rhmc_energy(nullptr, &P, q.data(), p.data(), q.data(), p.data(), 1, 1, 0) == RHMC_ERR_ARG,
        "energy");
  CHECK(rhmc_energy_device(nullptr, &P, q.data(), p.data(), q.data(), p.data(), 1, 1, 0,
                           nullptr) == RHMC_ERR_ARG, "energy_device");
  CHECK(rhmc_integrate(nullptr, &P, 1, q.data(), p.data(), 1, 1, 1, 0, nullptr) == RHMC_ERR_ARG,
        "integrate");
  CHECK(rhmc_mh(nullptr, &P, q.data(), 1, 1, 1, 1, 0, nullptr, nullptr, 1, nullptr) ==
            RHMC_ERR_ARG, "mh");
  CHECK(rhmc_ctx_set_option(nullptr, RHMC_OPT_KERNEL, 0) == RHMC_ERR_ARG, "set_option");
  CHECK(rhmc_ctx_set_image(nullptr, D.data(), 48, 48) == RHMC_ERR_ARG, "set_image");
  CHECK(rhmc_ctx_synchronize(nullptr) == RHMC_ERR_ARG, "synchronize");
  rhmc_ctx_destroy(nullptr);
}

// n chains of K stars around the image centre, momenta ~ 0.1 N(0, 1) (flux
// momenta scaled by sqrt(f)).
static void chains(Rng& r, int64_t n, int K, int side, std::vector<double>& q,
                   std::vector<double>& p) {
  q.assign(n * 3 * K, 0.0);
  p.assign(n * 3 * K, 0.0);
  for (int64_t c = 0; c < n; ++c)
    for (int k = 0; k < K; ++k) {
      double* s = &q[(c * K + k) * 3];
      s[0] = 800.0 + 400.0 * r.uni();
      s[1] = side * (0.25 + 0.5 * r.uni());
      s[2] = side * (0.25 + 0.5 * r.uni());
      double* m = &p[(c * K + k) * 3];
      m[0] = 0.1 * std::sqrt(s[0]) * r.normal();
      m[1] = 0.1 * r.normal();
      m[2] = 0.1 * r.normal();
    }
}

static void gpu_checks() {
  Rng r;
  rhmc_params P = params();
  for (int round = 0; round < 2; ++round) {  // context churn
    rhmc_ctx* ctx = nullptr;
    CHECK(rhmc_ctx_create(0, nullptr, 0, 0, &ctx) == RHMC_OK && ctx, "create (no image)");
    if (!ctx) return;
    // image: a Poisson realisation of one star, installed on the device
    const double truth[3] = {994.53, 24.3, 23.8};
    std::vector<double> model(48 * 48);
    CHECK(rhmc_gen_image(ctx, &P, truth, 1, 48, 48, 0, 0, model.data(), 0) == RHMC_OK, "model");
    CHECK(all_finite(model) && model[24 * 48 + 24] > P.B_count, "model values");
    CHECK(rhmc_gen_image(ctx, &P, truth, 1, 48, 48, 1, 77, nullptr, 1) == RHMC_OK, "install");
    std::vector<double> reals(3 * 32 * 32);
    CHECK(rhmc_gen_image(ctx, &P, truth, 1, 32, 32, 3, 5, reals.data(), 0) == RHMC_OK, "reals");

    for (int K : {1, 3, 12, 100}) {
      const int64_t n = (K == 1) ? 37 : 13;  // ragged: not a multiple of any wave size
      std::vector<double> q, p;
      chains(r, n, K, 48, q, p);
      std::vector<double> q2 = q, p2 = p, q0 = q, p0 = p;
      std::vector<int32_t> it(2 * n), st(n);
      CHECK(rhmc_leapfrog(ctx, &P, q.data(), p.data(), n, K, 20, it.data(), st.data()) == RHMC_OK,
            "leapfrog K=%d", K);
      // random stars on a one-star image can legitimately blow up (the
      // reference does too); what must hold is that exactly those chains are
      // flagged, and that a second run is bit-identical
      for (int64_t c = 0; c < n; ++c) {
        bool fin = true;
        for (int i = 0; i < 3 * K; ++i)
          fin = fin && std::isfinite(q[c * 3 * K + i]) && std::isfinite(p[c * 3 * K + i]);
        CHECK(fin == !(st[c] & RHMC_STATUS_NONFINITE), "NONFINITE flag chain %lld K=%d",
              (long long)c, K);
      }
      CHECK(rhmc_leapfrog(ctx, &P, q2.data(), p2.data(), n, K, 20, nullptr, nullptr) == RHMC_OK &&
                std::memcmp(q2.data(), q.data(), q.size() * sizeof(double)) == 0 &&
                std::memcmp(p2.data(), p.data(), p.size() * sizeof(double)) == 0,
            "leapfrog deterministic K=%d", K);
      q = q0;  // the other entry points start from the (finite) initial states
      p = p0;
      std::vector<double> g(n * 3 * K), V(n), T(n);
      CHECK(rhmc_gradient(ctx, &P, q.data(), g.data(), n, K, 1) == RHMC_OK && all_finite(g),
            "gradient K=%d", K);
      CHECK(rhmc_energy(ctx, &P, q.data(), p.data(), V.data(), T.data(), n, K, 0) == RHMC_OK,
            "energy K=%d", K);
      {  // the device-buffer entry point on the context's stream: the same launch, same bits
        double *dq = nullptr, *dp = nullptr, *dV = nullptr, *dT = nullptr;
        const size_t sb = q.size() * sizeof(double), eb = (size_t)n * sizeof(double);
        CHECK(hipMalloc(&dq, sb) == hipSuccess && hipMalloc(&dp, sb) == hipSuccess &&
                  hipMalloc(&dV, eb) == hipSuccess && hipMalloc(&dT, eb) == hipSuccess,
              "hipMalloc K=%d", K);
        CHECK(hipMemcpy(dq, q.data(), sb, hipMemcpyHostToDevice) == hipSuccess &&
                  hipMemcpy(dp, p.data(), sb, hipMemcpyHostToDevice) == hipSuccess,
              "H2D K=%d", K);
        CHECK(rhmc_energy_device(ctx, &P, dq, dp, dV, dT, n, K, 0, nullptr) == RHMC_OK &&
                  rhmc_ctx_synchronize(ctx) == RHMC_OK, "energy_device K=%d", K);
        std::vector<double> V2(n), T2(n);
        CHECK(hipMemcpy(V2.data(), dV, eb, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemcpy(T2.data(), dT, eb, hipMemcpyDeviceToHost) == hipSuccess,
              "D2H K=%d", K);
        CHECK(std::memcmp(V2.data(), V.data(), eb) == 0 && std::memcmp(T2.data(), T.data(), eb) == 0,
              "energy_device == energy K=%d", K);
        CHECK(rhmc_energy_device(ctx, &P, nullptr, dp, dV, dT, n, K, 0, nullptr) == RHMC_ERR_ARG,
              "energy_device NULL q");
        (void)hipFree(dq);
        (void)hipFree(dp);
        (void)hipFree(dV);
        (void)hipFree(dT);
      }
      for (int solver = RHMC_SOLVER_HMC; solver <= RHMC_SOLVER_RHMC_LEAPFROG; ++solver) {
        std::vector<double> qs = q, ps = p;
        CHECK(rhmc_integrate(ctx, &P, solver, qs.data(), ps.data(), n, K, 10, 1, st.data()) ==
                  RHMC_OK, "integrate solver=%d K=%d", solver, K);
      }
      std::vector<double> dtv(3 * K);
      for (int k = 0; k < K; ++k) {
        dtv[3 * k] = 2.0;
        dtv[3 * k + 1] = dtv[3 * k + 2] = 0.02;
      }
      std::vector<int32_t> steps(n);
      for (int64_t c = 0; c < n; ++c) steps[c] = 1 + (int32_t)(c % 7);
      std::vector<double> qh = q, ph = p;
      CHECK(rhmc_hmc_random(ctx, &P, dtv.data(), qh.data(), ph.data(), steps.data(), n, K,
                            st.data()) == RHMC_OK, "hmc_random K=%d", K);
      // MH: host randoms with every record, then device randoms without
      const int iters = 3, nst = 10;
      std::vector<double> z((size_t)iters * n * 3 * K), u((size_t)iters * n);
      for (double& v : z) v = r.normal();
      for (double& v : u) v = r.uni();
      std::vector<double> qc((size_t)iters * n * 3 * K), Ec(iters * n), Vc(iters * n),
          Tc(iters * n);
      std::vector<int32_t> acc(iters * n);
      rhmc_mh_record rec{qc.data(), Ec.data(), Vc.data(), Tc.data(), acc.data()};
      std::vector<double> qm = q;
      CHECK(rhmc_mh(ctx, &P, qm.data(), n, K, iters, nst, 0, z.data(), u.data(), 0, &rec) ==
                RHMC_OK, "mh host randoms K=%d", K);
      CHECK(all_finite(qm) && all_finite(qc), "mh finite K=%d", K);
      CHECK(rhmc_mh(ctx, &P, qm.data(), n, K, iters, nst, 0, nullptr, nullptr, 123, nullptr) ==
                RHMC_OK, "mh philox K=%d", K);
    }
    // resize the image (48 -> 32 px), options, errors on a live context
    std::vector<double> D32(reals.begin(), reals.begin() + 32 * 32);
    CHECK(rhmc_ctx_set_image(ctx, D32.data(), 32, 32) == RHMC_OK, "set_image 32");
    CHECK(rhmc_ctx_set_image(ctx, D32.data(), 32, 16) == RHMC_ERR_ARG, "non-square image");
    CHECK(rhmc_ctx_set_option(ctx, RHMC_OPT_KERNEL, RHMC_KERNEL_WINDOWED) == RHMC_OK, "option");
    CHECK(rhmc_ctx_set_option(ctx, 99, 0) == RHMC_ERR_ARG, "unknown option");
    {
      std::vector<double> q, p;
      chains(r, 9, 2, 32, q, p);
      std::vector<int32_t> st(9);
      CHECK(rhmc_leapfrog(ctx, &P, q.data(), p.data(), 9, 2, 15, nullptr, st.data()) == RHMC_OK,
            "leapfrog 32 px windowed");
      for (int c = 0; c < 9; ++c) {
        bool fin = true;
        for (int i = 0; i < 6; ++i) fin = fin && std::isfinite(q[c * 6 + i]) && std::isfinite(p[c * 6 + i]);
        CHECK(fin == !(st[c] & RHMC_STATUS_NONFINITE), "NONFINITE flag 32 px chain %d", c);
      }
      CHECK(rhmc_leapfrog(ctx, &P, q.data(), p.data(), 9, 1025, 1, nullptr, nullptr) ==
                RHMC_ERR_ARG, "K = 1025 rejected");
      rhmc_params bad = P;
      bad.reserved = 1;
      CHECK(rhmc_leapfrog(ctx, &bad, q.data(), p.data(), 9, 2, 1, nullptr, nullptr) ==
                RHMC_ERR_ARG, "reserved != 0 rejected");
    }
    CHECK(rhmc_ctx_synchronize(ctx) == RHMC_OK, "synchronize");
    rhmc_ctx_destroy(ctx);
  }
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  cpu_checks();
  if (gpu) gpu_checks();
  std::printf("capi_asan %s: %s (%d failed checks)\n", gpu ? "gpu" : "cpu",
              g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
