// mfma_bench.hip — fp64 matrix-core cost on gfx950 and whether it overlaps
// VALU fp64 work of another wave on the same SIMD (tools only, not shipped;
// the question behind DESIGN §9's MFMA direction for the many-star pixel
// passes).  One workgroup of 4 or 8 waves per CU: wave w runs on SIMD w % 4.
//   mfma : every wave issues 4 independent v_mfma_f64_16x16x4_f64 chains
//   valu : every wave issues 8 independent fp64 FMA streams
//   mixed: waves 0-3 the MFMA loop, waves 4-7 the VALU loop (one of each per SIMD)
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_bench tools/mfma_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma_loop(double* out, int iters) {
  const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999999;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  const d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
}

__device__ __forceinline__ void valu_loop(double* out, int iters) {
  double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
         a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const double m = 0.9999999, c = 1e-7;
  for (int i = 0; i < iters; ++i) {
    a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
    a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// MODE 0: all waves MFMA; 1: all waves VALU; 2: waves 0-3 MFMA, 4-7 VALU
template <int MODE>
__global__ void bench(double* out, int mi, int vi) {
  const int w = threadIdx.x / 64;
  if (MODE == 0 || (MODE == 2 && w < 4)) mfma_loop(out, mi);
  else valu_loop(out, vi);
}

template <int MODE>
static float run(int blocks, int threads, double* out, int mi, int vi) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  bench<MODE><<<blocks, threads>>>(out, 8, 8);
  hipEventRecord(a);
  bench<MODE><<<blocks, threads>>>(out, mi, vi);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const double ghz = 2.4;
  double* out;
  hipMalloc(&out, (size_t)cus * 512 * 8);
  const int mi = 20000, vi = 40000;
  for (int wps : {1, 2}) {
    const int th = 256 * wps;
    const float tm = run<0>(cus, th, out, mi, vi);
    const float tv = run<1>(cus, th, out, mi, vi);
    printf("waves/SIMD %d  mfma 16x16x4 f64 x4 chains: %7.3f ms  %6.2f cycles/MFMA per SIMD\n", wps,
           tm, tm * 1e-3 * ghz * 1e9 / (wps * mi * 4.0));
    printf("waves/SIMD %d  fp64 fma x8 streams:        %7.3f ms  %6.2f cycles/wave-FMA per SIMD\n",
           wps, tv, tv * 1e-3 * ghz * 1e9 / (wps * vi * 8.0));
  }
  const float t0 = run<0>(cus, 256, out, mi, vi);
  const float t1 = run<1>(cus, 256, out, mi, vi);
  const float t2 = run<2>(cus, 512, out, mi, vi);
  printf("one MFMA wave + one VALU wave per SIMD: %7.3f ms (MFMA alone %7.3f, VALU alone %7.3f;"
         " overlap if ~max, serial if ~sum)\n", t2, t0, t1);
  return 0;
}
