// isa_bench.hip — fp64 VALU issue costs on gfx950 (tools only, not shipped).
// Prints SIMD-cycles per wave64 instruction for independent FMA streams,
// independent v_rcp_f64 streams, dependent FMA chains, and the accuracy of
// raw v_rcp_f64 / one Newton step against IEEE 1/x.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/isa_bench tools/isa_bench.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../hmc-stellar-toy-model_amd/csrc/rhmc_exp.hpp"

template <int MODE>
__global__ void thr(double* out, double seed, int iters) {
  double a0 = seed + threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
         a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const double m = 0.9999999, c = 1e-7;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {  // 8 independent fma streams
      a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
      a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
    } else if (MODE == 1) {  // 8 independent rcp streams
      a0 = __builtin_amdgcn_rcp(a0); a1 = __builtin_amdgcn_rcp(a1);
      a2 = __builtin_amdgcn_rcp(a2); a3 = __builtin_amdgcn_rcp(a3);
      a4 = __builtin_amdgcn_rcp(a4); a5 = __builtin_amdgcn_rcp(a5);
      a6 = __builtin_amdgcn_rcp(a6); a7 = __builtin_amdgcn_rcp(a7);
    } else if (MODE == 2) {  // one dependent fma chain (latency)
      a0 = fma(a0, m, c); a0 = fma(a0, m, c); a0 = fma(a0, m, c); a0 = fma(a0, m, c);
      a0 = fma(a0, m, c); a0 = fma(a0, m, c); a0 = fma(a0, m, c); a0 = fma(a0, m, c);
    } else if (MODE == 3) {  // two interleaved dependent chains
      a0 = fma(a0, m, c); a1 = fma(a1, m, c); a0 = fma(a0, m, c); a1 = fma(a1, m, c);
      a0 = fma(a0, m, c); a1 = fma(a1, m, c); a0 = fma(a0, m, c); a1 = fma(a1, m, c);
    } else if (MODE == 4) {  // 8 independent v_mul_f64
      a0 *= m; a1 *= m; a2 *= m; a3 *= m; a4 *= m; a5 *= m; a6 *= m; a7 *= m;
    } else if (MODE == 5) {  // rcp mixed 1:6 with fma (pixel-loop ratio)
      a0 = __builtin_amdgcn_rcp(a0); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
      a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
    } else if (MODE == 7) {  // rcp dependent chain (latency)
      a0 = __builtin_amdgcn_rcp(a0); a0 = __builtin_amdgcn_rcp(a0);
      a0 = __builtin_amdgcn_rcp(a0); a0 = __builtin_amdgcn_rcp(a0);
      a0 = __builtin_amdgcn_rcp(a0); a0 = __builtin_amdgcn_rcp(a0);
      a0 = __builtin_amdgcn_rcp(a0); a0 = __builtin_amdgcn_rcp(a0);
    } else if (MODE == 8) {  // 8 independent f32 -> f64 conversions
      a0 = (double)(float)a1; a1 = (double)(float)a2; a2 = (double)(float)a3;
      a3 = (double)(float)a4; a4 = (double)(float)a5; a5 = (double)(float)a6;
      a6 = (double)(float)a7; a7 = (double)(float)a0;
    } else if (MODE == 9) {  // dependent add chain through a DPP move (quad_perm)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const long long b = __double_as_longlong(a0);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)b, 0xB1, 0xF, 0xF, false);
        const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), 0xB1, 0xF, 0xF, false);
        a0 = a0 * m + __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
      }
    } else if (MODE == 10) {  // 8 independent 32-bit integer adds (v_add_u32)
      int i0 = __double_as_longlong(a0), i1 = i0 + 1, i2 = i0 + 2, i3 = i0 + 3, i4 = i0 + 4,
          i5 = i0 + 5, i6 = i0 + 6, i7 = i0 + 7;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        asm volatile("v_add_u32 %0, %0, 3\n v_add_u32 %1, %1, 3\n v_add_u32 %2, %2, 3\n"
                     " v_add_u32 %3, %3, 3\n v_add_u32 %4, %4, 3\n v_add_u32 %5, %5, 3\n"
                     " v_add_u32 %6, %6, 3\n v_add_u32 %7, %7, 3"
                     : "+v"(i0), "+v"(i1), "+v"(i2), "+v"(i3), "+v"(i4), "+v"(i5), "+v"(i6),
                       "+v"(i7));
      }
      a0 += (double)(i0 + i1 + i2 + i3 + i4 + i5 + i6 + i7) * 1e-30;
    } else if (MODE == 11) {  // 8 dependent 32-bit integer adds (one chain)
      int i0 = __double_as_longlong(a0);
#pragma unroll
      for (int k = 0; k < 4; ++k)
        asm volatile("v_add_u32 %0, %0, 3\n v_add_u32 %0, %0, 3\n v_add_u32 %0, %0, 3\n"
                     " v_add_u32 %0, %0, 3\n v_add_u32 %0, %0, 3\n v_add_u32 %0, %0, 3\n"
                     " v_add_u32 %0, %0, 3\n v_add_u32 %0, %0, 3"
                     : "+v"(i0));
      a0 += (double)i0 * 1e-30;
    } else if (MODE == 12) {  // dependent ds_bpermute chain (cross-lane through LDS)
      int i0 = (int)__double_as_longlong(a0);
#pragma unroll
      for (int k = 0; k < 8; ++k) i0 = __builtin_amdgcn_ds_bpermute(((threadIdx.x + 1) & 63) * 4, i0);
      a0 += (double)i0 * 1e-30;
    } else if (MODE == 6) {  // exp (ocml) x8 independent
      a0 = exp(-a0); a1 = exp(-a1); a2 = exp(-a2); a3 = exp(-a3);
      a4 = exp(-a4); a5 = exp(-a5); a6 = exp(-a6); a7 = exp(-a7);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__global__ void rcp_acc(const double* x, unsigned long long* stat, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  const double ref = 1.0 / d;
  const double r0 = __builtin_amdgcn_rcp(d);
  const double r1 = fma(r0, fma(-d, r0, 1.0), r0);
  auto ulp = [](double a, double b) {
    long long x = __double_as_longlong(a) - __double_as_longlong(b);
    return (unsigned long long)(x < 0 ? -x : x);
  };
  atomicMax(&stat[0], ulp(r0, ref));
  atomicMax(&stat[1], ulp(r1, ref));
  if (r1 != ref) atomicAdd(&stat[2], 1ull);
}

template <int MODE>
float run(int blocks, int iters) {
  double* out;
  hipMalloc(&out, (size_t)blocks * 64 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  thr<MODE><<<blocks, 64>>>(out, 1.5, 10);
  hipEventRecord(a);
  thr<MODE><<<blocks, 64>>>(out, 1.5, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipFree(out);
  return ms;
}

__global__ void exp_acc(unsigned long long* stat, int n, double lo) {
  __shared__ double tab[rhmc::kExpTab];
  rhmc::exp_tab_fill(tab);
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = lo * ((double)i / n) * (1.0 + 1e-9 * (i % 1013));
  const double a = rhmc::exp_neg(t, tab), b = exp(t);
  long long d = __double_as_longlong(a) - __double_as_longlong(b);
  d = d < 0 ? -d : d;
  atomicMax(&stat[0], (unsigned long long)d);
  if (d) atomicAdd(&stat[1], 1ull);
}

__global__ void exp_thr(double* out, double seed, int iters) {
  __shared__ double tab[rhmc::kExpTab];
  rhmc::exp_tab_fill(tab);
  __syncthreads();
  double a0 = -(seed + threadIdx.x * 1e-3), a1 = a0 - 1, a2 = a0 - 2, a3 = a0 - 3;
  for (int i = 0; i < iters; ++i) {
    a0 = -rhmc::exp_neg(a0, tab); a1 = -rhmc::exp_neg(a1, tab);
    a2 = -rhmc::exp_neg(a2, tab); a3 = -rhmc::exp_neg(a3, tab);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int simds = prop.multiProcessorCount * 4;
  const double ghz = 2.4;
  const char* names[] = {"fma x8 indep", "rcp x8 indep", "fma dep chain", "fma 2 chains",
                         "mul x8 indep", "rcp:fma 1:7", "exp x8 indep", "rcp dep chain",
                         "cvt f32->f64 x8", "dpp+fma dep x8", "u32 add x8 indep",
                         "u32 add dep x8", "bpermute dep x8"};
  const int iters = 20000;
  for (int wps : {1, 2, 4}) {
    const int blocks = simds * wps;
    float t[13];
    t[0] = run<0>(blocks, iters);
    t[1] = run<1>(blocks, iters);
    t[2] = run<2>(blocks, iters);
    t[3] = run<3>(blocks, iters);
    t[4] = run<4>(blocks, iters);
    t[5] = run<5>(blocks, iters);
    t[6] = run<6>(blocks, iters / 20);
    t[7] = run<7>(blocks, iters);
    t[8] = run<8>(blocks, iters);
    t[9] = run<9>(blocks, iters);
    t[10] = run<10>(blocks, iters);
    t[11] = run<11>(blocks, iters);
    t[12] = run<12>(blocks, iters);
    for (int m = 0; m < 13; ++m) {
      // wave-ops per SIMD (the u32 modes issue 32 adds per iteration)
      const double ops = (double)wps * iters / (m == 6 ? 20 : 1) * (m == 10 || m == 11 ? 32 : 8);
      printf("waves/SIMD %d  %-14s %8.3f ms  %6.2f cycles/wave-op @%.1fGHz\n", wps, names[m],
             t[m], t[m] * 1e-3 * ghz * 1e9 / ops, ghz);
    }
  }
  const int n = 1 << 24;
  std::vector<double> hx(n);
  for (int i = 0; i < n; ++i) hx[i] = 24.98 * std::pow(2.0, 14.0 * (double)i / n) * (1 + 1e-7 * (i % 977));
  double* dx;
  unsigned long long* st;
  hipMalloc(&dx, n * 8);
  hipMalloc(&st, 24);
  hipMemset(st, 0, 24);
  hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice);
  rcp_acc<<<n / 256, 256>>>(dx, st, n);
  unsigned long long hs[3];
  hipMemcpy(hs, st, 24, hipMemcpyDeviceToHost);
  printf("v_rcp_f64: max %llu ulp; + 1 Newton: max %llu ulp, %llu / %d differ from IEEE\n",
         hs[0], hs[1], hs[2], n);
  {
    unsigned long long* es;
    hipMalloc(&es, 16);
    for (double lo : {-30.0, -745.0, -1500.0}) {
      hipMemset(es, 0, 16);
      exp_acc<<<n / 256, 256>>>(es, n, lo);
      unsigned long long he[2];
      hipMemcpy(he, es, 16, hipMemcpyDeviceToHost);
      printf("exp_neg vs exp on [%g, 0]: max %llu ulp, %llu / %d differ\n", lo, he[0], he[1], n);
    }
    double* out;
    hipMalloc(&out, (size_t)simds * 4 * 64 * 8);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    exp_thr<<<simds * 4, 64>>>(out, 1.5, 10);
    hipEventRecord(a);
    exp_thr<<<simds * 4, 64>>>(out, 1.5, 1000);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("waves/SIMD 4  exp_neg x4 dep   %8.3f ms  %6.2f cycles/wave-op @2.4GHz\n", ms,
           ms * 1e-3 * 2.4e9 / (4.0 * 1000 * 4));
  }
  return 0;
}
