// Issue-rate microbenchmark (lab tool, not product): v_exp_f32 vs v_exp_f16 vs v_pk_max_f16 vs
// v_max3_f32 in a dependent-free unrolled loop, one wave per SIMD, timed with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  float x[16];
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 1e-3f + i * 1e-2f;
  unsigned h[16];
  for (int i = 0; i < 16; ++i) h[i] = __float_as_uint(x[i]);
  long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (OP == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
      else if constexpr (OP == 1) asm volatile("v_exp_f16 %0, %0" : "+v"(h[i]));
      else if constexpr (OP == 2) asm volatile("v_pk_max_f16 %0, %0, %0" : "+v"(h[i]));
      else if constexpr (OP == 3) asm volatile("v_max3_f32 %0, %0, %0, %0" : "+v"(x[i]));
      else if constexpr (OP == 4) asm volatile("v_cvt_pkrtz_f16_f32 %0, %0, %0" : "+v"(h[i]));
      else if constexpr (OP == 5) asm volatile("v_pk_fma_f16 %0, %0, %0, %0" : "+v"(h[i]));
      else if constexpr (OP == 6) asm volatile("v_fma_f32 %0, %0, %0, %0" : "+v"(x[i]));
    }
  }
  long t1 = __builtin_readcyclecounter();
  float s = 0;
  for (int i = 0; i < 16; ++i) s += x[i] + __uint_as_float(h[i]);
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(t1 - t0) / (iters * 16.0f);
  if (s == 12345.f) out[1] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * 4);
  const char* names[] = {"v_exp_f32", "v_exp_f16", "v_pk_max_f16", "v_max3_f32", "v_cvt_pkrtz_f16_f32", "v_pk_fma_f16", "v_fma_f32"};
  for (int wps = 1; wps <= 2; ++wps) {
    for (int op = 0; op < 7; ++op) {
      auto launch = [&](int iters) {
        switch (op) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 5: hipLaunchKernelGGL(k<5>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
          case 6: hipLaunchKernelGGL(k<6>, dim3(256), dim3(64 * 4 * wps), 0, 0, d, iters); break;
        }
      };
      launch(100);
      hipDeviceSynchronize();
      launch(2000);
      float h;
      hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
      printf("waves/SIMD %d  %-22s %.2f cycles per wave-instruction (s_memtime ticks)\n", wps, names[op], h);
    }
  }
  return 0;
}
