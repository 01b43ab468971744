// ISA lab (development only): semantics and issue cost of single instructions on gfx950.
//   1. v_dot2_f32_bf16 via __builtin_amdgcn_fdot2_f32_bf16 against a host computation
//   2. issue cycles per instruction for a stream of independent v_exp_f32 / v_exp_f16 /
//      v_dot2_f32_bf16 / v_add_f32 / v_pk_add_f32 (one wave per SIMD and four, s_memtime)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void dot2_test(const uint32_t* a, const uint32_t* b, const float* c, float* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n)
    out[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a[i]), __builtin_bit_cast(bf16x2_t, b[i]), c[i], false);
}

template <int OP>
__global__ void issue_bench(float* out, long long* cyc, float seed) {
  float x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = seed * (threadIdx.x + i) * 1e-3f;
  uint32_t u[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) u[i] = __float_as_uint(x[i]);
  typedef float f32x16 __attribute__((ext_vector_type(16)));
  typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
  f32x16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  bf8 ma, mb;
#pragma unroll
  for (int r = 0; r < 8; ++r) { ma[r] = (__bf16)(seed * r); mb[r] = (__bf16)(seed * (r + threadIdx.x)); }
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 256; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (OP == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
      if constexpr (OP == 1) asm volatile("v_exp_f16 %0, %0" : "+v"(u[i]));
      if constexpr (OP == 2) asm volatile("v_dot2_f32_bf16 %0, %1, %1, %0" : "+v"(x[i]) : "v"(u[i]));
      if constexpr (OP == 3) asm volatile("v_add_f32 %0, %0, %0" : "+v"(x[i]));
      if constexpr (OP == 4) asm volatile("v_max3_f32 %0, %0, %1, %0" : "+v"(x[i]) : "v"(x[(i + 1) & 15]));
      if constexpr (OP == 5) asm volatile("v_cvt_pk_bf16_f32 %0, %1, %1" : "=v"(u[i]) : "v"(x[i]));
      if constexpr (OP == 6) asm volatile("v_exp_f16_e64 %0, %0 clamp" : "+v"(u[i]));
      if constexpr (OP == 10) { asm volatile("v_exp_f32 %0, %0" : "+v"(x[i])); asm volatile("v_add_f32 %0, %0, %0" : "+v"(u[i])); }
      if constexpr (OP == 11) { asm volatile("v_exp_f32 %0, %0" : "+v"(x[i])); asm volatile("v_cvt_pk_bf16_f32 %0, %1, %1" : "=v"(u[i]) : "v"(x[(i + 3) & 15])); }
      if constexpr (OP == 12 || OP == 13 || OP == 14 || OP == 15) {
        if ((i & 3) == 0) acc[i >> 2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ma, mb, acc[i >> 2], 0, 0, 0);
        if constexpr (OP == 12) asm volatile("v_exp_f32 %0, %0" : "+v"(x[i]));
        if constexpr (OP == 13) asm volatile("v_add_f32 %0, %0, %0" : "+v"(x[i]));
        if constexpr (OP == 15) { asm volatile("v_exp_f32 %0, %0" : "+v"(x[i])); asm volatile("v_exp_f32 %0, %0" : "+v"(u[i])); }
      }
      if constexpr (OP == 7) asm volatile("v_exp_f16_sdwa %0, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1" : "+v"(u[i]));
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i] + __uint_as_float(u[i]);
#pragma unroll
  for (int j = 0; j < 4; ++j) s += acc[j][threadIdx.x & 15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) {
    cyc[2 * (blockIdx.x * 32 + threadIdx.x / 64)] = t0;
    cyc[2 * (blockIdx.x * 32 + threadIdx.x / 64) + 1] = t1;
  }
}

static uint16_t bf(float f) { uint32_t u; std::memcpy(&u, &f, 4); return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16); }
static float fb(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; std::memcpy(&f, &u, 4); return f; }

template <int OP> void run(const char* name, float* dout, long long* dcyc, int waves_per_simd) {
  // one workgroup of 64 * 4 * waves_per_simd threads per CU: waves spread over the 4 SIMDs
  const int threads = 256 * waves_per_simd, blocks = 256;
  hipLaunchKernelGGL(issue_bench<OP>, dim3(blocks), dim3(threads), 0, 0, dout, dcyc, 1.0f);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(issue_bench<OP>, dim3(blocks), dim3(threads), 0, 0, dout, dcyc, 1.0f);
  hipDeviceSynchronize();
  std::vector<long long> c(blocks * 64);
  hipMemcpy(c.data(), dcyc, blocks * 64 * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  const int nw = threads / 64;
  for (int b = 0; b < blocks; ++b) {
    long long lo = c[2 * b * 32], hi = c[2 * b * 32 + 1];
    for (int w = 1; w < nw; ++w) { lo = std::min(lo, c[2 * (b * 32 + w)]); hi = std::max(hi, c[2 * (b * 32 + w) + 1]); }
    avg += hi - lo;
  }
  avg /= blocks;
  // s_memtime ticks at the shader clock; per instruction per wave
  std::printf("%-14s waves/SIMD=%d  %.2f cycles per instruction per wave, %.2f per SIMD\n", name, waves_per_simd,
              avg / (256.0 * 16), avg / (256.0 * 16) / waves_per_simd);
}

int main() {
  const int n = 1024;
  std::vector<uint32_t> a(n), b(n);
  std::vector<float> c(n), out(n);
  for (int i = 0; i < n; ++i) {
    float a0 = (i % 17) * 0.37f - 2, a1 = (i % 13) * 0.21f + 1, b0 = 1.f, b1 = (i % 5) * 0.5f;
    a[i] = bf(a0) | ((uint32_t)bf(a1) << 16);
    b[i] = bf(b0) | ((uint32_t)bf(b1) << 16);
    c[i] = i * 0.01f;
  }
  uint32_t *da, *db; float *dc, *dout; long long* dcyc;
  hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dout, 1 << 22); hipMalloc(&dcyc, 256 * 64 * 8);
  hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dc, c.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(dot2_test, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
  hipMemcpy(out.data(), dout, n * 4, hipMemcpyDeviceToHost);
  double maxerr = 0;
  for (int i = 0; i < n; ++i) {
    float ref = fb(a[i] & 0xFFFF) * fb(b[i] & 0xFFFF) + fb(a[i] >> 16) * fb(b[i] >> 16) + c[i];
    double e = std::abs(out[i] - ref);
    if (e > maxerr) maxerr = e;
    if (i < 4) std::printf("dot2[%d] = %g ref %g\n", i, out[i], ref);
  }
  std::printf("dot2 max err %g\n", maxerr);
  for (int w : {1, 2, 4}) {
    run<10>("exp+add", dout, dcyc, w);
    run<11>("exp+cvt", dout, dcyc, w);
    run<14>("mfma x4", dout, dcyc, w);
    run<12>("mfma4+exp16", dout, dcyc, w);
    run<15>("mfma4+exp32", dout, dcyc, w);
    run<13>("mfma4+add16", dout, dcyc, w);
  }
  for (int w : {1, 2, 4}) {
    run<0>("v_exp_f32", dout, dcyc, w);
    run<1>("v_exp_f16", dout, dcyc, w);
    run<6>("v_exp_f16 e64", dout, dcyc, w);
    run<7>("v_exp_f16 sdwa", dout, dcyc, w);
    run<2>("v_dot2_f32_bf16", dout, dcyc, w);
    run<3>("v_add_f32", dout, dcyc, w);
    run<4>("v_max3_f32", dout, dcyc, w);
    run<5>("v_cvt_pk_bf16", dout, dcyc, w);
  }
  return 0;
}
