// Encoder self-attention output projection + residual + post-norm LayerNorm (bf16 models):
//
//     src = LayerNorm(src + attn . Wo^T + bo)            (REV/models/transformer.py:161-162, norm1)
//
// HBM-bound (K = N = 256: 512 multiply-adds per 1.5 KB moved per row).  The streaming GEMM's
// LayerNorm variant (gemm_stream.hip) runs one 4-wave workgroup per CU (the 128 KB W slice fills
// LDS) and spills; here 8 waves share the LDS-resident Wo, two per SIMD, each streaming 16-row
// tiles with the next tile's A and residual in flight, and the row's 256 columns live in the
// four lanes fg of one wave (the C^T form MFMA(Wo, A)), so the LayerNorm is two shuffle steps.
// In place (C == R) is safe: a wave writes only the rows it has already read.
#include "spe_common.h"
#include "spe_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int D = 256, NT = 512, NW = 8, KB = D * 2, KF = D / 32, JF = D / 16;

__global__ __launch_bounds__(NT, 1) void lnproj_kernel(GemmArgs g, int row_tiles) {
  __shared__ __attribute__((aligned(1024))) char wl[D * KB];
  __shared__ __attribute__((aligned(16))) float sb[D], sg[D], sbt[D];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fg = lane >> 4, fr = lane & 15;
  {
    // W -> LDS: row n, 16-byte chunk c at n*KB + (c ^ (n & wkey_mask(KB)))*16 (swizzle on the source)
    constexpr int INS = D * KB / 1024;
    for (int q = wid; q < INS; q += NW) {
      const int o = q * 1024 + lane * 16;
      const int n = o / KB, within = o - n * KB;
      const int chunk = (within >> 4) ^ (n & wkey_mask(KB));
      __builtin_amdgcn_global_load_lds((const void*)((const char*)g.B + (size_t)n * g.ldb * 2 + chunk * 16),
                                       (lds_ptr_t)(wl + q * 1024), 16, 0, 0);
    }
    for (int i = tid; i < D; i += NT) {
      sb[i] = g.bias ? g.bias[i] : 0.f;
      sg[i] = g.ln_g[i];
      sbt[i] = g.ln_b[i];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  auto w_addr = [](int n, int chunk) { return wkey_addr(n, chunk, KB); };

  auto load = [&](int t, u32x4 (&x)[KF], u32x2 (&r)[JF]) {
    t = t < row_tiles ? t : row_tiles - 1;
    int m = t * 16 + fr;
    m = m < g.M ? m : g.M - 1;
    const char* pa = (const char*)g.A + (size_t)m * g.lda * 2 + fg * 16;
#pragma unroll
    for (int kf = 0; kf < KF; ++kf) x[kf] = ld16(pa + kf * 64);
    const char* pr = (const char*)g.R + ((size_t)m * g.ldr + 4 * fg) * 2;
#pragma unroll
    for (int j = 0; j < JF; ++j) r[j] = ld8(pr + j * 32);
  };

  // W fragment bases: row 16j+fr, chunk 4kf+fg lives at wb[kf&3][j>>3] + (j&7)*8192 + (kf>>2)*256 (the
  // key n & 15 = fr touches the chunk's low 4 bits only; the rest are immediates); the bases are
  // opaque to the compiler so it cannot re-derive one address register per (j, kf).
  int wb[4][2];
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      wb[p][h] = w_addr(fr + 128 * h, 4 * p + fg);
      asm volatile("" : "+v"(wb[p][h]));
    }
  auto tile = [&](int t, const u32x4 (&x)[KF], const u32x2 (&r)[JF]) {
    asm volatile("" ::: "memory");              // (W fragments: loop-invariant LDS reads, not hoisted)
    // accumulators start at the bias (no bias adds in the epilogue)
    f32x4 acc[JF];
#pragma unroll
    for (int j = 0; j < JF; ++j) acc[j] = *reinterpret_cast<const f32x4*>(sb + 16 * j + 4 * fg);
#pragma unroll
    for (int kf = 0; kf < KF; ++kf) {
      const bf16x8 av = __builtin_bit_cast(bf16x8, x[kf]);
#pragma unroll
      for (int j = 0; j < JF; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            __builtin_bit_cast(bf16x8, ld16(wl + wb[kf & 3][j >> 3] + (j & 7) * 8192 + (kf >> 2) * 256)), av, acc[j], 0, 0, 0);
    }
    // lane: row m = fr, columns 16j + 4fg + e
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < JF; ++j) {
      acc[j][0] += __uint_as_float(r[j].x << 16);
      acc[j][1] += __uint_as_float(r[j].x & 0xffff0000u);
      acc[j][2] += __uint_as_float(r[j].y << 16);
      acc[j][3] += __uint_as_float(r[j].y & 0xffff0000u);
      s += (acc[j][0] + acc[j][1]) + (acc[j][2] + acc[j][3]);
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < JF; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) q += (acc[j][e] - mean) * (acc[j][e] - mean);
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.f / D) + 1e-5f);
    const int m = t * 16 + fr;
    if (m < g.M) {
      char* cp = (char*)g.C + ((size_t)m * g.ldc + 4 * fg) * 2;
#pragma unroll
      for (int j = 0; j < JF; ++j) {
        const f32x4 gm = *reinterpret_cast<const f32x4*>(sg + 16 * j + 4 * fg);
        const f32x4 bt = *reinterpret_cast<const f32x4*>(sbt + 16 * j + 4 * fg);
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (acc[j][e] - mean) * rs * gm[e] + bt[e];
        st8(cp + j * 32, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
      }
    }
  };

  const int G = gridDim.x, stride = G * NW;
  const int t0 = xcd_remap(blockIdx.x, G) * NW + wid;
  if (t0 >= row_tiles) return;
  // two operand sets in rotation, unrolled by two (register arrays never indexed at run time)
  u32x4 a0[KF], a1[KF];
  u32x2 r0[JF], r1[JF];
  load(t0, a0, r0);
  for (int t = t0;;) {
    load(t + stride, a1, r1);
    tile(t, a0, r0);
    t += stride;
    if (t >= row_tiles) break;
    load(t + stride, a0, r0);
    tile(t, a1, r1);
    t += stride;
    if (t >= row_tiles) break;
  }
}

}  // namespace

// bf16, K = N = 256, residual + LayerNorm, no activation (SPE_LNPROJ=0 disables it)
bool spe_lnproj_applies(const GemmArgs& g) {
  static const int on = [] { const char* e = getenv("SPE_LNPROJ"); return e ? atoi(e) : 1; }();
  return on && g.M > 0 && g.K == D && g.N == D && g.ln_g && g.ln_b && g.R && !g.act && !g.res_post && !g.out_f32 &&
         !g.out_f16 && g.vt_T == 0 && g.r_period == 0 && !g.P && g.lda % 8 == 0 && g.ldb >= D && g.ldc % 4 == 0 &&
         g.ldr % 4 == 0;
}

// 1 = not a problem for this kernel
int spe_launch_lnproj(const GemmArgs& g, hipStream_t s) {
  if (!spe_lnproj_applies(g)) return 1;
  const int row_tiles = (g.M + 15) / 16;
  // one workgroup per CU, but no more than the tiles need (each workgroup stages all of W first:
  // the decoder's 704-row launches take 6 workgroups, not 256 that would load W and exit)
  const int grid = std::min(spe_cu_count(), (row_tiles + NW - 1) / NW);
  hipLaunchKernelGGL(lnproj_kernel, dim3(grid), dim3(NT), 0, s, g, row_tiles);
  spe_gemm_last_path = 4;
  return (int)hipGetLastError();
}
