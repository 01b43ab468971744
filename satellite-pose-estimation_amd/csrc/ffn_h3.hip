// fp32h3 encoder FFN in one pass: y = LayerNorm(x + ReLU(x W1^T + b1) W2^T + b2) (REV/models/
// transformer.py:164-167, the forward_post branch), fp32 in / out, every product on the scaled
// two-way fp16 split of gemm.hip's fp32h3 kernels (three v_mfma_f32_32x32x16_f16 per product).
//
// The unfused pair wrote the 2048-wide hidden activation in fp32 (1.4 GB per encoder layer at
// B = 64) and read it back; here a workgroup owns 128 rows (4 waves x 32 tokens) for the whole
// hidden dimension:
//   * x: each wave keeps its 32 rows' split fp16 planes in registers as the phase-1 MFMA B operand
//     (lane: token l & 31, K elements 16 kb + 8 (l >> 5) + 0..7), scale from the LayerNorm bound;
//   * per hidden chunk of 32: phase 1 H^T = W1_c x^T (A operand: W1's hi / lo planes, the h3
//     finalize form), then h = ReLU(H^T 2^-e / s_x + b1) is scaled by the static hidden bound's
//     power of two s_h and split in registers; its lane holds hidden rows 8 (r >> 2) + 4 (l >> 5) +
//     (r & 3), so W2's columns are stored in that order within each chunk (spe_ffn_h3_perm) and
//     the split h is directly the phase-2 B operand; phase 2 out^T += W2_c h^T;
//   * W1 / W2 chunks (2 x 32 KB hi + lo planes, XOR-swizzled rows) and the chunk's (2^-e, b1) pairs
//     stream through two LDS slots by buffer_load ... lds, one chunk ahead;
//   * epilogue: out = acc 2^-e2 / s_h + b2 + x, LayerNorm over the 256 columns of a token (lane l
//     and l + 32 hold its two halves), 16-byte stores in place over x.
// s_h: |h_j| <= |b1_j| + ||W1_j||_2 ||x||_2 and ||x||_2 <= max|gamma1| sqrt(256) + ||beta1||_2 for a
// LayerNorm output, so the bound never under-estimates; an over-estimate by 2^k only moves the
// split's absolute error floor to (bound) 2^-38 2^k.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int FH_BM = 128, FH_NT = 256, FH_HC = 32, FH_D = 256;
constexpr int FH_W1 = 2 * FH_HC * FH_D * 2;     // 32 KB: [plane][32 rows][512 B]
constexpr int FH_W2 = 2 * FH_D * FH_HC * 2;     // 32 KB: [plane][256 rows][64 B]
constexpr int FH_META = 2 * FH_HC * 4;          // 2^-e1[32], b1[32]
constexpr int FH_S1 = FH_W1 + FH_META;          // W1 ring slot: the chunk's planes + (2^-e1, b1)
constexpr int FH_R2 = 2 * FH_S1;                // W2 ring: 2 slots of FH_W2 from here
constexpr int FH_EPI = 4 * FH_D * 4;            // 2^-e2, b2, gamma2, beta2
constexpr int FH_EP = FH_R2 + 2 * FH_W2;
constexpr int FH_SMEM = FH_EP + FH_EPI;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

SPE_DEV u32x4 h_pack(const float* v) {
  return u32x4{pack_f16x2(v[0], v[1]), pack_f16x2(v[2], v[3]), pack_f16x2(v[4], v[5]), pack_f16x2(v[6], v[7])};
}
// 8 floats (already scaled) -> fp16 hi plane, lo plane (the remainder of the RNE hi, exact in fp32)
SPE_DEV void h_split8(const float* f, u32x4& h, u32x4& l) {
  h = h_pack(f);
  const f16x8 hv = __builtin_bit_cast(f16x8, h);
  float r[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = f[e] - (float)hv[e];
  l = h_pack(r);
}

__global__ __launch_bounds__(FH_NT, 1) void ffn_h3_kernel(FfnH3Args a) {
  __shared__ __attribute__((aligned(1024))) char smem[FH_SMEM];
  const int tid = threadIdx.x, lane = tid & 63, l31 = lane & 31, hi = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * FH_BM;
  const int nch = a.F / FH_HC;
  float sx = 1.f, inv_sx = 1.f;
  if (a.amax_x) {
    const float am = *a.amax_x;
    if (am > 0.f && am <= 3.0e38f) {
      const int e = __builtin_amdgcn_frexp_expf(am);
      sx = __builtin_ldexpf(1.f, 13 - e);
      inv_sx = __builtin_ldexpf(1.f, e - 13);
    }
  }
  const float sh = a.sh, inv_sh = 1.f / a.sh;          // powers of two: exact

  // ---- epilogue parameters to LDS (published by the first barrier)
  {
    float* ep = reinterpret_cast<float*>(smem + FH_EP);
    ep[tid] = a.sinv2[tid];
    ep[FH_D + tid] = a.b2[tid];
    ep[2 * FH_D + tid] = a.gamma[tid];
    ep[3 * FH_D + tid] = a.beta[tid];
  }

  // ---- chunk DMA: wave w issues pieces w + 4 i (0..31 W1, 32..63 W2) and wave 0 the meta piece
  const size_t p1 = (size_t)a.F * a.ld1 * 2, p2 = (size_t)FH_D * a.ld2 * 2;   // plane strides (bytes)
  const __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w1, (short)0, (int)(2 * p1), 0x00020000);
  const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc((void*)a.w2, (short)0, (int)(2 * p2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)a.meta1, (short)0, a.F * 8, 0x00020000);
  // W1 and W2 chunks in separate two-slot rings: iteration c multiplies chunk c + 1's phase 1 (W1 slot
  // (c + 1) & 1) beside chunk c's phase 2 (W2 slot c & 1) and refills W1 slot c & 1 with chunk c + 2
  // and W2 slot (c + 1) & 1 with chunk c + 1, one iteration ahead of their use
  auto issue_w1 = [&](int c, int slot) {
    char* base = smem + slot * FH_S1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {                      // piece k = w + 4i: plane k >> 4, rows 2 (k & 15) + hi
      const int k = wid + 4 * i, p = k >> 4, row = 2 * (k & 15) + hi, pos = l31;
      const int ch = pos ^ (row & 15);
      const int off = (int)(p * p1) + (c * FH_HC + row) * a.ld1 * 2 + ch * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r1, (lds_ptr_t)(base + k * 1024), 16, off, 0, 0, 0);
    }
    if (wid == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rm, (lds_ptr_t)(base + FH_W1), 4, (c * 64 + lane) * 4, 0, 0, 0);
  };
  auto issue_w2 = [&](int c, int slot) {
    char* base = smem + FH_R2 + slot * FH_W2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {                      // piece k: plane k >> 4, rows 16 (k & 15) + lane / 4
      const int k = wid + 4 * i, p = k >> 4, n = 16 * (k & 15) + (lane >> 2), pos = lane & 3;
      const int ch = pos ^ ((n >> 2) & 3);
      const int off = (int)(p * p2) + n * a.ld2 * 2 + c * FH_HC * 2 + ch * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r2, (lds_ptr_t)(base + k * 1024), 16, off, 0, 0, 0);
    }
  };
  issue_w1(0, 0);
  if (nch > 1) issue_w1(1, 1);
  issue_w2(0, 0);

  // ---- x rows of this wave: split planes in registers (B operand of phase 1)
  const int row = m0 + wid * 32 + l31;
  const bool rok = row < a.M;
  u32x4 xh[16], xl[16];
  {
    const float* xp = (const float*)a.x + (size_t)(rok ? row : 0) * a.ldx + 8 * hi;
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
      float f[8];
      const u32x4 v0 = rok ? ld16(xp + 16 * kb) : u32x4{0, 0, 0, 0};
      const u32x4 v1 = rok ? ld16(xp + 16 * kb + 4) : u32x4{0, 0, 0, 0};
      unpack16<float>(v0, f);
      unpack16<float>(v1, f + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sx;
      h_split8(f, xh[kb], xl[kb]);
    }
  }
  auto mf = [](u32x4 x, u32x4 y, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, x), __builtin_bit_cast(f16x8, y), c, 0, 0, 0);
  };
  f32x16 acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  // fragment offsets: W1 row l31, logical 16-byte chunk 2 kb + hi at (chunk ^ (row & 15));
  // W2 row 32 j + l31, chunk 2 kb + hi at (chunk ^ ((row >> 2) & 3))
  const int w1o = l31 * 512, w1x = l31 & 15;
  const int w2x = (l31 >> 2) & 3;
  // ---- phase 1 of a chunk: H^T[32 hidden][32 tokens] over K = 256 (16 K-blocks), W1 slot s1
  auto phase1 = [&](const char* s1, f32x16& hacc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[r] = 0.f;
    u32x4 fa[3][2];
    auto rd1 = [&](int kb, u32x4* f) {
      const int off = w1o + (((2 * kb + hi) ^ w1x) << 4);
      f[0] = ld16(s1 + off);                          // hi plane
      f[1] = ld16(s1 + FH_W1 / 2 + off);              // lo plane
    };
    rd1(0, fa[0]);
    rd1(1, fa[1]);
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
      if (kb + 2 < 16) rd1(kb + 2, fa[(kb + 2) % 3]);
      const u32x4* f = fa[kb % 3];
      hacc = mf(f[1], xh[kb], hacc);
      hacc = mf(f[0], xl[kb], hacc);
      hacc = mf(f[0], xh[kb], hacc);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // ---- h = ReLU(hacc 2^-e1 / s_x + b1) s_h, split: lane rows 8 (r >> 2) + 4 hi + (r & 3); in steps
  // (0..3: the four row groups, 4 / 5: the two K-block splits) so phase 2's MFMAs can carry them
  float hv[16];
  auto hconv = [&](const char* s1, const f32x16& hacc, int step, u32x4* hh, u32x4* hl) {
    if (step < 4) {
      const float* meta = reinterpret_cast<const float*>(s1 + FH_W1);
      const f32x4 si = *reinterpret_cast<const f32x4*>(meta + 8 * step + 4 * hi);
      const f32x4 bi = *reinterpret_cast<const f32x4*>(meta + FH_HC + 8 * step + 4 * hi);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        hv[4 * step + e] = fmaxf(hacc[4 * step + e] * (si[e] * inv_sx) + bi[e], 0.f) * sh;
    } else {
      h_split8(hv + 8 * (step - 4), hh[step - 4], hl[step - 4]);
    }
  };
  // ---- phase 2 of chunk c from W2 slot s2 with h (hh, hl), chunk c + 1's conversion interleaved
  auto phase2 = [&](const char* s2, const u32x4* hh, const u32x4* hl, bool conv, const char* s1n,
                    const f32x16& haccn, u32x4* hhn, u32x4* hln) {
    u32x4 fb[3][2];
    auto rd2 = [&](int t, u32x4* f) {                 // t = 2 j + kb
      const int j = t >> 1, kb = t & 1;
      const int off = (32 * j + l31) * 64 + (((2 * kb + hi) ^ w2x) << 4);
      f[0] = ld16(s2 + off);
      f[1] = ld16(s2 + FH_W2 / 2 + off);
    };
    rd2(0, fb[0]);
    rd2(1, fb[1]);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (t + 2 < 16) rd2(t + 2, fb[(t + 2) % 3]);
      const u32x4* f = fb[t % 3];
      const int j = t >> 1, kb = t & 1;
      acc[j] = mf(f[1], hh[kb], acc[j]);
      acc[j] = mf(f[0], hl[kb], acc[j]);
      acc[j] = mf(f[0], hh[kb], acc[j]);
      if (conv && t >= 4 && t < 10) hconv(s1n, haccn, t - 4, hhn, hln);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  __builtin_amdgcn_s_waitcnt(0);                      // W1 chunks 0, 1, W2 chunk 0, epilogue parameters
  __syncthreads();
  u32x4 hh[2], hl[2], hhn[2], hln[2];
  {
    f32x16 hacc;
    phase1(smem, hacc);
#pragma unroll
    for (int st = 0; st < 6; ++st) hconv(smem, hacc, st, hh, hl);
  }
  __syncthreads();                                     // W1 slot 0 read by every wave: free for chunk 2
  for (int c = 0; c < nch; ++c) {
    const bool more = c + 1 < nch;
    if (c + 2 < nch) issue_w1(c + 2, c & 1);
    if (more) issue_w2(c + 1, (c + 1) & 1);
    const char* s1n = smem + ((c + 1) & 1) * FH_S1;
    f32x16 haccn;
    if (more) phase1(s1n, haccn);
    else
#pragma unroll
      for (int r = 0; r < 16; ++r) haccn[r] = 0.f;
    phase2(smem + FH_R2 + (c & 1) * FH_W2, hh, hl, more, s1n, haccn, hhn, hln);
#pragma unroll
    for (int i = 0; i < 2; ++i) { hh[i] = hhn[i]; hl[i] = hln[i]; }
    __builtin_amdgcn_s_waitcnt(0);                    // this wave's pieces of W1 c + 2, W2 c + 1
    __syncthreads();                                   // ... everyone's; the slots read this iteration free
  }

  // ---- epilogue: v = acc 2^-e2 / s_h + b2 + x, LayerNorm over the token's 256 columns
  // (lane: token l31, columns 32 j + 8 q + 4 hi + 0..3)
  const float* ep = reinterpret_cast<const float*>(smem + FH_EP);
  const float* xr = (const float*)a.x + (size_t)(rok ? row : 0) * a.ldx;
  float sum = 0.f;
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {                    // two halves of the residual loads in flight
    f32x4 rv[4][4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        rv[jj][q] = rok ? __builtin_bit_cast(f32x4, ld16(xr + 32 * (4 * hf + jj) + 8 * q + 4 * hi)) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * hf + jj;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = 32 * j + 8 * q + 4 * hi;
        const f32x4 s2 = *reinterpret_cast<const f32x4*>(ep + n);
        const f32x4 b2 = *reinterpret_cast<const f32x4*>(ep + FH_D + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = acc[j][4 * q + e] * (s2[e] * inv_sh) + b2[e] + rv[jj][q][e];
          acc[j][4 * q + e] = v;
          sum += v;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  const float mean = (sum + __shfl_xor(sum, 32, 64)) * (1.f / FH_D);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float dv = acc[j][r] - mean;
      ss += dv * dv;
    }
  const float rs = rsqrtf((ss + __shfl_xor(ss, 32, 64)) * (1.f / FH_D) + 1e-5f);
  float* yr = (float*)a.y + (size_t)(rok ? row : 0) * a.ldy;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 32 * j + 8 * q + 4 * hi;
      const f32x4 ga = *reinterpret_cast<const f32x4*>(ep + 2 * FH_D + n);
      const f32x4 be = *reinterpret_cast<const f32x4*>(ep + 3 * FH_D + n);
      float y[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = (acc[j][4 * q + e] - mean) * rs * ga[e] + be[e];
      if (rok) st16(yr + n, pack16<float>(y));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

}  // namespace

// position p (0..31) of a 32-wide hidden chunk in W2's column order -> the hidden unit it holds:
// the phase-1 accumulator lane (token, half h) holds units 8 (r >> 2) + 4 h + (r & 3), r = 0..15,
// and supplies K-block kb's elements 8 h + 0..7 from its r = 8 kb .. 8 kb + 7
int spe_ffn_h3_perm(int p) {
  const int kb = p >> 4, h = (p >> 3) & 1, r = 8 * kb + (p & 7);
  return 8 * (r >> 2) + 4 * h + (r & 3);
}

int spe_launch_ffn_h3(const FfnH3Args& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (a.D != FH_D || a.F % FH_HC || !a.x || !a.y || !a.w1 || !a.w2 || !a.meta1 || !a.sinv2 || !a.b2 || !a.gamma ||
      !a.beta || !(a.sh > 0.f) || (a.ldx & 3) || (a.ldy & 3) || (a.ld1 & 7) || (a.ld2 & 7) || a.ld1 < FH_D ||
      a.ld2 < a.F || (reinterpret_cast<uintptr_t>(a.x) & 15) || (reinterpret_cast<uintptr_t>(a.y) & 15))
    return -1;
  constexpr long long LIM = (1LL << 31) - (1LL << 24);
  if (2LL * a.F * a.ld1 * 2 >= LIM || 2LL * FH_D * a.ld2 * 2 >= LIM) return -1;
  hipLaunchKernelGGL(ffn_h3_kernel, dim3((a.M + FH_BM - 1) / FH_BM), dim3(FH_NT), 0, s, a);
  return (int)hipGetLastError();
}
