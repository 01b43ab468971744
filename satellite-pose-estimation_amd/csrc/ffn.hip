// Fused transformer FFN block for gfx950 (bf16 storage, fp32 accumulate):
//
//     y = LayerNorm( x + W2 . relu(W1 . x + b1) + b2 )          (post-norm, eps 1e-5)
//
// i.e. linear1 -> ReLU -> linear2 -> residual -> norm2 of TransformerEncoderLayer.forward_post
// (REV/models/transformer.py:164-167) and norm3 of the decoder layer (:235-238).  The
// [rows x 2048] hidden activation never leaves registers: per 128-row block each wave owns 32
// rows and keeps its x rows (as MFMA B fragments) and its 256 output columns (as transposed
// accumulators out^T[n][m]) in registers while the block streams W1/W2 in chunks of 32 hidden
// units through LDS:
//     H^T[j][m] = W1[j][:] . x[m][:]                 16x16x32 MFMAs, K = 256
//     out^T[n][m] += W2[n][j] . relu(H^T + b1)[j][m]   16x16x32 MFMAs, K = 32; the H^T accumulator
//                                                    is re-packed in registers as the B operand
//                                                    (k order permuted; W2 reads follow it)
// The epilogue adds b2 and the residual, does the row LayerNorm with two lane shuffles
// (each row's 256 columns live in 4 lanes) and stores bf16 in place over x.
// Versus two GEMM launches + a LayerNorm launch this removes the 2 x rows x 2048 x 2 B round
// trip of the hidden activation through HBM and two kernel boundaries per layer.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int NT = 256;
constexpr int BM = 128;                 // rows per block (32 per wave)
constexpr int HC = 32;                  // hidden units per chunk
constexpr int D = 256;
constexpr int W1_BYTES = HC * D * 2;    // 16 KiB: W1[j][d], 32 rows of 512 B
constexpr int W2_BYTES = D * HC * 2;    // 16 KiB: W2[n][j], 256 rows of 64 B
constexpr int STAGE = W1_BYTES + W2_BYTES;
constexpr int FMAX = 4096;              // largest dim_feedforward (b1 staged in LDS)

// W1 chunk: 16-byte chunk c (of 32 per row) lives at slot c ^ (row & 15)
SPE_DEV int w1_off(int row, int c) { return row * 512 + ((c ^ (row & 15)) << 4); }
// W2 chunk: 8-byte unit u (of 8 per row) lives at slot u ^ ((row >> 1) & 7): the 16 rows one
// ds_read_b64 / ds_read2_b64 lane group touches land on 16 distinct 8-byte bank pairs
SPE_DEV int w2_key(int row) { return (row >> 1) & 7; }
SPE_DEV int w2_off(int row, int u) { return row * 64 + ((u ^ w2_key(row)) << 3); }

struct Staged {
  u32x4 w1[4], w2[4];
  SPE_DEV void load(const FfnArgs& a, int chunk, int tid) {
    const char* W1 = (const char*)a.w1 + (size_t)(chunk * HC) * a.ld1 * 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {               // 32 rows x 32 chunks
      const int idx = tid + i * NT, row = idx >> 5, c = idx & 31;
      w1[i] = ld16(W1 + ((size_t)row * a.ld1 + c * 8) * 2);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {               // 256 rows x 4 chunks of 16 B
      const int idx = tid + i * NT, row = idx >> 2, c = idx & 3;
      w2[i] = ld16((const char*)a.w2 + ((size_t)row * a.ld2 + chunk * HC + c * 8) * 2);
    }
  }
  SPE_DEV void store(char* st, int tid) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NT, row = idx >> 5, c = idx & 31;
      st16(st + w1_off(row, c), w1[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int idx = tid + i * NT, row = idx >> 2, c = idx & 3;
      // units 2c, 2c+1 land in one aligned slot pair, swapped when the row key is odd
      const bool swap = w2_key(row) & 1;
      const u32x4 v = swap ? u32x4{w2[i].z, w2[i].w, w2[i].x, w2[i].y} : w2[i];
      st16(st + W1_BYTES + (w2_off(row, 2 * c) & ~15), v);
    }
  }
};

__global__ __launch_bounds__(NT, 1) void ffn_ln_kernel(FfnArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  __shared__ __attribute__((aligned(16))) float sb1[FMAX];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // b1 lives in LDS: a global load inside the chunk loop would make the wave wait (vmcnt is
  // in-order) for the next chunk's weight prefetch issued just before it.
  for (int i = tid; i < a.F; i += NT) sb1[i] = a.b1[i];
  const int g = lane >> 4, c16 = lane & 15;
  const int m0 = blockIdx.x * BM + wid * 32;

  // x rows of this wave as B fragments: xf[mb][ks] = x[m0 + 16mb + c16][32ks + 8g .. +7]
  bf16x8 xf[2][8];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int m = m0 + 16 * mb + c16;
    const bf16* xr = (const bf16*)a.x + (size_t)(m < a.M ? m : 0) * a.ldx;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
      xf[mb][ks] = __builtin_bit_cast(bf16x8, m < a.M ? ld16(xr + 32 * ks + 8 * g) : u32x4{0, 0, 0, 0});
  }
  f32x4 acc[16][2];
#pragma unroll
  for (int nb = 0; nb < 16; ++nb) { acc[nb][0] = f32x4{0, 0, 0, 0}; acc[nb][1] = f32x4{0, 0, 0, 0}; }

  const int nchunks = a.F / HC;
  Staged stg;
  stg.load(a, 0, tid);
  stg.store(smem, tid);
  __syncthreads();
  for (int ch = 0; ch < nchunks; ++ch) {
    const char* st = smem + (ch & 1) * STAGE;
    const bool more = ch + 1 < nchunks;
    if (more) stg.load(a, ch + 1, tid);
    // All of this chunk's LDS operand reads are issued up front (one wave per SIMD: nothing else
    // hides LDS latency); the phase-2 W2 reads land while the phase-1 MFMAs run.
    u32x4 wa[8][2];
    u32x2 wlo[16], whi[16];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks)
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) wa[ks][jb] = ld16(st + w1_off(16 * jb + c16, 4 * ks + g));
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const int row = 16 * nb + c16;
      wlo[nb] = ld8(st + W1_BYTES + w2_off(row, g));        // j = 4g .. 4g+3
      whi[nb] = ld8(st + W1_BYTES + w2_off(row, 4 + g));    // j = 16+4g .. +3
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- H^T chunk: [32 j][32 m] = W1[j] . x[m]
    f32x4 h[2][2];
#pragma unroll
    for (int jb = 0; jb < 2; ++jb) { h[jb][0] = f32x4{0, 0, 0, 0}; h[jb][1] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int jb = 0; jb < 2; ++jb) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, wa[ks][jb]);
        h[jb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, xf[0][ks], h[jb][0], 0, 0, 0);
        h[jb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, xf[1][ks], h[jb][1], 0, 0, 0);
      }
    }
    // ---- bias + ReLU, repack as the K=32 B operand: element e <- hidden 4g+e (e<4), 16+4g+e-4
    const f32x4 b1a = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 4 * g);
    const f32x4 b1b = *reinterpret_cast<const f32x4*>(sb1 + ch * HC + 16 + 4 * g);
    bf16x8 hb[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = fmaxf(h[0][mb][r] + b1a[r], 0.f);
        v[4 + r] = fmaxf(h[1][mb][r] + b1b[r], 0.f);
      }
      hb[mb] = __builtin_bit_cast(bf16x8, pack16<bf16>(v));
    }
    // ---- out^T[n][m] += W2[n][chunk j] . H^T[j][m]
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const bf16x8 wb = __builtin_bit_cast(bf16x8, u32x4{wlo[nb].x, wlo[nb].y, whi[nb].x, whi[nb].y});
      acc[nb][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb, hb[0], acc[nb][0], 0, 0, 0);
      acc[nb][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb, hb[1], acc[nb][1], 0, 0, 0);
    }
    if (more) stg.store(smem + ((ch + 1) & 1) * STAGE, tid);
    __syncthreads();
  }

  // ---- epilogue: + b2 + residual, LayerNorm over n, bf16 store.  Lane holds, for each of its
  // two rows m = m0 + 16mb + c16, columns n = 16nb + 4g + r (r = 0..3, nb = 0..15).
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    const int m = m0 + 16 * mb + c16;
    const bool live = m < a.M;
    const bf16* xr = (const bf16*)a.x + (size_t)(live ? m : 0) * a.ldx;
    float s = 0.f;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const int n = 16 * nb + 4 * g;
      const f32x4 b2 = *reinterpret_cast<const f32x4*>(a.b2 + n);
      const u32x2 rv = live ? ld8(xr + n) : u32x2{0, 0};
      const float r0 = __uint_as_float(rv.x << 16), r1 = __uint_as_float(rv.x & 0xffff0000u);
      const float r2 = __uint_as_float(rv.y << 16), r3 = __uint_as_float(rv.y & 0xffff0000u);
      acc[nb][mb][0] += b2[0] + r0;
      acc[nb][mb][1] += b2[1] + r1;
      acc[nb][mb][2] += b2[2] + r2;
      acc[nb][mb][3] += b2[3] + r3;
      s += acc[nb][mb][0] + acc[nb][mb][1] + acc[nb][mb][2] + acc[nb][mb][3];
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const float mean = s * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dv = acc[nb][mb][r] - mean;
        q += dv * dv;
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    const float rs = rsqrtf(q * (1.f / D) + 1e-5f);
    if (!live) continue;
    bf16* yr = (bf16*)a.y + (size_t)m * a.ldy;
    // optional second output y + pos (the encoder's last layer: the cross-attention K input)
    const bf16* pr = a.ypos ? (const bf16*)a.pos + (size_t)(m % a.pos_period) * D : nullptr;
    bf16* ypr = a.ypos ? (bf16*)a.ypos + (size_t)m * a.ldy : nullptr;
#pragma unroll
    for (int nb = 0; nb < 16; ++nb) {
      const int n = 16 * nb + 4 * g;
      const f32x4 ga = *reinterpret_cast<const f32x4*>(a.gamma + n);
      const f32x4 be = *reinterpret_cast<const f32x4*>(a.beta + n);
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (acc[nb][mb][r] - mean) * rs * ga[r] + be[r];
      st8(yr + n, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
      if (ypr) {
        const u32x2 pv = ld8(pr + n);
        st8(ypr + n, u32x2{pack_bf16x2(o[0] + __uint_as_float(pv.x << 16), o[1] + __uint_as_float(pv.x & 0xffff0000u)),
                           pack_bf16x2(o[2] + __uint_as_float(pv.y << 16), o[3] + __uint_as_float(pv.y & 0xffff0000u))});
      }
    }
  }
}

}  // namespace

int spe_launch_ffn_ln(const FfnArgs& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (a.ypos && (!a.pos || a.pos_period <= 0)) return -5;
  if (a.D != D || a.F % HC || a.F > FMAX || (a.ldx % 8) || (a.ldy % 8) || (a.ld1 % 8) || (a.ld2 % 8)) return -5;
  hipLaunchKernelGGL(ffn_ln_kernel, dim3((a.M + BM - 1) / BM), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}
