// Decoder self-attention block of the bf16 models, one launch per layer:
//
//     tgt = LayerNorm(tgt + SelfAttn(q = k = tgt + query_pos, v = tgt) . Wo^T + bo)       (norm1)
//
// REV/models/transformer.py:218-228 (TransformerDecoderLayer.forward_post, self_attn + norm1).
// The block mixes rows only within one image (its Q object queries), so one workgroup owns one
// image and keeps its rows in LDS from the first read of tgt to the LayerNorm's store: the
// separate path (q/k and v projections, attention, output projection + norm: four launches of
// a few rows each, with q/k/v and the attention output round-tripping HBM) becomes one.
//
//   1. q, k, v = tgt . [Wqk; Wv]^T + b (+ query_pos . Wqk^T, precomputed [Q][512], on q and k):
//      16x16x32 bf16 MFMAs in the C^T form D[n][m] = W[n] . x[m] (W fragments from L2/global,
//      the x rows from LDS), stored to LDS as bf16 -- the rounding the separate path's GEMM
//      output had.
//   2. attention per (query, head) on the VALU in fp32: scores scaled by 1/sqrt(32), softmax
//      (max pass, then exp-weighted sums of v), written over the query's own q slot as bf16.
//   3. out-projection the same way as 1., + bo + tgt (the residual as stored), fp32 rows to LDS,
//      then the LayerNorm (one wave per row, 4 columns a lane) and the bf16 store of tgt.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int D = 256, NT = 256, QMAX = 64;
constexpr int XLD = D + 8;                 // x rows in LDS (bf16 elements): 528 B, conflict-free b128 reads
constexpr int QKVLD = 3 * D + 8;           // q | k | v rows (bf16): 1552 B
constexpr int YLD = D + 4;                 // fp32 rows before the LayerNorm

// D^T tile (16 output columns n0.. x 16 rows m0..) += W[n0..][K] . x[m0..][K]^T over K = 256:
// lane l: A = W row n0 + (l & 15), k 8 (l >> 4) .. +8 of each 32-wide step; B = x row m0 + (l & 15)
SPE_DEV f32x4 tile_wx(const bf16* w, int ldw, int n0, const bf16* xs, int xld, int m0, int lane) {
  const bf16* wp = w + (size_t)(n0 + (lane & 15)) * ldw + 8 * (lane >> 4);
  const bf16* xp = xs + (m0 + (lane & 15)) * xld + 8 * (lane >> 4);
  u32x4 wf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) wf[ks] = ld16(wp + 32 * ks);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ks]),
                                                  __builtin_bit_cast(bf16x8, ld16(xp + 32 * ks)), acc, 0, 0, 0);
  return acc;                                // lane: row m0 + (l & 15), columns n0 + 4 (l >> 4) + e
}

__global__ __launch_bounds__(NT) void decsa_kernel(DecSaArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 xs[QMAX * XLD];
  __shared__ __attribute__((aligned(16))) char big[QMAX * QKVLD * 2];   // q|k|v, then the fp32 rows
  bf16* qkv = reinterpret_cast<bf16*>(big);
  float* ys = reinterpret_cast<float*>(big);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x, Q = a.Q, RT = (Q + 15) / 16;
  bf16* tg = (bf16*)a.tgt + (size_t)b * Q * a.ldt;

  // tgt rows -> LDS (rows past Q zero)
  for (int i = tid; i < RT * 16 * (D / 8); i += NT) {
    const int r = i / (D / 8), c = i % (D / 8);
    st16(xs + r * XLD + 8 * c, r < Q ? ld16(tg + (size_t)r * a.ldt + 8 * c) : u32x4{0, 0, 0, 0});
  }
  __syncthreads();

  // ---- 1. q | k | v: 48 column tiles of 16, 12 per wave
  for (int ct = wid; ct < 3 * D / 16; ct += NT / 64) {
    const int n0 = ct * 16;
    const bool isv = n0 >= 2 * D;
    const bf16* w = isv ? (const bf16*)a.wv : (const bf16*)a.wqk;
    const int ldw = isv ? a.ldv : a.ldqk, nw = isv ? n0 - 2 * D : n0;
    const int ncol = n0 + 4 * (lane >> 4);
    const f32x4 bias = *reinterpret_cast<const f32x4*>((isv ? a.bv : a.bqk) + nw + 4 * (lane >> 4));
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 acc = tile_wx(w, ldw, nw, xs, XLD, rt * 16, lane);
      const int m = rt * 16 + (lane & 15);
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = acc[e] + bias[e];
      if (!isv && m < Q) {                     // + query_pos . Wqk^T
        const u32x2 pw = ld8((const bf16*)a.qpos + (size_t)m * 2 * D + nw + 4 * (lane >> 4));
        o[0] += __uint_as_float(pw.x << 16); o[1] += __uint_as_float(pw.x & 0xffff0000u);
        o[2] += __uint_as_float(pw.y << 16); o[3] += __uint_as_float(pw.y & 0xffff0000u);
      }
      st8(qkv + m * QKVLD + ncol, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
    }
  }
  __syncthreads();

  // ---- 2. attention, one thread per (query i, head h); o_ih overwrites q_ih (only this thread reads it)
  for (int idx = tid; idx < 8 * Q; idx += NT) {
    const int i = idx >> 3, h = idx & 7;
    float q[32];
#pragma unroll
    for (int c = 0; c < 4; ++c) unpack16<bf16>(ld16(qkv + i * QKVLD + h * 32 + 8 * c), q + 8 * c);
#pragma unroll
    for (int e = 0; e < 32; ++e) q[e] *= a.scale;
    auto score = [&](int j) {
      const bf16* kp = qkv + j * QKVLD + D + h * 32;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float k[8];
        unpack16<bf16>(ld16(kp + 8 * c), k);
#pragma unroll
        for (int e = 0; e < 8; ++e) s = fmaf(q[8 * c + e], k[e], s);
      }
      return s;
    };
    float mx = -INFINITY;
    for (int j = 0; j < Q; ++j) mx = fmaxf(mx, score(j));
    float o[32], l = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) o[e] = 0.f;
    for (int j = 0; j < Q; ++j) {
      const float p = expf(score(j) - mx);
      l += p;
      const bf16* vp = qkv + j * QKVLD + 2 * D + h * 32;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float v[8];
        unpack16<bf16>(ld16(vp + 8 * c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[8 * c + e] = fmaf(p, v[e], o[8 * c + e]);
      }
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int e = 0; e < 32; ++e) o[e] *= inv;
#pragma unroll
    for (int c = 0; c < 4; ++c) st16(qkv + i * QKVLD + h * 32 + 8 * c, pack16<bf16>(o + 8 * c));
  }
  __syncthreads();

  // ---- 3. out-projection + bo + residual (registers), then the fp32 rows over q|k|v
  f32x4 yo[4][QMAX / 16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n0 = (wid * 4 + j) * 16;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(a.bo + n0 + 4 * (lane >> 4));
#pragma unroll
    for (int rt = 0; rt < QMAX / 16; ++rt) {
      if (rt >= RT) break;
      f32x4 acc = tile_wx((const bf16*)a.wo, a.ldo, n0, qkv, QKVLD, rt * 16, lane);
      const int m = rt * 16 + (lane & 15);
      const u32x2 r = ld8(xs + m * XLD + n0 + 4 * (lane >> 4));
      acc[0] += bias[0] + __uint_as_float(r.x << 16);
      acc[1] += bias[1] + __uint_as_float(r.x & 0xffff0000u);
      acc[2] += bias[2] + __uint_as_float(r.y << 16);
      acc[3] += bias[3] + __uint_as_float(r.y & 0xffff0000u);
      yo[j][rt] = acc;
    }
  }
  __syncthreads();                              // every wave done reading the attention output
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n0 = (wid * 4 + j) * 16;
#pragma unroll
    for (int rt = 0; rt < QMAX / 16; ++rt) {
      if (rt >= RT) break;
      const int m = rt * 16 + (lane & 15);
      *reinterpret_cast<f32x4*>(ys + m * YLD + n0 + 4 * (lane >> 4)) = yo[j][rt];
    }
  }
  __syncthreads();

  // LayerNorm, one wave per row, columns 4 lane .. +4
  const f32x4 gm = *reinterpret_cast<const f32x4*>(a.g + 4 * lane);
  const f32x4 bt = *reinterpret_cast<const f32x4*>(a.b + 4 * lane);
  for (int m = wid; m < Q; m += NT / 64) {
    const f32x4 y = *reinterpret_cast<const f32x4*>(ys + m * YLD + 4 * lane);
    const float mean = wave_sum((y[0] + y[1]) + (y[2] + y[3])) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (y[e] - mean) * (y[e] - mean);
    const float rs = rsqrtf(wave_sum(q) * (1.f / D) + 1e-5f);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (y[e] - mean) * rs * gm[e] + bt[e];
    st8(tg + (size_t)m * a.ldt + 4 * lane, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
  }
}

}  // namespace

// 1 = not applicable (the caller runs the separate launches)
int spe_launch_decsa(const DecSaArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.Q < 1 || a.Q > QMAX || a.ldt % 8 || a.ldqk % 8 || a.ldv % 8 || a.ldo % 8 || !a.tgt || !a.wqk || !a.wv ||
      !a.wo || !a.bqk || !a.bv || !a.bo || !a.qpos || !a.g || !a.b)
    return 1;
  hipLaunchKernelGGL(decsa_kernel, dim3(a.B), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}
