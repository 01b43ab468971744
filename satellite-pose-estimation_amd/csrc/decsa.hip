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
//   2. attention per (query, head) on the VALU in fp32, four lanes of 8 dims each: scores scaled
//      by 1/sqrt(32), softmax (max pass, then exp-weighted sums of v), written over the query's
//      own q slot as bf16 (the out-projection's W fragments are in flight meanwhile).
//   3. out-projection the same way as 1., + bo + tgt (the residual as stored), fp32 rows to LDS,
//      then the LayerNorm (one wave per row, 4 columns a lane) and the bf16 store of tgt.
#include "spe_common.h"
#include "spe_kernels.h"

#include <cstdlib>

namespace {

constexpr int D = 256, NT = 512, NW = NT / 64, QMAX = 64;
constexpr int XLD = D + 8;                 // x rows in LDS (bf16 elements): 528 B, conflict-free b128 reads
constexpr int QKVLD = 3 * D + 8;           // q | k | v rows (bf16): 1552 B
constexpr int YLD = D + 4;                 // fp32 rows before the LayerNorm

// W fragments of one 16-column tile (A operand of the C^T form): lane l holds row 16 t + (l & 15),
// k 8 (l >> 4) .. +8 of each of the 8 32-wide K steps.  The weights are stored fragment-packed
// (spe_launch_wfrag_pack), so each K-step is one contiguous 1 KB wave load; from row-major rows
// every lane of a load sat on its own 128-byte line, 16 lines per 16 lanes.  All of a wave's tiles
// are fetched before the first MFMA (the few rows give each tile only RT x 8 MFMAs).
SPE_DEV void w_frags(u32x4 (&wf)[8], const void* w, int tile, int lane) {
  const bf16* wp = (const bf16*)w + ((size_t)tile * 8 * 64 + lane) * 8;
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) wf[ks] = ld16(wp + 512 * ks);
}
// D^T tile (16 output columns x 16 rows m0..) = W . x[m0..]^T over K = 256; B = x row m0 + (l & 15)
SPE_DEV f32x4 tile_wx(const u32x4 (&wf)[8], const bf16* xs, int xld, int m0, int lane,
                      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f}) {
  const bf16* xp = xs + (m0 + (lane & 15)) * xld + 8 * (lane >> 4);
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[ks]),
                                                  __builtin_bit_cast(bf16x8, ld16(xp + 32 * ks)), acc, 0, 0, 0);
  return acc;                                // lane: row m0 + (l & 15), columns n0 + 4 (l >> 4) + e
}

// QM: the rows the LDS is sized for (16: Q <= 16, a quarter of the 64-row form's 133 KB)
template <int QM>
__global__ __launch_bounds__(NT) void decsa_kernel(DecSaArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 xs[QM * XLD];
  __shared__ __attribute__((aligned(16))) char big[QM * QKVLD * 2];   // q|k|v, then the fp32 rows
  bf16* qkv = reinterpret_cast<bf16*>(big);
  float* ys = reinterpret_cast<float*>(big);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x, Q = a.Q, RT = (Q + 15) / 16;
  bf16* tg = (bf16*)a.tgt + (size_t)b * Q * a.ldt;

  // ---- 1. q | k | v: 48 column tiles of 16, 6 per wave (tile wid + 8 j); the W fragments are
  // requested first, so their round trip overlaps the tgt rows' (which stage through LDS)
  constexpr int CT1 = 3 * D / 16 / NW;
  u32x4 wf1[CT1][8];
  auto tile1 = [&](int j) { return wid + NW * j; };
#pragma unroll
  for (int j = 0; j < CT1; ++j) {
    const int n0 = tile1(j) * 16;
    const bool isv = n0 >= 2 * D;
    w_frags(wf1[j], isv ? a.wv : a.wqk, (isv ? n0 - 2 * D : n0) / 16, lane);
  }
  // tgt rows -> LDS (rows past Q zero)
  for (int i = tid; i < RT * 16 * (D / 8); i += NT) {
    const int r = i / (D / 8), c = i % (D / 8);
    st16(xs + r * XLD + 8 * c, r < Q ? ld16(tg + (size_t)r * a.ldt + 8 * c) : u32x4{0, 0, 0, 0});
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < CT1; ++j) {
    const int n0 = tile1(j) * 16;
    const bool isv = n0 >= 2 * D;
    const int nw = isv ? n0 - 2 * D : n0;
    const int ncol = n0 + 4 * (lane >> 4);
    const f32x4 bias = *reinterpret_cast<const f32x4*>((isv ? a.bv : a.bqk) + nw + 4 * (lane >> 4));
    for (int rt = 0; rt < RT; ++rt) {
      f32x4 acc = tile_wx(wf1[j], xs, XLD, rt * 16, lane);
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
  // the out-projection's W fragments travel during the attention
  constexpr int CT3 = D / 16 / NW;
  u32x4 wf3[CT3][8];
#pragma unroll
  for (int j = 0; j < CT3; ++j) w_frags(wf3[j], a.wo, wid * CT3 + j, lane);
  __syncthreads();

  // ---- 2. attention: four lanes per (query i, head h), 8 of the head's 32 dims each (the score's
  // partial dot products summed over the four lanes); o_ih overwrites the lane's own q dims
  for (int idx = tid; idx < 32 * Q; idx += NT) {
    const int c = idx & 3, h = (idx >> 2) & 7, i = idx >> 5;
    const int col = h * 32 + 8 * c;
    float q[8];
    unpack16<bf16>(ld16(qkv + i * QKVLD + col), q);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] *= a.scale;
    auto score = [&](int j) {
      float k[8];
      unpack16<bf16>(ld16(qkv + j * QKVLD + D + col), k);
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s = fmaf(q[e], k[e], s);
      // sum over the lane quad: DPP quad_perm [1,0,3,2] then [2,3,0,1] (no LDS round trip)
      s += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0xB1, 0xF, 0xF, false));
      return s + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s), 0x4E, 0xF, 0xF, false));
    };
    float mx = -INFINITY;
    for (int j = 0; j < Q; ++j) mx = fmaxf(mx, score(j));
    float o[8], l = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
    for (int j = 0; j < Q; ++j) {
      const float p = expf(score(j) - mx);
      l += p;
      float v[8];
      unpack16<bf16>(ld16(qkv + j * QKVLD + 2 * D + col), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fmaf(p, v[e], o[e]);
    }
    const float inv = 1.f / l;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] *= inv;
    st16(qkv + i * QKVLD + col, pack16<bf16>(o));
  }
  __syncthreads();

  // ---- 3. out-projection + bo + residual (registers), then the fp32 rows over q|k|v
  f32x4 yo[CT3][QM / 16];
#pragma unroll
  for (int j = 0; j < CT3; ++j) {
    const int n0 = (wid * CT3 + j) * 16;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(a.bo + n0 + 4 * (lane >> 4));
#pragma unroll
    for (int rt = 0; rt < QM / 16; ++rt) {
      if (rt >= RT) break;
      f32x4 acc = tile_wx(wf3[j], qkv, QKVLD, rt * 16, lane);
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
  for (int j = 0; j < CT3; ++j) {
    const int n0 = (wid * CT3 + j) * 16;
#pragma unroll
    for (int rt = 0; rt < QM / 16; ++rt) {
      if (rt >= RT) break;
      const int m = rt * 16 + (lane & 15);
      *reinterpret_cast<f32x4*>(ys + m * YLD + n0 + 4 * (lane >> 4)) = yo[j][rt];
    }
  }
  __syncthreads();

  // LayerNorm, one wave per row, columns 4 lane .. +4
  const f32x4 gm = *reinterpret_cast<const f32x4*>(a.g + 4 * lane);
  const f32x4 bt = *reinterpret_cast<const f32x4*>(a.b + 4 * lane);
  for (int m = wid; m < Q; m += NW) {
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

// tgt = LayerNorm(tgt + x . Wo^T + bo) per image: the cross-attention's out-projection + norm2
// (REV/models/transformer.py:233-234), decsa's phase 3 on its own -- one launch instead of a
// few-row GEMM and a LayerNorm, the rows never leaving LDS between them.
template <int QM>
__global__ __launch_bounds__(NT) void decproj_kernel(DecProjArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 rs[QM * XLD];   // tgt rows (the residual)
  __shared__ __attribute__((aligned(16))) bf16 xs[QM * XLD];   // input rows
  __shared__ __attribute__((aligned(16))) float ys[QM * YLD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x, Q = a.Q, RT = (Q + 15) / 16;
  bf16* tg = (bf16*)a.tgt + (size_t)b * Q * a.ldt;
  const bf16* xg = (const bf16*)a.x + (size_t)b * Q * a.ldx;
  constexpr int CT3 = D / 16 / NW;
  u32x4 wf[CT3][8];
#pragma unroll
  for (int j = 0; j < CT3; ++j) w_frags(wf[j], a.wo, wid * CT3 + j, lane);
  for (int i = tid; i < RT * 16 * (D / 8); i += NT) {
    const int r = i / (D / 8), c = i % (D / 8);
    st16(xs + r * XLD + 8 * c, r < Q ? ld16(xg + (size_t)r * a.ldx + 8 * c) : u32x4{0, 0, 0, 0});
    st16(rs + r * XLD + 8 * c, r < Q ? ld16(tg + (size_t)r * a.ldt + 8 * c) : u32x4{0, 0, 0, 0});
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < CT3; ++j) {
    const int n0 = (wid * CT3 + j) * 16;
    const f32x4 bias = *reinterpret_cast<const f32x4*>(a.bo + n0 + 4 * (lane >> 4));
#pragma unroll
    for (int rt = 0; rt < QM / 16; ++rt) {
      if (rt >= RT) break;
      f32x4 acc = tile_wx(wf[j], xs, XLD, rt * 16, lane);
      const int m = rt * 16 + (lane & 15);
      const u32x2 r = ld8(rs + m * XLD + n0 + 4 * (lane >> 4));
      acc[0] += bias[0] + __uint_as_float(r.x << 16);
      acc[1] += bias[1] + __uint_as_float(r.x & 0xffff0000u);
      acc[2] += bias[2] + __uint_as_float(r.y << 16);
      acc[3] += bias[3] + __uint_as_float(r.y & 0xffff0000u);
      *reinterpret_cast<f32x4*>(ys + m * YLD + n0 + 4 * (lane >> 4)) = acc;
    }
  }
  __syncthreads();
  const f32x4 gm = *reinterpret_cast<const f32x4*>(a.g + 4 * lane);
  const f32x4 bt = *reinterpret_cast<const f32x4*>(a.b + 4 * lane);
  for (int m = wid; m < Q; m += NW) {
    const f32x4 y = *reinterpret_cast<const f32x4*>(ys + m * YLD + 4 * lane);
    const float mean = wave_sum((y[0] + y[1]) + (y[2] + y[3])) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (y[e] - mean) * (y[e] - mean);
    const float rsd = rsqrtf(wave_sum(q) * (1.f / D) + 1e-5f);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (y[e] - mean) * rsd * gm[e] + bt[e];
    st8(tg + (size_t)m * a.ldt + 4 * lane, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
  }
}

// The cross-attention's tail and its out-projection + norm2 as one launch per layer (Q <= 48):
//   u_h = the key-split merge of xattn.hip's partials, o_h = Wv_h u_h + bv_h rounded to bf16 (the
//   rounding the separate merge kernel stored), tgt = LayerNorm(tgt + o . Wo^T + bo)
// (REV/models/transformer.py:230-234) -- xattn's merge + value-projection kernel and decproj as one
// launch, u never leaving LDS.  u enters the value projection's bf16 MFMAs as hi + lo planes (u to
// about 2^-17 relative, as the separate kernel's fp32 FMAs had it), 16 queries at a time.
constexpr int QX = 16, QXM = 48, ULD = 8 * D + 8;   // u planes [16][2048 + 8] bf16: 4112 B rows, conflict-free b128 reads
constexpr float XNEG = -1.0e30f;
__global__ __launch_bounds__(NT) void decxproj_kernel(DecProjArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 uh[QX * ULD];
  __shared__ __attribute__((aligned(16))) bf16 ul[QX * ULD];
  __shared__ __attribute__((aligned(16))) bf16 xs[QXM * XLD];   // o rows
  float* ys = reinterpret_cast<float*>(uh);                      // fp32 rows once u has been read
  static_assert(QXM * YLD * 4 <= QX * ULD * 2, "ys fits the hi plane");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int b = blockIdx.x, Q = a.Q, R = 8 * Q, S = a.splits, QC = (Q + QX - 1) / QX;
  bf16* tg = (bf16*)a.tgt + (size_t)b * Q * a.ldt;
  // wave wid: head wid of the value projection and columns 32 wid .. +32 of the out-projection;
  // Wv's fragments travel while the first partials are merged
  u32x4 wvf[2][8], wf[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j) w_frags(wvf[j], a.wv, 2 * wid + j, lane);
  f32x4 bvv[2], bov[2];                         // biases and the LayerNorm affine: loaded up front too
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    bvv[j] = *reinterpret_cast<const f32x4*>(a.bv + 32 * wid + 16 * j + 4 * (lane >> 4));
    bov[j] = *reinterpret_cast<const f32x4*>(a.bo + 32 * wid + 16 * j + 4 * (lane >> 4));
  }
  const f32x4 gm = *reinterpret_cast<const f32x4*>(a.g + 4 * lane);
  const f32x4 bt = *reinterpret_cast<const f32x4*>(a.b + 4 * lane);
  const size_t base = (size_t)b * S * R;
  // 1. u = sum_s 2^(m_s - M) U_s / sum_s 2^(m_s - M) l_s per attention row r = 8 q + h of queries
  // q0 .. q0 + 16, 16 dims an item, merged online four splits at a time (all four splits' loads in
  // flight together), into plane row q - q0, columns 256 h ..
  auto merge = [&](int q0) {
    const int nq = min(QX, Q - q0);
    for (int i = tid; i < (QX - nq) * D; i += NT) {   // plane rows past the queries: zero (256 chunks a row)
      const int r = nq + i / D, c = i % D;
      st16(uh + r * ULD + 8 * c, u32x4{0, 0, 0, 0});
      st16(ul + r * ULD + 8 * c, u32x4{0, 0, 0, 0});
    }
    for (int it = tid; it < 8 * nq * 16; it += NT) {
      const int r = 8 * q0 + (it >> 4), c = it & 15;
      float M = XNEG, L = 0.f;
      f32x4 u[4] = {};
      for (int s0 = 0; s0 < S; s0 += 4) {
        float ms[4], ls[4];
        f32x4 us[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const size_t pr = base + (size_t)min(s0 + j, S - 1) * R + r;
          ms[j] = s0 + j < S ? a.pm[pr] : XNEG;
          ls[j] = a.pl[pr];
#pragma unroll
          for (int g = 0; g < 4; ++g) us[j][g] = *reinterpret_cast<const f32x4*>(a.pu + pr * D + 16 * c + 4 * g);
        }
        const float Mn = fmaxf(fmaxf(M, fmaxf(ms[0], ms[1])), fmaxf(ms[2], ms[3]));
        const float sc = __builtin_amdgcn_exp2f(M - Mn);
        L *= sc;
#pragma unroll
        for (int g = 0; g < 4; ++g) u[g] *= sc;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float w = __builtin_amdgcn_exp2f(ms[j] - Mn);   // 0 for the padded splits
          L += w * ls[j];
#pragma unroll
          for (int g = 0; g < 4; ++g) u[g] += w * us[j][g];
        }
        M = Mn;
      }
      const float il = 1.f / L;
      uint32_t hi[8], lo[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float x0 = u[e >> 1][2 * (e & 1)] * il, x1 = u[e >> 1][2 * (e & 1) + 1] * il;
        hi[e] = pack_bf16x2(x0, x1);
        lo[e] = pack_bf16x2(x0 - __uint_as_float(hi[e] << 16), x1 - __uint_as_float(hi[e] & 0xffff0000u));
      }
      const int off = ((r >> 3) - q0) * ULD + (r & 7) * D + 16 * c;
      st16(uh + off, u32x4{hi[0], hi[1], hi[2], hi[3]});
      st16(uh + off + 8, u32x4{hi[4], hi[5], hi[6], hi[7]});
      st16(ul + off, u32x4{lo[0], lo[1], lo[2], lo[3]});
      st16(ul + off + 8, u32x4{lo[4], lo[5], lo[6], lo[7]});
    }
  };
  // 2. o_h = Wv_h (u_hi + u_lo) + bv_h, bf16 rows q0 .. into xs
  auto value_proj = [&](int q0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n0 = 32 * wid + 16 * j;
      f32x4 acc = tile_wx(wvf[j], uh + wid * D, ULD, 0, lane);
      acc = tile_wx(wvf[j], ul + wid * D, ULD, 0, lane, acc);
      const f32x4 bias = bvv[j];
      st8(xs + (q0 + (lane & 15)) * XLD + n0 + 4 * (lane >> 4),
          u32x2{pack_bf16x2(acc[0] + bias[0], acc[1] + bias[1]), pack_bf16x2(acc[2] + bias[2], acc[3] + bias[3])});
    }
  };
  for (int rc = 0; rc + 1 < QC; ++rc) {
    merge(QX * rc);
    __syncthreads();
    value_proj(QX * rc);
    __syncthreads();                            // the planes free for the next queries
  }
  merge(QX * (QC - 1));
  // Wo's fragments travel during the last value projection (not up front: registers)
#pragma unroll
  for (int j = 0; j < 2; ++j) w_frags(wf[j], a.wo, 2 * wid + j, lane);
  __syncthreads();
  value_proj(QX * (QC - 1));
  __syncthreads();                              // o visible; the hi plane becomes ys
  // 3. out-projection + bo + residual (tgt as stored), then the LayerNorm (decproj's phases)
  for (int rt = 0; rt < QC; ++rt) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n0 = 32 * wid + 16 * j;
      const f32x4 bias = bov[j];
      f32x4 acc = tile_wx(wf[j], xs, XLD, 16 * rt, lane);
      const int m = 16 * rt + (lane & 15);
      const u32x2 r = m < Q ? ld8(tg + (size_t)m * a.ldt + n0 + 4 * (lane >> 4)) : u32x2{0, 0};
      acc[0] += bias[0] + __uint_as_float(r.x << 16);
      acc[1] += bias[1] + __uint_as_float(r.x & 0xffff0000u);
      acc[2] += bias[2] + __uint_as_float(r.y << 16);
      acc[3] += bias[3] + __uint_as_float(r.y & 0xffff0000u);
      *reinterpret_cast<f32x4*>(ys + m * YLD + n0 + 4 * (lane >> 4)) = acc;
    }
  }
  __syncthreads();
  for (int m = wid; m < Q; m += NW) {
    const f32x4 y = *reinterpret_cast<const f32x4*>(ys + m * YLD + 4 * lane);
    const float mean = wave_sum((y[0] + y[1]) + (y[2] + y[3])) * (1.f / D);
    float q = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) q += (y[e] - mean) * (y[e] - mean);
    const float rsd = rsqrtf(wave_sum(q) * (1.f / D) + 1e-5f);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (y[e] - mean) * rsd * gm[e] + bt[e];
    st8(tg + (size_t)m * a.ldt + 4 * lane, u32x2{pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])});
  }
}

}  // namespace

int spe_launch_decproj(const DecProjArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.pm) {                                   // the merge form (x comes from the partials)
    if (a.Q < 1 || a.Q > QXM || a.splits < 1 || a.ldt % 8 || !a.pl || !a.pu || !a.wv ||
        !a.bv || !a.tgt || !a.wo || !a.bo || !a.g || !a.b)
      return 1;
    hipLaunchKernelGGL(decxproj_kernel, dim3(a.B), dim3(NT), 0, s, a);
    return (int)hipGetLastError();
  }
  if (a.Q < 1 || a.Q > QMAX || a.ldt % 8 || a.ldx % 8 || !a.tgt || !a.x || !a.wo || !a.bo || !a.g || !a.b)
    return 1;
  if (a.Q <= 16) hipLaunchKernelGGL(decproj_kernel<16>, dim3(a.B), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(decproj_kernel<QMAX>, dim3(a.B), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}

// 1 = not applicable (the caller runs the separate launches)
int spe_launch_decsa(const DecSaArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.Q < 1 || a.Q > QMAX || a.ldt % 8 || !a.tgt || !a.wqk || !a.wv ||
      !a.wo || !a.bqk || !a.bv || !a.bo || !a.qpos || !a.g || !a.b)
    return 1;
  if (a.Q <= 16) hipLaunchKernelGGL(decsa_kernel<16>, dim3(a.B), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(decsa_kernel<QMAX>, dim3(a.B), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}

namespace {
// The decoder FFN's split-F product for few rows (bf16, d = 256; REV/models/transformer.py:236-238):
// workgroup (16-row tile, 256-wide hidden chunk c): H = relu(x . W1c^T + b1c) rounded to bf16 (the
// rounding ffn.hip's hidden has), partial_c = H . W2c^T in fp32; ffn.hip's reduce kernel then
// writes y = LN(x + sum_c partial_c + b2).  B.Q = 704 rows give 44 x 8 = 352 workgroups, each
// with its 256 KB of weight fragments in flight from the start (the 128-row split-F tiles of
// ffn.hip ran 48 workgroups through an 8-step chunk loop).  W1 fragment-packed as [F] rows, W2
// per chunk (columns 256 c .. of [256][F] packed as a [256][256] block).
__global__ __launch_bounds__(NT) void decffn_kernel(DecFfnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 xs[16 * XLD];
  __shared__ __attribute__((aligned(16))) bf16 hs[16 * XLD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = a.F / D, c = blockIdx.x % nc, r0 = (blockIdx.x / nc) * 16;
  u32x4 w1f[2][8], w2f[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    w_frags(w1f[j], a.w1, 16 * c + 2 * wid + j, lane);
    w_frags(w2f[j], (const bf16*)a.w2 + (size_t)c * D * D, 2 * wid + j, lane);
  }
  f32x4 b1v[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b1v[j] = *reinterpret_cast<const f32x4*>(a.b1 + D * c + 32 * wid + 16 * j + 4 * (lane >> 4));
  if (tid < 16 * (D / 8)) {
    const int r = tid / (D / 8), q = tid % (D / 8);
    st16(xs + r * XLD + 8 * q, r0 + r < a.M ? ld16((const bf16*)a.x + (size_t)(r0 + r) * a.ldx + 8 * q) : u32x4{0, 0, 0, 0});
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 acc = tile_wx(w1f[j], xs, XLD, 0, lane);
    float h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) h[e] = fmaxf(acc[e] + b1v[j][e], 0.f);
    st8(hs + (lane & 15) * XLD + 32 * wid + 16 * j + 4 * (lane >> 4),
        u32x2{pack_bf16x2(h[0], h[1]), pack_bf16x2(h[2], h[3])});
  }
  __syncthreads();
  const int m = r0 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 acc = tile_wx(w2f[j], hs, XLD, 0, lane);
    if (m < a.M) *reinterpret_cast<f32x4*>(a.partial + ((size_t)c * a.M + m) * D + 32 * wid + 16 * j + 4 * (lane >> 4)) = acc;
  }
}

// y = x . W^T (+ bias) + R[m % period] in bf16 over K = 256 for the decoder's few rows: the
// cross-attention's folded query projection q' (2048 columns, R = query_pos . Wqk^T + bqk), one
// workgroup per (16 rows, 256 columns) with its 128 KB of packed W fragments requested up front.
__global__ __launch_bounds__(NT) void decq_kernel(DecQArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 xs[16 * XLD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nc = a.N / D, c = blockIdx.x % nc, r0 = (blockIdx.x / nc) * 16;
  u32x4 wf[2][8];
#pragma unroll
  for (int j = 0; j < 2; ++j) w_frags(wf[j], a.w, 16 * c + 2 * wid + j, lane);
  if (tid < 16 * (D / 8)) {
    const int r = tid / (D / 8), q = tid % (D / 8);
    st16(xs + r * XLD + 8 * q, r0 + r < a.M ? ld16((const bf16*)a.x + (size_t)(r0 + r) * a.ldx + 8 * q) : u32x4{0, 0, 0, 0});
  }
  const int m = r0 + (lane & 15);
  u32x2 rv[2] = {};
  f32x4 bv[2] = {};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = D * c + 32 * wid + 16 * j + 4 * (lane >> 4);
    if (m < a.M && a.R) rv[j] = ld8((const bf16*)a.R + (size_t)(m % a.period) * a.ldr + n);
    if (a.bias) bv[j] = *reinterpret_cast<const f32x4*>(a.bias + n);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const f32x4 acc = tile_wx(wf[j], xs, XLD, 0, lane);
    const int n = D * c + 32 * wid + 16 * j + 4 * (lane >> 4);
    const float o0 = acc[0] + bv[j][0] + __uint_as_float(rv[j].x << 16);
    const float o1 = acc[1] + bv[j][1] + __uint_as_float(rv[j].x & 0xffff0000u);
    const float o2 = acc[2] + bv[j][2] + __uint_as_float(rv[j].y << 16);
    const float o3 = acc[3] + bv[j][3] + __uint_as_float(rv[j].y & 0xffff0000u);
    if (m < a.M) st8((bf16*)a.y + (size_t)m * a.ldy + n, u32x2{pack_bf16x2(o0, o1), pack_bf16x2(o2, o3)});
  }
}

__global__ __launch_bounds__(256) void wfrag_pack_kernel(const bf16* w, int ld, int N, bf16* dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // one 16-byte fragment: (tile, K-step, lane)
  if (i >= N * 32) return;
  const int l = i & 63, ks = (i >> 6) & 7, t = i >> 9;
  st16(dst + (size_t)i * 8, ld16(w + (size_t)(16 * t + (l & 15)) * ld + 32 * ks + 8 * (l >> 4)));
}
}  // namespace

int spe_launch_wfrag_pack(const void* w, int ld, int N, void* dst, hipStream_t s) {
  if (!w || !dst || N < 16 || N % 16 || ld < D || ld % 8) return -5;
  hipLaunchKernelGGL(wfrag_pack_kernel, dim3((N * 32 + 255) / 256), dim3(256), 0, s, (const bf16*)w, ld, N, (bf16*)dst);
  return (int)hipGetLastError();
}

int spe_launch_decffn(const DecFfnArgs& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (!a.x || !a.w1 || !a.b1 || !a.w2 || !a.partial || a.F < D || a.F % D || a.ldx % 8) return -5;
  hipLaunchKernelGGL(decffn_kernel, dim3(((a.M + 15) / 16) * (a.F / D)), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_decq(const DecQArgs& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (!a.x || !a.w || !a.y || a.N < D || a.N % D || a.ldx % 8 || a.ldy % 4 || (a.R && (a.period < 1 || a.ldr % 4)))
    return -5;
  hipLaunchKernelGGL(decq_kernel, dim3(((a.M + 15) / 16) * (a.N / D)), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}
