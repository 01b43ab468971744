// MFMA GEMM / implicit-GEMM convolution for gfx950 with fused epilogues.
//
// One kernel serves every contraction on the path except attention:
//   * ResNet-50 convs (REV/models/backbone.py:114-131 via torchvision), FrozenBN folded into
//     the weights + bias (REV/models/backbone.py:44-54), ReLU / residual add fused;
//   * neck 1x1 / 3x3 convs (REV/models/backbone.py:127-131), concat fused by writing into a
//     channel slice of one NHWC buffer (ldc + column offset);
//   * input_proj (REV/models/detr_speed.py:54-55) and every nn.Linear / MHA projection of the
//     transformer (REV/models/transformer.py:137-145,181-191), with the `src + pos` /
//     `tgt + query_pos` add fused into the A-operand load (REV/models/transformer.py:158,225)
//     and the value projection optionally stored head-transposed ([g][b][hd][token]) for the
//     attention kernel's V^T tiles.
//
// C[M,N] = A[M,K] . W[N,K]^T (+bias, +residual, ReLU).  Activations are NHWC / token-major
// rows, weights row-major [N][Kpad] (Kpad % 64 == 0, zero padded).
// Tile 128x128, 256 threads = 4 waves (2x2), wave tile 64x64 = 4x4 16x16 MFMA fragments.
// One K-step moves 128 bytes of every row: 64 bf16 (2 x mfma_f32_16x16x32_bf16) or 32 fp32
// (8 x mfma_f32_16x16x4f32, exact f32).  Global -> register -> LDS staging, double-buffered,
// XOR-swizzled 16-byte slots (conflict-free ds_read_b128 fragment reads), one barrier per step.
// X3 (the fp32x3 parity mode, SPE_DTYPE_F32X3): fp32 operands are split while they are staged,
// x = hi + lo with hi = bf16(x), lo = bf16(x - hi) (x - hi is exact in fp32), the 32-element
// K-step's hi halves in slots 0-3 and lo halves in slots 4-7 of the same 128-byte LDS row, and
// each fragment product is hi.hi + hi.lo + lo.hi: three mfma_f32_16x16x32_bf16 with fp32
// accumulation instead of eight mfma_f32_16x16x4f32 -- a relative error of ~2^-17 per product
// (the dropped lo.lo term and lo's own rounding) at 5x fewer matrix cycles.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256;
constexpr int STAGE_BYTES = (BM + BN) * 128;          // 32 KiB per stage
constexpr int EPI_LD = BN + 4;                         // fp32 row stride of the epilogue tile
constexpr int SMEM_BYTES = (2 * STAGE_BYTES > BM * EPI_LD * 4) ? 2 * STAGE_BYTES : BM * EPI_LD * 4;

SPE_DEV int swz(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <typename T, int MODE, int RS = 32>
struct ALoader {
  static constexpr int CE = Chunk<T>::CE;
  // per-thread: 4 rows RS apart, one chunk column
  const char* base[4];
  int ih0[4], iw0[4];
  bool rv[4];

  SPE_DEV void init(const GemmArgs& g, int m0, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int m = m0 + (tid >> 3) + RS * i;
      rv[i] = m < g.M;
      int mm = rv[i] ? m : 0;
      if (MODE == GEMM_CONV) {
        int hw = g.Ho * g.Wo;
        int b = mm / hw, r = mm - b * hw;
        int oh = r / g.Wo, ow = r - oh * g.Wo;
        ih0[i] = oh * g.stride - g.pad;
        iw0[i] = ow * g.stride - g.pad;
        base[i] = (const char*)g.A + (size_t)b * g.H * g.W * g.Cin * sizeof(T);
      } else {
        base[i] = (const char*)g.A + (size_t)mm * g.lda * sizeof(T);
        ih0[i] = (MODE == GEMM_LINEAR_ADD) ? (mm % g.prow) : 0;
        iw0[i] = 0;
      }
    }
  }

  SPE_DEV void load(const GemmArgs& g, int kstep, int tid, u32x4* r) const {
    constexpr int BKE = 128 / sizeof(T);
    const int k = kstep * BKE + (tid & 7) * CE;
    const bool kv = k < g.K;
    if (MODE == GEMM_CONV) {
      int kh, kw, ci;
      conv_k_decode(k, g.Cin, g.KW, g.KH * g.KW, kh, kw, ci);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int ih = ih0[i] + kh, iw = iw0[i] + kw;
        bool v = kv && rv[i] && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        r[i] = v ? ld16(base[i] + ((size_t)(ih * g.W + iw) * g.Cin + ci) * sizeof(T)) : u32x4{0, 0, 0, 0};
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool v = kv && rv[i];
        u32x4 x = v ? ld16(base[i] + (size_t)k * sizeof(T)) : u32x4{0, 0, 0, 0};
        if (MODE == GEMM_LINEAR_ADD) {
          if (v) {
            u32x4 p = ld16((const char*)g.P + ((size_t)ih0[i] * g.ldp + k) * sizeof(T));
            float fx[CE], fp[CE];
            unpack16<T>(x, fx);
            unpack16<T>(p, fp);
#pragma unroll
            for (int e = 0; e < CE; ++e) fx[e] += fp[e];
            x = pack16<T>(fx);
          }
        }
        r[i] = x;
      }
    }
  }
};

template <typename T, int NR = 4, int RS = 32>
SPE_DEV void load_b(const GemmArgs& g, int n0, int kstep, int tid, u32x4* r) {
  constexpr int BKE = 128 / sizeof(T);
  const int k = kstep * BKE + (tid & 7) * Chunk<T>::CE;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    int n = n0 + (tid >> 3) + RS * i;
    r[i] = (n < g.N) ? ld16((const char*)g.B + ((size_t)n * g.ldb + k) * sizeof(T)) : u32x4{0, 0, 0, 0};
  }
}

// split 4 fp32 into bf16 hi (returned) and lo (out) words: RNE both, lo of the exact remainder
SPE_DEV u32x2 split4(u32x4 x, u32x2& lo) {
  const f32x4 f = __builtin_bit_cast(f32x4, x);
  const uint32_t h0 = pack_bf16x2(f[0], f[1]), h1 = pack_bf16x2(f[2], f[3]);
  const float r0 = f[0] - __uint_as_float(h0 << 16), r1 = f[1] - __uint_as_float(h0 & 0xffff0000u);
  const float r2 = f[2] - __uint_as_float(h1 << 16), r3 = f[3] - __uint_as_float(h1 & 0xffff0000u);
  lo = u32x2{pack_bf16x2(r0, r1), pack_bf16x2(r2, r3)};
  return u32x2{h0, h1};
}

// X3 stage: the thread's chunk c (fp32 elements 4c..4c+3 of the K-step) -> hi piece at byte
// 8 * (c & 1) of 16-byte slot c >> 1, lo piece likewise in slot 4 + (c >> 1)
SPE_DEV void store_stage_x3(char* st, int tid, const u32x4* ra, const u32x4* rb) {
  const int c = tid & 7, half = (c & 1) * 8;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (tid >> 3) + 32 * i;
    u32x2 lo;
    u32x2 hi = split4(ra[i], lo);
    st8(st + swz(row, c >> 1) + half, hi);
    st8(st + swz(row, 4 + (c >> 1)) + half, lo);
    hi = split4(rb[i], lo);
    st8(st + BM * 128 + swz(row, c >> 1) + half, hi);
    st8(st + BM * 128 + swz(row, 4 + (c >> 1)) + half, lo);
  }
}

SPE_DEV void mma_step_x3(const char* st, int wr, int wc, int lane, f32x4 (&acc)[4][4]) {
  const int g = lane >> 4, rr = lane & 15;
  u32x4 ah[4], al[4], bh[4], bl[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wr * 64 + i * 16 + rr;
    ah[i] = ld16(st + swz(row, g));
    al[i] = ld16(st + swz(row, 4 + g));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = wc * 64 + j * 16 + rr;
    bh[j] = ld16(st + BM * 128 + swz(row, g));
    bl[j] = ld16(st + BM * 128 + swz(row, 4 + g));
  }
  auto mf = [](u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // small terms first, then the large one (each MFMA rounds its sum to fp32)
      acc[i][j] = mf(al[i], bh[j], acc[i][j]);
      acc[i][j] = mf(ah[i], bl[j], acc[i][j]);
      acc[i][j] = mf(ah[i], bh[j], acc[i][j]);
    }
}

SPE_DEV void store_stage(char* st, int tid, const u32x4* ra, const u32x4* rb) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int row = (tid >> 3) + 32 * i, c = tid & 7;
    st16(st + swz(row, c), ra[i]);
    st16(st + BM * 128 + swz(row, c), rb[i]);
  }
}

template <typename T>
SPE_DEV void mma_step(const char* st, int wr, int wc, int lane, f32x4 (&acc)[4][4]) {
  const int g = lane >> 4, rr = lane & 15;
  u32x4 a0[4], a1[4], b0[4], b1[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int row = wr * 64 + i * 16 + rr;
    a0[i] = ld16(st + swz(row, g));
    a1[i] = ld16(st + swz(row, g + 4));
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    int row = wc * 64 + j * 16 + rr;
    b0[j] = ld16(st + BM * 128 + swz(row, g));
    b1[j] = ld16(st + BM * 128 + swz(row, g + 4));
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (sizeof(T) == 2) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a0[i]),
                                                             __builtin_bit_cast(bf16x8, b0[j]), acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a1[i]),
                                                             __builtin_bit_cast(bf16x8, b1[j]), acc[i][j], 0, 0, 0);
      } else {
        f32x4 fa0 = __builtin_bit_cast(f32x4, a0[i]), fb0 = __builtin_bit_cast(f32x4, b0[j]);
        f32x4 fa1 = __builtin_bit_cast(f32x4, a1[i]), fb1 = __builtin_bit_cast(f32x4, b1[j]);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa0[s], fb0[s], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa1[s], fb1[s], acc[i][j], 0, 0, 0);
      }
    }
}

// bias / residual / activation / head-transposed or row stores of a BM_ x BN tile whose fp32
// accumulators are in LDS (ct, row stride EPI_LD), NT_ threads; bv = the thread's 8 bias values
template <typename T, int BM_, int NT_, int BN_ = BN>
SPE_DEV float store_tile(const GemmArgs& g, const float* ct, int m0, int n0, int tid, const float* bv) {
  float am = 0.f;                                  // max |stored value| (g.amax_c)
  const bool track = g.amax_c != nullptr;
  if (g.vt_T > 0) {
    // head-transposed store: column n = grp*256 + hd -> C[((grp*vt_B + b)*256 + hd)*T + tok]
    const int col = tid % BN_, n = n0 + col;
    if (n >= g.N) return am;
    const float bn = g.bias ? g.bias[n] : 0.f;
    const int grp = n >> 8, hd = n & 255;
    for (int rg = (tid / BN_) * 8; rg < BM_; rg += (NT_ / BN_) * 8) {
      const int m = m0 + rg;
      if (m >= g.M) break;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ct[(rg + e) * EPI_LD + col] + bn;
      if (track)
        for (int e = 0; e < 8 && m + e < g.M; ++e) am = fmaxf(am, fabsf(v[e]));
      const int b = m / g.vt_T, tok = m - b * g.vt_T;
      const size_t rowbase = ((size_t)(grp * g.vt_B + b) * 256 + hd) * g.vt_T;
      if constexpr (sizeof(T) == 4) {
        if (g.S) {                               // bf16 (fp16: s_f16) hi / lo planes (split attention operands)
          const size_t lo = (size_t)g.vt_B * g.N * g.vt_T;
          const float sf = g.s_f16 ? vplane_scale(g.amax_a, g.s_l1, g.s_bmax) : 1.f;
          if ((g.vt_T & 7) == 0 && m + 8 <= g.M) {   // 8 consecutive tokens of one row: two quads
            u32x2 hq[2], lq[2];
#pragma unroll
            for (int qd = 0; qd < 2; ++qd) {
              float w[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = v[4 * qd + e] * sf;
              if (g.s_f16) {
                split_f16x4(w, hq[qd], lq[qd]);
              } else {
                hq[qd] = u32x2{pack_bf16x2(w[0], w[1]), pack_bf16x2(w[2], w[3])};
                lq[qd] = u32x2{pack_bf16x2(w[0] - __uint_as_float(hq[qd].x << 16), w[1] - __uint_as_float(hq[qd].x & 0xffff0000u)),
                               pack_bf16x2(w[2] - __uint_as_float(hq[qd].y << 16), w[3] - __uint_as_float(hq[qd].y & 0xffff0000u))};
              }
              const size_t at = rowbase + (g.vt_swz ? vt_pos(tok + 4 * qd) : tok + 4 * qd);
              st8((bf16*)g.S + at, hq[qd]);
              st8((bf16*)g.S + lo + at, lq[qd]);
            }
            continue;
          }
          for (int e = 0; e < 8 && m + e < g.M; ++e) {
            const int me = m + e, be = me / g.vt_T, te = me - be * g.vt_T;
            const size_t idx = ((size_t)(grp * g.vt_B + be) * 256 + hd) * g.vt_T + (g.vt_swz ? vt_pos(te) : te);
            const float w = v[e] * sf;
            if (g.s_f16) {
              const f16 h = (f16)w;
              ((f16*)g.S)[idx] = h;
              ((f16*)g.S)[lo + idx] = (f16)(w - (float)h);
            } else {
              const bf16 h = from_f32<bf16>(w);
              ((bf16*)g.S)[idx] = h;
              ((bf16*)g.S)[lo + idx] = from_f32<bf16>(w - to_f32(h));
            }
          }
          continue;
        }
      }
      if ((g.vt_T & 7) == 0 && m + 8 <= g.M) {
        char* cp = (char*)g.C + (rowbase + tok) * sizeof(T);
        if constexpr (sizeof(T) == 2) {
          const u32x4 pk = pack_out8(v, g.out_f16);
          if (g.vt_swz) {                        // the two quads land apart (vt_pos)
            st8((char*)g.C + (rowbase + vt_pos(tok)) * 2, u32x2{pk.x, pk.y});
            st8((char*)g.C + (rowbase + vt_pos(tok + 4)) * 2, u32x2{pk.z, pk.w});
          } else {
            st16(cp, pk);
          }
        } else {
          st16(cp, pack16<T>(v));
          st16(cp + 16, pack16<T>(v + 4));
        }
      } else {
        for (int e = 0; e < 8 && m + e < g.M; ++e) {
          const int me = m + e, be = me / g.vt_T, te = me - be * g.vt_T;
          const size_t idx = ((size_t)(grp * g.vt_B + be) * 256 + hd) * g.vt_T + (g.vt_swz ? vt_pos(te) : te);
          if constexpr (sizeof(T) == 2) store_out1(g.C, idx, v[e], g.out_f16);
          else ((T*)g.C)[idx] = from_f32<T>(v[e]);
        }
      }
    }
    return am;
  }

  constexpr int CG = BN_ / 8;                       // 8-column groups per row
  const int cg = (tid % CG) * 8;
  const int n = n0 + cg;
  if (n >= g.N) return am;
  const bool full = n + 8 <= g.N;
  for (int rr = tid / CG; rr < BM_; rr += NT_ / CG) {
    const int m = m0 + rr;
    if (m >= g.M) break;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ct[rr * EPI_LD + cg + e] + bv[e];
    auto add_res = [&]() {                         // residual, or row-periodic add (pos . W^T)
      const T* rp = (const T*)g.R + (size_t)(g.r_period > 0 ? m % g.r_period : m) * g.ldr + n;
      if (full) {
        float f[8];
        unpack16<T>(ld16(rp), f);
        if constexpr (sizeof(T) == 4) unpack16<T>(ld16(rp + 4), f + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += f[e];
      } else {
        for (int e = 0; e < 8 && n + e < g.N; ++e) v[e] += to_f32(rp[e]);
      }
    };
    if (g.R && !g.res_post) add_res();
    if (g.act) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], g.act);
    }
    if (g.R && g.res_post) add_res();
    if (track)
      for (int e = 0; e < 8 && n + e < g.N; ++e) am = fmaxf(am, fabsf(v[e]));
    if constexpr (sizeof(T) == 4) {
      if (g.S && n >= g.s_col0) {                // bf16 hi / lo planes (fp32x3 attention operands)
        const int ns = g.N - g.s_col0;
        bf16* hp = (bf16*)g.S + (size_t)m * ns + (n - g.s_col0);
        bf16* lp = hp + (size_t)g.M * ns;
        float hv[8], lv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          hv[e] = to_f32(from_f32<bf16>(v[e]));
          lv[e] = v[e] - hv[e];
        }
        if (full) {
          st16(hp, pack16<bf16>(hv));
          st16(lp, pack16<bf16>(lv));
        } else {
          for (int e = 0; e < 8 && n + e < g.N; ++e) {
            hp[e] = from_f32<bf16>(hv[e]);
            lp[e] = from_f32<bf16>(lv[e]);
          }
        }
        continue;
      }
    }
    if (g.out_f32) {
      float* cp = (float*)g.C + (size_t)m * g.ldc + n;
      if (full) {
        st16(cp, pack16<float>(v));
        st16(cp + 4, pack16<float>(v + 4));
      } else {
        for (int e = 0; e < 8 && n + e < g.N; ++e) cp[e] = v[e];
      }
    } else {
      T* cp = (T*)g.C + (size_t)m * g.ldc + n;
      if (full) {
        if constexpr (sizeof(T) == 2) {
          st16(cp, pack_out8(v, g.out_f16));
        } else {
          st16(cp, pack16<T>(v));
          st16(cp + 4, pack16<T>(v + 4));
        }
      } else {
        for (int e = 0; e < 8 && n + e < g.N; ++e) {
          if constexpr (sizeof(T) == 2) store_out1(cp, e, v[e], g.out_f16);
          else cp[e] = from_f32<T>(v[e]);
        }
      }
    }
  }
  return am;
}

// one atomic max per wave of the lanes' |value| maxima (all lanes of the wave active); float bits
// compare as uint for values >= 0
SPE_DEV void amax_publish(float am, float* slot, float mul) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  if ((threadIdx.x & 63) == 0 && am > 0.f) amax_update(slot, am * (mul > 0.f ? mul : 1.f));
}

template <typename T, int MODE, bool X3 = false>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tilesN = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BN;
  constexpr int BKE = 128 / sizeof(T);
  const int nk = (g.K + BKE - 1) / BKE;

  ALoader<T, MODE> al;
  al.init(g, m0, tid);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // epilogue bias, fetched before the K loop (in the epilogue it would add an HBM round trip)
  float bv[8];
  {
    const int n = n0 + (tid & 15) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (g.bias && n + e < g.N) ? g.bias[n + e] : 0.f;
  }

  u32x4 ra[4], rb[4];
  auto stage = [&](char* st) {
    if constexpr (X3) store_stage_x3(st, tid, ra, rb);
    else store_stage(st, tid, ra, rb);
  };
  al.load(g, 0, tid, ra);
  load_b<T>(g, n0, 0, tid, rb);
  stage(smem);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) {
      al.load(g, ks + 1, tid, ra);
      load_b<T>(g, n0, ks + 1, tid, rb);
    }
    if constexpr (X3) mma_step_x3(smem + (ks & 1) * STAGE_BYTES, wr, wc, lane, acc);
    else mma_step<T>(smem + (ks & 1) * STAGE_BYTES, wr, wc, lane, acc);
    if (more) stage(smem + ((ks + 1) & 1) * STAGE_BYTES);
    __syncthreads();
  }

  // ---- epilogue: accumulators -> LDS fp32 tile -> fused bias/residual/ReLU -> wide stores
  float* ct = reinterpret_cast<float*>(smem);
  {
    const int q = lane >> 4, c = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(wr * 64 + i * 16 + q * 4 + r) * EPI_LD + wc * 64 + j * 16 + c] = acc[i][j][r];
  }
  __syncthreads();

  const float am = store_tile<T, BM, NT>(g, ct, m0, n0, tid, bv);
  if (g.amax_c) amax_publish(am, g.amax_c, g.amax_c_mul);
}

// ------------------------------------------------------------------ fp32x6 (near-fp32) kernel
// fp32 operands split while staged into three bf16 planes, x = h + m + l (h = bf16(x),
// m = bf16(x - h), l = bf16(x - h - m); both remainders exact in fp32, x - h - m - l within 2^-24
// of |x|), every fragment product as the six terms of relative order >= 2^-16 --
// l.h + h.l + m.m + m.h + h.m + h.h, small terms first -- on mfma_f32_16x16x32_bf16 with fp32
// accumulation: the product error is that of an fp32 FMA chain (~2^-24) at six bf16 MFMAs, i.e.
// 2.65x the fp32 MFMA ceiling (417 vs 157 TFLOP/s).  One 32-element K-step per stage: planes
// [3][rows][64 B] with the 16-byte chunk XOR-swizzled by row bits 2-3 (conflict-free ds_read_b128
// for the 16 rows of a fragment); waves of 64 x 64 output.  Two tile geometries (X6Geo):
//   BM 256: 8 waves, two stages (144 KiB) so the next step's loads and split overlap this step's
//           MFMAs, one workgroup per CU;
//   BM 128: 4 waves, one stage (48 KiB, 66 KiB with the epilogue tile) and two barriers per step,
//           two workgroups per CU whose phases interleave (one splits while the other multiplies).
constexpr int BN6 = 128;
template <int BM_> struct X6Geo {
  static constexpr int BM = BM_, NT = BM_ * 2, STAGES = BM_ == 256 ? 2 : 1, RS = NT / 8;
  static constexpr int PLANE_A = BM * 64, PLANE_B = BN6 * 64;
  static constexpr int STAGE = 3 * (PLANE_A + PLANE_B);
  static constexpr int SMEM = (STAGES * STAGE > BM * EPI_LD * 4) ? STAGES * STAGE : BM * EPI_LD * 4;
};
constexpr int BM6 = 256;                 // the launcher's tile-count heuristic (few-row problems)

// gfx950 serves a wave's ds_read_b128 in four lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}
// and the same + 32; MI355X_MICROARCH.md, LDS): a fragment read (lane l -> row l & 15, chunk
// l >> 4) puts rows 0-3, 12-15 of chunk g and rows 4-11 of chunk g ^ 1 in one group, so the chunk
// is XORed with (0, 3, 2, 1)[row bits 2-3] -- the 16 lanes of every group hit 16 distinct 16-byte
// slots of a 256-byte bank row
SPE_DEV int swz6(int row, int chunk) { return row * 64 + ((chunk ^ ((4 - ((row >> 2) & 3)) & 3)) << 4); }

// 4 fp32 -> bf16 planes h, m, l (4 values each, RNE; remainders exact)
SPE_DEV void split3(u32x4 x, u32x2& h, u32x2& m, u32x2& l) {
  const f32x4 f = __builtin_bit_cast(f32x4, x);
  const uint32_t h0 = pack_bf16x2(f[0], f[1]), h1 = pack_bf16x2(f[2], f[3]);
  const float r0 = f[0] - __uint_as_float(h0 << 16), r1 = f[1] - __uint_as_float(h0 & 0xffff0000u);
  const float r2 = f[2] - __uint_as_float(h1 << 16), r3 = f[3] - __uint_as_float(h1 & 0xffff0000u);
  const uint32_t m0 = pack_bf16x2(r0, r1), m1 = pack_bf16x2(r2, r3);
  const float s0 = r0 - __uint_as_float(m0 << 16), s1 = r1 - __uint_as_float(m0 & 0xffff0000u);
  const float s2 = r2 - __uint_as_float(m1 << 16), s3 = r3 - __uint_as_float(m1 & 0xffff0000u);
  h = u32x2{h0, h1};
  m = u32x2{m0, m1};
  l = u32x2{pack_bf16x2(s0, s1), pack_bf16x2(s2, s3)};
}

// the thread's fp32 chunk c4 (elements 4 c4 .. 4 c4 + 3 of the K-step) of `rows` rows RS apart
// -> 8-byte pieces of bf16 chunk c4 >> 1 in each plane
template <int NR, int RS, int PLANE>
SPE_DEV void store_split6(char* st, int tid, const u32x4* r) {
  const int c4 = tid & 7, half = (c4 & 1) * 8;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int row = (tid >> 3) + RS * i;
    u32x2 h, m, l;
    split3(r[i], h, m, l);
    const int o = swz6(row, c4 >> 1) + half;
    st8(st + o, h);
    st8(st + PLANE + o, m);
    st8(st + 2 * PLANE + o, l);
  }
}

template <typename G>
SPE_DEV void mma_step_x6(const char* st, int wr, int wc, int lane, f32x4 (&acc)[4][4]) {
  const int g = lane >> 4, rr = lane & 15;
  const char* sa = st;
  const char* sb = st + 3 * G::PLANE_A;
  // the B fragments (3 planes x 4) stay live across the step; A is read one 16-row block (3
  // planes) at a time, which keeps the two-ahead load registers of the caller spill-free
  u32x4 b[3][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o = swz6(wc * 64 + j * 16 + rr, g);
#pragma unroll
    for (int p = 0; p < 3; ++p) b[p][j] = ld16(sb + p * G::PLANE_B + o);
  }
  auto mf = [](u32x4 x, u32x4 y, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y), c, 0, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    u32x4 a[3];
    const int o = swz6(wr * 64 + i * 16 + rr, g);
#pragma unroll
    for (int p = 0; p < 3; ++p) a[p] = ld16(sa + p * G::PLANE_A + o);
    // one accumulator's six products back to back, small terms first (l.h, h.l, m.m, m.h, h.m,
    // h.h); measured faster than advancing the four accumulators of the block together
    // (product-major: FFN1 1.15 -> 1.27 ms, layer-1 3x3 0.58 -> 0.76 ms)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 c = acc[i][j];
      c = mf(a[2], b[0][j], c);
      c = mf(a[0], b[2][j], c);
      c = mf(a[1], b[1][j], c);
      c = mf(a[1], b[0][j], c);
      c = mf(a[0], b[1][j], c);
      acc[i][j] = mf(a[0], b[0][j], c);
    }
  }
}

// BP: the weights arrive pre-split (GemmArgs::B6, bf16 planes [3][N][ldb] written at finalize):
// 16-byte chunks per plane, no split work for the B tile
template <int MODE, bool BP, int BMX>
__global__ __launch_bounds__(X6Geo<BMX>::NT, BMX == 256 ? 1 : 2) void gemm_x6_kernel(GemmArgs g) {
  using G = X6Geo<BMX>;
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int tilesN = (g.N + BN6 - 1) / BN6;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tilesN) * G::BM, n0 = (t % tilesN) * BN6;
  const int nk = (g.K + 31) / 32;

  ALoader<float, MODE, G::RS> al;
  al.init(g, m0, tid);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // B tile: BP -- rows tid >> 2 (+ NT/4 per pass), 16-byte chunk tid & 3 of the step's 64 bytes,
  // in each plane; split path -- fp32 chunks as the A loader
  constexpr int BPASS = BN6 / (G::NT / 4);              // 1 (BM 256) or 2 (BM 128) rows per thread
  constexpr int NRB = BP ? 3 * BPASS : BN6 / G::RS;
  const int brow = tid >> 2, bch = tid & 3;
  const size_t pstride = (size_t)g.b6_rows * g.ldb;
  // one K-step's raw operands in registers: A fp32 chunks, B fp32 chunks or bf16 plane chunks
  auto load = [&](u32x4* ra, u32x4* rb, int kstep) {
    al.load(g, kstep, tid, ra);
    if constexpr (BP) {
#pragma unroll
      for (int i = 0; i < BPASS; ++i) {
        const int n = n0 + brow + i * (G::NT / 4);
        const char* src = (const char*)g.B6 + ((size_t)(n < g.N ? n : 0) * g.ldb + bch * 8 + (size_t)kstep * 32) * 2;
#pragma unroll
        for (int p = 0; p < 3; ++p) rb[3 * i + p] = n < g.N ? ld16(src + p * pstride * 2) : u32x4{0, 0, 0, 0};
      }
    } else {
      load_b<float, NRB, G::RS>(g, n0, kstep, tid, rb);
    }
  };
  auto stage = [&](char* st, const u32x4* ra, const u32x4* rb) {
    store_split6<4, G::RS, G::PLANE_A>(st, tid, ra);
    if constexpr (BP) {
#pragma unroll
      for (int i = 0; i < BPASS; ++i) {
        char* sb = st + 3 * G::PLANE_A + swz6(brow + i * (G::NT / 4), bch);
#pragma unroll
        for (int p = 0; p < 3; ++p) st16(sb + p * G::PLANE_B, rb[3 * i + p]);
      }
    } else {
      store_split6<NRB, G::RS, G::PLANE_B>(st + 3 * G::PLANE_A, tid, rb);
    }
  };
  if constexpr (G::STAGES == 2) {
    // loads run two K-steps ahead in two register sets (X, Y), so a step's split never waits on
    // the loads issued in that step; past the end the last step is re-loaded (every path issues
    // the same loads, which keeps the compiler's vmcnt waits counted instead of vmcnt(0))
    u32x4 xa[4], xb[NRB], ya[4], yb[NRB];
    const int last = nk - 1;
    load(xa, xb, 0);
    stage(smem, xa, xb);
    load(xa, xb, nk > 1 ? 1 : last);
    load(ya, yb, nk > 2 ? 2 : last);
    __syncthreads();
    for (int ks = 0; ks < nk; ks += 2) {
      mma_step_x6<G>(smem, wr, wc, lane, acc);                         // step ks (stage 0)
      if (ks + 1 < nk) stage(smem + G::STAGE, xa, xb);                 // step ks + 1
      load(xa, xb, ks + 3 < nk ? ks + 3 : last);
      __syncthreads();
      if (ks + 1 >= nk) break;
      mma_step_x6<G>(smem + G::STAGE, wr, wc, lane, acc);              // step ks + 1 (stage 1)
      if (ks + 2 < nk) stage(smem, ya, yb);                            // step ks + 2
      load(ya, yb, ks + 4 < nk ? ks + 4 : last);
      __syncthreads();
    }
  } else {
    u32x4 ra[4], rb[NRB];
    load(ra, rb, 0);
    for (int ks = 0; ks < nk; ++ks) {
      stage(smem, ra, rb);          // the previous step's reads are behind the loop-end barrier
      __syncthreads();
      if (ks + 1 < nk) load(ra, rb, ks + 1);
      mma_step_x6<G>(smem, wr, wc, lane, acc);
      __syncthreads();
    }
  }

  float bv[8];                      // (fetched after the K loop: its registers are the loop's)
  {
    const int n = n0 + (tid & 15) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (g.bias && n + e < g.N) ? g.bias[n + e] : 0.f;
  }
  float* ct = reinterpret_cast<float*>(smem);
  {
    const int q = lane >> 4, c = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          ct[(wr * 64 + i * 16 + q * 4 + r) * EPI_LD + wc * 64 + j * 16 + c] = acc[i][j][r];
  }
  __syncthreads();
  const float am = store_tile<float, G::BM, G::NT>(g, ct, m0, n0, tid, bv);
  if (g.amax_c) amax_publish(am, g.amax_c, g.amax_c_mul);
}

template <int BMX>
int launch_x6_geo(const GemmArgs& g, int mode, hipStream_t s) {
  const int tiles = ((g.M + BMX - 1) / BMX) * ((g.N + BN6 - 1) / BN6);
  if (tiles <= 0) return 0;
  dim3 grid(tiles), block(X6Geo<BMX>::NT);
  const bool bp = g.B6 != nullptr;
  switch (mode * 2 + bp) {
    case GEMM_LINEAR * 2: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_LINEAR, false, BMX>), grid, block, 0, s, g); break;
    case GEMM_LINEAR * 2 + 1: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_LINEAR, true, BMX>), grid, block, 0, s, g); break;
    case GEMM_LINEAR_ADD * 2: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_LINEAR_ADD, false, BMX>), grid, block, 0, s, g); break;
    case GEMM_LINEAR_ADD * 2 + 1: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_LINEAR_ADD, true, BMX>), grid, block, 0, s, g); break;
    case GEMM_CONV * 2: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_CONV, false, BMX>), grid, block, 0, s, g); break;
    case GEMM_CONV * 2 + 1: hipLaunchKernelGGL((gemm_x6_kernel<GEMM_CONV, true, BMX>), grid, block, 0, s, g); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// tile geometry: SPE_X6_TILE = 128 (default: 3-9 % faster than 256 across the bench shapes,
// scripts/x6_bench.py) or 256
int launch_x6(const GemmArgs& g, int mode, hipStream_t s) {
  static const int tile = [] { const char* e = getenv("SPE_X6_TILE"); return e ? atoi(e) : 128; }();
  return tile == 128 ? launch_x6_geo<128>(g, mode, s) : launch_x6_geo<256>(g, mode, s);
}

// ---------------------------------------------------------------- fp32x6, LDS-DMA staged
// The same six-product split as gemm_x6_kernel, restaged: both operands go global -> LDS by
// buffer_load ... lds (no staging registers, no ds_write, no per-step wait on loads issued in
// that step) -- A as raw fp32, split into its h / m / l planes by the waves that read the
// fragments; B from the pre-split weight planes (GemmArgs::B6).  One barrier per K-step (32
// elements); the DMA of step ks+1 is issued right behind step ks's barrier into the other stage
// and has all of step ks's MFMAs to land.  v_mfma_f32_32x32x16_bf16 fragments, FI x 2 per wave
// of (32 FI) x 64: tile 128 x 128 (FI = 2, 2 x 2 waves) or 128 x 64 (FI = 1, 4 x 1 waves, for the
// N = 64 convs of layer 1 that a 128-wide tile would compute half empty).  Per step and wave
// 24 FI MFMAs, 4 FI A reads (2 x 16 B per 8-element fragment row) + 12 B plane reads, 16 FI fp32
// split.
//   LDS stage: A [128 rows][128 B] fp32, chunk c of row r at slot c ^ ((r >> 1) & 7);
//   B planes [3][BN rows][64 B] bf16, chunk c at slot c ^ ((r >> 2) & 3) -- both keyed for
//   gfx950's ds_read_b128 lane groups under the 32x32 fragment's lane -> row map (lane & 31),
//   applied on the DMA source address.  Two stages (80 / 56 KiB) = two workgroups per CU.
// Used for GEMM_LINEAR and GEMM_CONV with K % 32 == 0 (Cin % 32 == 0), pre-split weights and
// 32-bit buffer offsets; everything else takes gemm_x6_kernel.
constexpr int D6_BM = 128, D6_NT = 256, D6_A = D6_BM * 128;
template <int FI> struct D6Geo {
  static constexpr int WN = FI, WM = 4 / WN, BN = 64 * WN;
  static constexpr int PB = BN * 64, STAGE = D6_A + 3 * PB;
  static constexpr int NBQ = 3 * BN / 64;              // B DMA pieces per wave per step
  static constexpr int SMEM = 2 * STAGE > D6_BM * EPI_LD * 4 ? 2 * STAGE : D6_BM * EPI_LD * 4;
  static constexpr int NQ = 12 * FI;                   // MFMAs per fragment set
};
constexpr int D6_BAD = 0x7ffffff0;          // out-of-range buffer offset -> zeros
typedef __attribute__((address_space(3))) void* lds_ptr6_t;
constexpr int d6_waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }  // vmcnt(n) only
constexpr int d6_waitcnt_vm0() { return d6_waitcnt_vm(0); }

SPE_DEV u32x4 cat2(u32x2 a, u32x2 b) { return u32x4{a.x, a.y, b.x, b.y}; }

// One 16-element half kk of a stage = one fragment set: the B planes b[p][j], and per A
// fragment row i the two 16-byte fp32 reads (halves h) split into 8-byte plane pieces.
// (namespace scope: a kernel-local class depending on the template parameter lost the
// kernel's host stub)
template <int FI> struct D6Frag {
  u32x4 b[3][2];
  u32x4 raw[FI][2];
  u32x2 ph[FI][2], pm[FI][2], pl[FI][2];
};

// PL (GEMM_CONV, Cin % 32 != 0, e.g. the stem's 4- or 8-channel input): a 32-element K-step
// spans several taps, so each lane decodes its own chunk's (kh, kw, ci) per step, and chunks past
// K read zeros (K need not be a multiple of 32)
template <int MODE, int FI, bool PL = false>
__device__ __forceinline__ void gemm_x6d_body(const GemmArgs& g) {
  using G = D6Geo<FI>;
  constexpr int D6_BN = G::BN, D6_PB = G::PB, D6_STAGE = G::STAGE, NBQ = G::NBQ, NQ = G::NQ;
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / G::WN, wc = wid % G::WN;
  const int tilesN = (g.N + D6_BN - 1) / D6_BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tilesN) * D6_BM, n0 = (t % tilesN) * D6_BN;
  const int nk = (g.K + 31) >> 5;
  const long long abytes = MODE == GEMM_CONV ? (long long)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 4
                                             : (long long)g.M * g.lda * 4;
  const size_t pstride = (size_t)g.b6_rows * g.ldb;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B6, (short)0, (int)(3 * pstride * 2), 0x00020000);

  // ---- DMA pieces of this wave: A pieces wid + 4q (rows 8p .. 8p+7, lane -> row 8p + lane/8,
  // slot lane & 7), B pieces wid + 4q (plane p / 8, rows 16 (p % 8) + lane/4, slot lane & 3)
  int avo[4], ih0[4], iw0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (wid + 4 * q) * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7), m = m0 + row;
    if constexpr (MODE == GEMM_CONV) {
      const int hw = g.Ho * g.Wo, mm = m < g.M ? m : 0;
      const int b = mm / hw, r = mm - b * hw, oh = r / g.Wo, ow = r - oh * g.Wo;
      ih0[q] = m < g.M ? oh * g.stride - g.pad : -(1 << 28);
      iw0[q] = ow * g.stride - g.pad;
      avo[q] = b * g.H * g.W * g.Cin + (PL ? 0 : c * 4);   // elements: image base (+ the lane's chunk)
    } else {
      avo[q] = m < g.M ? m * g.lda * 4 + c * 16 : D6_BAD;
      ih0[q] = iw0[q] = 0;
    }
  }
  int bvo[NBQ];
#pragma unroll
  for (int q = 0; q < NBQ; ++q) {
    const int p = wid + 4 * q, plane = p / (D6_BN / 16), row = (p % (D6_BN / 16)) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3), n = n0 + row;
    bvo[q] = n < g.N ? (int)((plane * pstride + (size_t)n * g.ldb) * 2) + c * 16 : D6_BAD;
  }
  // the lane's A chunk column: (lane & 7) ^ ((row >> 1) & 7) is the same for all four pieces
  const int ck = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
  auto issue = [&](int ks, int stg) {
    char* base = smem + stg * D6_STAGE;
    int kh = 0, kw = 0, ci = 0;
    bool kv = true;
    if constexpr (MODE == GEMM_CONV) {
      if constexpr (PL) {
        const int k = ks * 32 + ck * 4, tap = k / g.Cin;
        ci = k - tap * g.Cin;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
        kv = k < g.K;
      } else {
        conv_k_decode(ks * 32, g.Cin, g.KW, g.KH * g.KW, kh, kw, ci);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int off;
      if constexpr (MODE == GEMM_CONV) {
        const int ih = ih0[q] + kh, iw = iw0[q] + kw;
        const bool v = kv && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        off = v ? (avo[q] + (ih * g.W + iw) * g.Cin + ci) * 4 : D6_BAD;
      } else {
        off = avo[q];
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr6_t)(base + (wid + 4 * q) * 1024), 16, off,
                                               MODE == GEMM_CONV ? 0 : ks * 128, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NBQ; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr6_t)(base + D6_A + (wid + 4 * q) * 1024), 16, bvo[q],
                                               ks * 64, 0, 0);
  };

  // ---- fragment offsets: A row wr*32FI + 32i + (lane & 31), 16-byte chunks 4kk + 2(lane >> 5) + h;
  // B row wc*64 + 32j + (lane & 31), chunk 2kk + (lane >> 5)
  const int l31 = lane & 31, hi = lane >> 5;
  int aoff[2][2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      aoff[kk][h] = (wr * 32 * FI + l31) * 128 + (((4 * kk + 2 * hi + h) ^ ((l31 >> 1) & 7)) << 4);
    boff[kk] = D6_A + (wc * 64 + l31) * 64 + (((2 * kk + hi) ^ ((l31 >> 2) & 3)) << 4);
  }
  auto mf = [](u32x4 x, u32x4 y, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y), c, 0, 0, 0);
  };
  f32x16 acc[FI][2];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  using Frag = D6Frag<FI>;
  auto read_b = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int p = 0; p < 3; ++p) f.b[p][j] = ld16(st + boff[kk] + p * D6_PB + j * 2048);
  };
  auto read_a = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) f.raw[i][h] = ld16(st + aoff[kk][h] + i * 4096);
  };
  auto split_a = [&](Frag& f, int i, int h) { split3(f.raw[i][h], f.ph[i][h], f.pm[i][h], f.pl[i][h]); };
  // MFMA number q (0 .. NQ-1) of a set: accumulator q / 6, product q % 6 (l.h, h.l, m.m, m.h, h.m, h.h)
  auto mma1 = [&](const Frag& f, int q) {
    const int a = q / 6, i = a >> 1, j = a & 1, t = q % 6;
    const u32x4 ah = cat2(f.ph[i][0], f.ph[i][1]), am = cat2(f.pm[i][0], f.pm[i][1]), al = cat2(f.pl[i][0], f.pl[i][1]);
    const u32x4 xa = t == 0 ? al : (t == 1 || t == 4 || t == 5) ? ah : am;
    const u32x4 xb = (t == 0 || t == 3 || t == 5) ? f.b[0][j] : t == 1 ? f.b[2][j] : f.b[1][j];
    acc[i][j] = mf(xa, xb, acc[i][j]);
  };
#define D6_MMA(F, LO, HI)                                \
  _Pragma("unroll") for (int q = LO; q < HI; ++q) mma1(F, q); \
  __builtin_amdgcn_sched_barrier(0);

  // Software pipeline over K-step halves: X = the kk = 0 fragments, Y = kk = 1.  Phase A of step
  // ks multiplies X while Y is read and split from the same stage; then every wave's reads of
  // that stage are done and step ks+1's DMA has landed (issued a whole step earlier), so one
  // barrier frees the stage for step ks+2's DMA; phase B multiplies Y while step ks+1's X is read
  // and split from the other stage.  The loop body has no branches (past the last step the DMA
  // and reads fetch in-bounds or zeroed bytes nobody uses) and is pinned in chunks
  // (sched_barrier): the DS reads and DMA issues beside the first MFMAs, one split3 (4 values,
  // ~18 VALU) per 3 MFMAs -- the 24 free issue cycles of each 32-cycle MFMA.
  issue(0, 0);
  issue(1, 1);
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm(4 + NBQ));        // step 0's pieces (step 1's in flight)
  __syncthreads();
  Frag X, Y;
  read_b(smem, 0, X);
  read_a(smem, 0, X);
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h) split_a(X, i, h);
  constexpr int QA = NQ / 4, QB = 3 + NQ / 4;          // MFMAs before the first split of each phase
  for (int ks = 0; ks < nk; ++ks) {
    const char* st = smem + (ks & 1) * D6_STAGE;
    const char* sn = smem + ((ks + 1) & 1) * D6_STAGE;
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase A: X's MFMAs, Y read + split
    read_b(st, 1, Y);
    read_a(st, 1, Y);
    D6_MMA(X, 0, QA)
#pragma unroll
    for (int sp = 0; sp < 2 * FI; ++sp) {
      split_a(Y, sp >> 1, sp & 1);
      D6_MMA(X, QA + 3 * sp, QA + 3 * sp + 3)
    }
    D6_MMA(X, QA + 6 * FI, NQ)
    __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm0() & ~(15 << 8));  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase B: Y's MFMAs, step ks+2's DMA, step ks+1's X read + split
    issue(ks + 2, ks & 1);
    D6_MMA(Y, 0, 3)
    read_b(sn, 0, X);
    read_a(sn, 0, X);
    D6_MMA(Y, 3, QB)
#pragma unroll
    for (int sp = 0; sp < 2 * FI; ++sp) {
      split_a(X, sp >> 1, sp & 1);
      D6_MMA(Y, QB + 3 * sp, QB + 3 * sp + 3)
    }
    D6_MMA(Y, QB + 6 * FI, NQ)
  }
#undef D6_MMA
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm0());              // the past-the-end DMA, before the stages are reused
  __syncthreads();                                           // stages -> epilogue tile

  float bv[8];
  {
    const int n = n0 + (tid % (D6_BN / 8)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (g.bias && n + e < g.N) ? g.bias[n + e] : 0.f;
  }
  float* ct = reinterpret_cast<float*>(smem);
  // 32x32 accumulator: lane holds rows 8 (r >> 2) + 4 (lane >> 5) + (r & 3), column lane & 31
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        ct[(wr * 32 * FI + 32 * i + 8 * (r >> 2) + 4 * hi + (r & 3)) * EPI_LD + wc * 64 + 32 * j + l31] = acc[i][j][r];
  __syncthreads();
  const float am = store_tile<float, D6_BM, D6_NT, D6_BN>(g, ct, m0, n0, tid, bv);
  if (g.amax_c) amax_publish(am, g.amax_c, g.amax_c_mul);
}

// (non-template entry points: the host stubs of a template of this body were not emitted)
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_linear(GemmArgs g) { gemm_x6d_body<GEMM_LINEAR, 2>(g); }
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_linear_n64(GemmArgs g) { gemm_x6d_body<GEMM_LINEAR, 1>(g); }
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_conv(GemmArgs g) { gemm_x6d_body<GEMM_CONV, 2>(g); }
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_conv_n64(GemmArgs g) { gemm_x6d_body<GEMM_CONV, 1>(g); }
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_conv_pl(GemmArgs g) { gemm_x6d_body<GEMM_CONV, 2, true>(g); }
__global__ __launch_bounds__(D6_NT, 2) void gemm_x6d_conv_pl_n64(GemmArgs g) { gemm_x6d_body<GEMM_CONV, 1, true>(g); }

// 1 = not a problem for the DMA kernel
int launch_x6d(const GemmArgs& g, int mode, hipStream_t s) {
  static const int en = [] { const char* e = getenv("SPE_X6_DMA"); return e ? atoi(e) : 1; }();
  if (!en || !g.B6 || (mode != GEMM_LINEAR && mode != GEMM_CONV) || (g.lda & 3)) return 1;
  const bool pl = mode == GEMM_CONV && (g.Cin & 31);      // per-lane tap decode (stem)
  if (pl ? ((g.Cin & 3) || (g.K & 3) || g.K != g.Cin * g.KH * g.KW) : (g.K & 31)) return 1;
  if ((reinterpret_cast<uintptr_t>(g.A) & 15) || (reinterpret_cast<uintptr_t>(g.B6) & 15) || (g.ldb & 7)) return 1;
  constexpr long long LIM = (1LL << 31) - (1LL << 24);
  if ((long long)3 * g.b6_rows * g.ldb * 2 >= LIM || g.b6_rows < g.N) return 1;
  if (mode == GEMM_CONV) {
    if ((long long)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 4 >= LIM) return 1;
  } else if ((long long)(g.M + D6_BM) * g.lda * 4 + (long long)g.K * 4 >= LIM) {
    return 1;
  }
  // N <= 64: the 128 x 64 tile (SPE_X6_N64=0 keeps 128 x 128)
  static const int n64 = [] { const char* e = getenv("SPE_X6_N64"); return e ? atoi(e) : 1; }();
  const bool narrow = n64 && g.N <= 64;
  const int bn = narrow ? 64 : 128;
  const int tiles = ((g.M + D6_BM - 1) / D6_BM) * ((g.N + bn - 1) / bn);
  if (tiles <= 0) return 0;
  const dim3 grid(tiles), block(D6_NT);
  if (mode == GEMM_CONV && pl) {
    if (narrow) hipLaunchKernelGGL(gemm_x6d_conv_pl_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_x6d_conv_pl, grid, block, 0, s, g);
  } else if (mode == GEMM_CONV) {
    if (narrow) hipLaunchKernelGGL(gemm_x6d_conv_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_x6d_conv, grid, block, 0, s, g);
  } else {
    if (narrow) hipLaunchKernelGGL(gemm_x6d_linear_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_x6d_linear, grid, block, 0, s, g);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- fp32h3, LDS-DMA staged
// fp32 operands at near-fp32 precision on HALF the x6 kernel's MFMAs: fp16 carries 11 significand
// bits against bf16's 8, so a two-way split x.s = hi + lo (fp16 RNE each, the remainder exact in
// fp32) represents x to ~2^-22 -- bf16's three-way split to ~2^-24 -- and the three products
// lo.hi + hi.lo + hi.hi (small first) on v_mfma_f32_32x32x16_f16 (the bf16 rate) give an fp32-level
// product.  fp16's range needs scales, powers of two so they cost no precision: the weights are
// split at finalize per output channel (h3_sinv[n] = 2^-e_n undoes it), the activations per tensor
// from max |A| (amax_a, published by the producing launch: 2^13 / amax rounded down to a power of
// two puts the tensor's largest element in [2^12, 2^13), so hi <= 65504 always and a value 2^-36 of
// the maximum still splits to fp32 accuracy).  oracle/study_split_precision.py: this scheme moves
// the bench weights' keypoints 2.2e-5 from exact fp32, the x6 scheme 2.2e-5, fp32x3 3.9e-4.
// Geometry: 4 waves stacked in M, wave tile 32 x 32 FJ (FJ = 4: 128 x 128, FJ = 2: 128 x 64 for N <= 64),
// so every A row is split by exactly one wave (the x6 kernel's 2 x 2 waves split each row twice);
// per K-step (32) and wave 6 FJ MFMAs, 16 fp32 values split per lane.  LDS stage: A [128][128 B]
// fp32 (chunk c of row r at slot c ^ ((r >> 1) & 7)) + B planes [2][BN][64 B] fp16 (chunk c at
// c ^ ((r >> 2) & 3)), both by buffer_load ... lds with the swizzle on the source address; two
// stages + one barrier per step; the same pinned two-phase pipeline as gemm_x6d_body.
constexpr int H3_BM = 128, H3_NT = 256, H3_A = H3_BM * 128;
template <int FJ> struct H3Geo {
  static constexpr int BN = 32 * FJ;
  static constexpr int PB = BN * 64, STAGE = H3_A + 2 * PB;
  static constexpr int NBQ = 2 * BN / 64;              // B DMA pieces per wave per step
  static constexpr int SMEM = 2 * STAGE > H3_BM * EPI_LD * 4 ? 2 * STAGE : H3_BM * EPI_LD * 4;
  static constexpr int NQ = 3 * FJ;                    // MFMAs per fragment set (K-step half)
};

// 4 fp32 -> (x s) fp16 planes hi, lo (4 values each)
SPE_DEV void split2h(u32x4 x, float sc, u32x2& h, u32x2& l) {
  const f32x4 f = __builtin_bit_cast(f32x4, x) * sc;
  const f16x2 h0 = __builtin_convertvector((f32x2){f[0], f[1]}, f16x2);
  const f16x2 h1 = __builtin_convertvector((f32x2){f[2], f[3]}, f16x2);
  const f32x2 b0 = __builtin_convertvector(h0, f32x2), b1 = __builtin_convertvector(h1, f32x2);
  const f16x2 l0 = __builtin_convertvector((f32x2){f[0] - b0[0], f[1] - b0[1]}, f16x2);
  const f16x2 l1 = __builtin_convertvector((f32x2){f[2] - b1[0], f[3] - b1[1]}, f16x2);
  h = u32x2{__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1)};
  l = u32x2{__builtin_bit_cast(uint32_t, l0), __builtin_bit_cast(uint32_t, l1)};
}

template <int FJ> struct H3Frag {
  u32x4 b[2][FJ];
  u32x4 raw[2];
  u32x2 ph[2], pl[2];
};

// the A operand's scale: 2^(13 - e) with max |A| in [2^(e-1), 2^e)
SPE_DEV void h3_scale(const float* amax, float& sa, float& inv) {
  sa = inv = 1.f;
  if (!amax) return;
  const float am = *amax;
  if (!(am > 0.f) || !(am <= 3.0e38f)) return;
  const int e = __builtin_amdgcn_frexp_expf(am);
  sa = __builtin_ldexpf(1.f, 13 - e);
  inv = __builtin_ldexpf(1.f, e - 13);
}

template <int MODE, int FJ, bool PL = false>
__device__ __forceinline__ void gemm_h3d_body(const GemmArgs& g) {
  using G = H3Geo<FJ>;
  constexpr int BNH = G::BN, PB = G::PB, STG = G::STAGE, NBQ = G::NBQ, NQ = G::NQ;
  constexpr int LDL = EPI_LD;                          // epilogue tile row stride (floats)
  constexpr int SMEM = 2 * STG > H3_BM * LDL * 4 ? 2 * STG : H3_BM * LDL * 4;
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (g.N + BNH - 1) / BNH;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tilesN) * H3_BM, n0 = (t % tilesN) * BNH;
  const int nk = (g.K + 31) >> 5;
  const long long abytes = MODE == GEMM_CONV ? (long long)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 4
                                             : (long long)g.M * g.lda * 4;
  const size_t pstride = (size_t)g.h3_rows * g.ldb;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.H3, (short)0, (int)(2 * pstride * 2), 0x00020000);
  float sa, inv_sa;
  h3_scale(g.amax_a, sa, inv_sa);

  // ---- DMA pieces of this wave: A pieces wid + 4q (rows 8p .. 8p+7, lane -> row 8p + lane/8,
  // slot lane & 7), B pieces wid + 4q (plane p / (BN/16), rows 16 (p % (BN/16)) + lane/4, slot lane & 3)
  int avo[4], ih0[4], iw0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (wid + 4 * q) * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7), m = m0 + row;
    if constexpr (MODE == GEMM_CONV) {
      const int hw = g.Ho * g.Wo, mm = m < g.M ? m : 0;
      const int b = mm / hw, r = mm - b * hw, oh = r / g.Wo, ow = r - oh * g.Wo;
      ih0[q] = m < g.M ? oh * g.stride - g.pad : -(1 << 28);
      iw0[q] = ow * g.stride - g.pad;
      avo[q] = b * g.H * g.W * g.Cin + (PL ? 0 : c * 4);
    } else {
      avo[q] = m < g.M ? m * g.lda * 4 + c * 16 : D6_BAD;
      ih0[q] = iw0[q] = 0;
    }
  }
  int bvo[NBQ];
#pragma unroll
  for (int q = 0; q < NBQ; ++q) {
    const int p = wid + 4 * q, plane = p / (BNH / 16), row = (p % (BNH / 16)) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3), n = n0 + row;
    bvo[q] = n < g.N ? (int)((plane * pstride + (size_t)n * g.ldb) * 2) + c * 16 : D6_BAD;
  }
  const int ck = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
  auto issue = [&](int ks, int stg) {
    char* base = smem + stg * STG;
    int kh = 0, kw = 0, ci = 0;
    bool kv = true;
    if constexpr (MODE == GEMM_CONV) {
      if constexpr (PL) {
        const int k = ks * 32 + ck * 4, tap = k / g.Cin;
        ci = k - tap * g.Cin;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
        kv = k < g.K;
      } else {
        conv_k_decode(ks * 32, g.Cin, g.KW, g.KH * g.KW, kh, kw, ci);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int off;
      if constexpr (MODE == GEMM_CONV) {
        const int ih = ih0[q] + kh, iw = iw0[q] + kw;
        const bool v = kv && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        off = v ? (avo[q] + (ih * g.W + iw) * g.Cin + ci) * 4 : D6_BAD;
      } else {
        off = avo[q];
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr6_t)(base + (wid + 4 * q) * 1024), 16, off,
                                               MODE == GEMM_CONV ? 0 : ks * 128, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NBQ; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr6_t)(base + H3_A + (wid + 4 * q) * 1024), 16, bvo[q],
                                               ks * 64, 0, 0);
  };

  // ---- fragment offsets: A row 32 wid + (lane & 31), 16-byte chunks 4kk + 2(lane >> 5) + h;
  // B row 32 j + (lane & 31), chunk 2kk + (lane >> 5)
  const int l31 = lane & 31, hi = lane >> 5;
  int aoff[2][2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      aoff[kk][h] = (wid * 32 + l31) * 128 + (((4 * kk + 2 * hi + h) ^ ((l31 >> 1) & 7)) << 4);
    boff[kk] = H3_A + l31 * 64 + (((2 * kk + hi) ^ ((l31 >> 2) & 3)) << 4);
  }
  auto mf = [](u32x4 x, u32x4 y, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, x), __builtin_bit_cast(f16x8, y), c, 0, 0, 0);
  };
  f32x16 acc[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  using Frag = H3Frag<FJ>;
  auto read_b = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) f.b[p][j] = ld16(st + boff[kk] + p * PB + j * 2048);
  };
  auto read_a = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int h = 0; h < 2; ++h) f.raw[h] = ld16(st + aoff[kk][h]);
  };
  auto split_a = [&](Frag& f, int h) { split2h(f.raw[h], sa, f.ph[h], f.pl[h]); };
  // MFMA number q (0 .. NQ-1) of a set: accumulator q / 3, product q % 3 (lo.hi, hi.lo, hi.hi)
  auto mma1 = [&](const Frag& f, int q) {
    const int j = q / 3, t = q % 3;
    const u32x4 xa = t == 0 ? cat2(f.pl[0], f.pl[1]) : cat2(f.ph[0], f.ph[1]);
    const u32x4 xb = t == 1 ? f.b[1][j] : f.b[0][j];
    acc[j] = mf(xa, xb, acc[j]);
  };
#define H3_MMA(F, LO, HI)                                \
  _Pragma("unroll") for (int q = LO; q < HI; ++q) mma1(F, q); \
  __builtin_amdgcn_sched_barrier(0);

  // Software pipeline over K-step halves as in gemm_x6d_body: phase A multiplies X (kk = 0) while
  // Y (kk = 1) is read and split; one barrier; phase B multiplies Y while the next step's X is read
  // from the other stage, whose DMA was issued a whole step earlier.
  issue(0, 0);
  issue(1, 1);
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm(4 + NBQ));
  __syncthreads();
  Frag X, Y;
  read_b(smem, 0, X);
  read_a(smem, 0, X);
  split_a(X, 0);
  split_a(X, 1);
  constexpr int QA = NQ / 3;                           // MFMAs before / between the two splits (phase A)
  constexpr int Q1 = NQ / 6 > 0 ? NQ / 6 : 1, Q2 = Q1 + NQ / 4, Q3 = Q2 + NQ / 4;   // phase B
  for (int ks = 0; ks < nk; ++ks) {
    const char* st = smem + (ks & 1) * STG;
    const char* sn = smem + ((ks + 1) & 1) * STG;
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase A: X's MFMAs, Y read + split
    read_b(st, 1, Y);
    read_a(st, 1, Y);
    H3_MMA(X, 0, QA)
    split_a(Y, 0);
    H3_MMA(X, QA, 2 * QA)
    split_a(Y, 1);
    H3_MMA(X, 2 * QA, NQ)
    __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm0() & ~(15 << 8));  // vmcnt(0) lgkmcnt(0)
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase B: Y's MFMAs, step ks+2's DMA, step ks+1's X read + split
    issue(ks + 2, ks & 1);
    H3_MMA(Y, 0, Q1)
    read_b(sn, 0, X);
    read_a(sn, 0, X);
    H3_MMA(Y, Q1, Q2)
    split_a(X, 0);
    H3_MMA(Y, Q2, Q3)
    split_a(X, 1);
    H3_MMA(Y, Q3, NQ)
  }
#undef H3_MMA
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm0());
  __syncthreads();

  float* ct = reinterpret_cast<float*>(smem);
  // 32x32 accumulator: lane holds rows 8 (r >> 2) + 4 (lane >> 5) + (r & 3), column lane & 31;
  // the column's scale 2^-e_n / s_a (exact) before the bias / residual / activation epilogue
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int n = n0 + 32 * j + l31;
    const float cs = n < g.N ? g.h3_sinv[n] * inv_sa : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      ct[(wid * 32 + 8 * (r >> 2) + 4 * hi + (r & 3)) * LDL + 32 * j + l31] = acc[j][r] * cs;
  }
  __syncthreads();
  float bv[8];
  {
    const int n = n0 + (tid % (BNH / 8)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) bv[e] = (g.bias && n + e < g.N) ? g.bias[n + e] : 0.f;
  }
  const float am = store_tile<float, H3_BM, H3_NT, BNH>(g, ct, m0, n0, tid, bv);
  if (g.amax_c) amax_publish_block(am, g.amax_c, g.amax_c_mul, ct);
}

__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_linear(GemmArgs g) { gemm_h3d_body<GEMM_LINEAR, 4>(g); }
__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_linear_n64(GemmArgs g) { gemm_h3d_body<GEMM_LINEAR, 2>(g); }
__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_conv(GemmArgs g) { gemm_h3d_body<GEMM_CONV, 4>(g); }
__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_conv_n64(GemmArgs g) { gemm_h3d_body<GEMM_CONV, 2>(g); }
__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_conv_pl(GemmArgs g) { gemm_h3d_body<GEMM_CONV, 4, true>(g); }
__global__ __launch_bounds__(H3_NT, 2) void gemm_h3d_conv_pl_n64(GemmArgs g) { gemm_h3d_body<GEMM_CONV, 2, true>(g); }

// Persistent form of gemm_h3d for row-store epilogues (bias, residual / row-periodic residual,
// activation, fp32 C, max |C|): one workgroup per occupancy slot walks its tiles (round i: tile
// i * grid + xcd_remap(block), so an XCD's workgroups share A panels), and the K-steps of
// consecutive tiles form ONE pipeline -- the DMA of the next tile's first steps is issued while the
// current tile's last steps multiply, so no workgroup starts cold.  The accumulators are the
// transposed product (weights as the MFMA's first operand: a lane holds one output row and columns
// 8q + 4(lane >> 5) + 0..3), stored straight from registers with 16-byte buffer stores -- no LDS
// round trip, no barrier -- and left in flight: vmcnt counts loads and stores in issue order, so
// the step after a tile's epilogue waits vmcnt(S) (its DMA is older than the S stores) and only the
// step after that drains them.  To keep that count exact every lane issues all S stores (rows past
// M go to an out-of-range offset, which the buffer unit drops), the per-column bias and scale come
// by LDS-DMA with the tile's first step (two regions, by tile parity), a residual tile is loaded
// into registers before the DMA of the step that ends the tile, and max |C| is published once per
// workgroup.  Needs nk >= NS (the bias region of tile i + 2 is written after tile i's epilogue).
// (The non-persistent kernel with its stores removed ran the encoder's linear1 in 0.63 instead of
// 1.14 ms: the store phase, not the MFMAs, was half of that launch.)
constexpr int H3P_EPI = 2 * 128 * 4;                 // bias[BN] + sinv[BN] floats (BN <= 128) per region
// WM: waves stacked in M (4: 128-row tiles, two workgroups per CU; 8: 256-row tiles, one 8-wave
// workgroup per CU); NS: LDS stages (the DMA runs NS - 1 K-steps ahead; with NS = 3 a tile's stores
// are waited for only 2.5 steps after they were issued).  The launcher uses WM = 4, NS = 2.
template <int FJ, int WM, int NS> struct H3PGeo {
  static constexpr int BM = 32 * WM, BN = 32 * FJ, NT = 64 * WM;
  static constexpr int AB = BM * 128, PB = BN * 64, STG = AB + 2 * PB;
  static constexpr int NBQ = BN / (8 * WM);           // B DMA pieces per wave per step
  static constexpr int NQ = 3 * FJ;
  static constexpr int D = 4 + NBQ;                   // DMA instructions per wave per step (bias pieces aside)
  static constexpr int SMEM = NS * STG + 2 * H3P_EPI;
};
// EPI: 0 fp32 rows; 1 rows, columns n >= s_col0 (a whole number of tiles) as the bf16 hi / lo planes
// of GemmArgs::S (the q/k projection: K for the fp32x3 attention); 2 head-transposed (vt_T: the V^T
// projections), fp32 or S planes -- from the untransposed accumulator, whose lane holds one column
// and four consecutive tokens: one contiguous 16- / 8-byte piece of a V^T row.  Every (j, q) issues
// two stores (a dropped one where the output has one) so the store count stays a constant.
template <int MODE, int FJ, bool PL, bool RES, int WM = 4, int NS = 2, int EPI = 0>
__device__ __forceinline__ void gemm_h3p_body(const GemmArgs& g) {
  using G = H3PGeo<FJ, WM, NS>;
  constexpr int BM = G::BM, BNH = G::BN, PB = G::PB, STG = G::STG, NBQ = G::NBQ, NQ = G::NQ, D = G::D;
  constexpr bool TR = EPI < 2;                         // transposed accumulators (row stores)
  static_assert(!(EPI >= 2 && RES), "no residual on head-transposed stores");
  constexpr int S_ST = FJ * 4 * (EPI == 0 ? 1 : EPI == 3 ? 4 : 2);   // stores per lane per tile
  static_assert(NBQ >= 1 && NS >= 2 && (NS - 1) * D <= 63 && (NS - 2) * D + S_ST <= 63, "geometry / vmcnt");
  __shared__ __attribute__((aligned(1024))) char smem[G::SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tilesN = (g.N + BNH - 1) / BNH, ntiles = ((g.M + BM - 1) / BM) * tilesN;
  const int GR = gridDim.x, w0 = xcd_remap(blockIdx.x, GR);
  const int nk = (g.K + 31) >> 5;
  const int total = w0 < ntiles ? ((ntiles - 1 - w0) / GR + 1) * nk : 0;
  const long long abytes = MODE == GEMM_CONV ? (long long)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 4
                                             : (long long)g.M * g.lda * 4;
  const size_t pstride = (size_t)g.h3_rows * g.ldb;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, (int)abytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.H3, (short)0, (int)(2 * pstride * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rse = __builtin_amdgcn_make_buffer_rsrc((void*)g.h3_sinv, (short)0, g.N * 4, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsbias =
      __builtin_amdgcn_make_buffer_rsrc((void*)(g.bias ? g.bias : g.h3_sinv), (short)0, g.N * 4, 0x00020000);
  const long long cbytes = EPI >= 2 ? (long long)g.vt_B * g.N * g.vt_T * 4 : (long long)g.M * g.ldc * 4;
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(g.C, (short)0, (int)cbytes, 0x00020000);
  const int ns = g.N - g.s_col0;                       // EPI 1: columns in the planes
  const long long sbytes = EPI == 2 ? (long long)g.vt_B * g.N * g.vt_T * 4 : (long long)g.M * ns * 4;
  const __amdgpu_buffer_rsrc_t rss =
      __builtin_amdgcn_make_buffer_rsrc(g.S ? g.S : g.C, (short)0, g.S ? (int)sbytes : 0, 0x00020000);
  float sa, inv_sa;
  h3_scale(g.amax_a, sa, inv_sa);
  const float vsf = EPI == 2 && g.S && g.s_f16 ? vplane_scale(g.amax_a, g.s_l1, g.s_bmax) : 1.f;
  if (total == 0) return;

  // ---- issue side: the tile / K-step of the next DMA and that tile's per-lane source offsets
  int it = w0, iks = 0, iord = 0;
  int avo[4], ih0[4], iw0[4], bvo[NBQ], evo = 0;
  // the tile's sinv / bias piece of this wave (64 columns each): four waves one piece each, two
  // waves (64-column tiles at most) the first half of sinv and of bias
  static_assert(WM >= 4 || (WM == 2 && BNH <= 64), "sinv / bias pieces");
  const int ep = WM >= 4 ? wid : 2 * wid;
  auto setup = [&](int t) {
    const int m0 = (t / tilesN) * BM, n0 = (t % tilesN) * BNH;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = (wid + WM * q) * 8 + (lane >> 3), c = (lane & 7) ^ ((row >> 1) & 7), m = m0 + row;
      if constexpr (MODE == GEMM_CONV) {
        const int hw = g.Ho * g.Wo, mm = m < g.M ? m : 0;
        const int b = mm / hw, r = mm - b * hw, oh = r / g.Wo, ow = r - oh * g.Wo;
        ih0[q] = m < g.M ? oh * g.stride - g.pad : -(1 << 28);
        iw0[q] = ow * g.stride - g.pad;
        avo[q] = b * g.H * g.W * g.Cin + (PL ? 0 : c * 4);
      } else {
        avo[q] = m < g.M ? m * g.lda * 4 + c * 16 : D6_BAD;
        ih0[q] = iw0[q] = 0;
      }
    }
#pragma unroll
    for (int q = 0; q < NBQ; ++q) {
      const int p = wid + WM * q, plane = p / (BNH / 16), row = (p % (BNH / 16)) * 16 + (lane >> 2);
      const int c = (lane & 3) ^ ((row >> 2) & 3), n = n0 + row;
      bvo[q] = n < g.N ? (int)((plane * pstride + (size_t)n * g.ldb) * 2) + c * 16 : D6_BAD;
    }
    const int en = n0 + lane + (ep & 1) * 64;          // pieces 0/1: sinv, 2/3: bias
    evo = en < g.N && en < n0 + BNH ? en * 4 : D6_BAD;
  };
  const int ck = (lane & 7) ^ ((wid * 4 + (lane >> 4)) & 7);
  auto issue_next = [&](int stg) {
    char* base = smem + stg * STG;
    int kh = 0, kw = 0, ci = 0;
    bool kv = true;
    if constexpr (MODE == GEMM_CONV) {
      if constexpr (PL) {
        const int k = iks * 32 + ck * 4;
        if (g.Cin == 4 && g.KW == 7) {                 // the fp32 stem (7x7, 4 channels): constant divisors
          const unsigned tap = (unsigned)k >> 2;
          ci = k & 3;
          kh = (int)(tap / 7u);
          kw = (int)tap - kh * 7;
        } else {
          const int tap = k / g.Cin;
          ci = k - tap * g.Cin;
          kh = tap / g.KW;
          kw = tap - kh * g.KW;
        }
        kv = k < g.K;
      } else {
        conv_k_decode(iks * 32, g.Cin, g.KW, g.KH * g.KW, kh, kw, ci);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int off;
      if constexpr (MODE == GEMM_CONV) {
        const int ih = ih0[q] + kh, iw = iw0[q] + kw;
        const bool v = kv && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        off = v ? (avo[q] + (ih * g.W + iw) * g.Cin + ci) * 4 : D6_BAD;
      } else {
        off = avo[q];
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_ptr6_t)(base + (wid + WM * q) * 1024), 16, off,
                                               MODE == GEMM_CONV ? 0 : iks * 128, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NBQ; ++q)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (lds_ptr6_t)(base + G::AB + (wid + WM * q) * 1024), 16, bvo[q],
                                               iks * 64, 0, 0);
    if (iks == 0 && ep < 4) {                        // the tile's sinv / bias columns, 4 bytes a lane
      char* eb = smem + NS * STG + (iord & 1) * H3P_EPI + (ep >> 1) * (128 * 4) + (ep & 1) * 256;
      if (ep < 2) __builtin_amdgcn_raw_ptr_buffer_load_lds(rse, (lds_ptr6_t)eb, 4, evo, 0, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rsbias, (lds_ptr6_t)eb, 4, g.bias ? evo : D6_BAD, 0, 0, 0);
    }
    if (++iks == nk) {                               // past the last tile: keep issuing the last tile's
      iks = 0;                                       // offsets (in range or dropped), never consumed
      ++iord;
      it += GR;
      if (it < ntiles) setup(it);
    }
  };

  // ---- fragment offsets (as gemm_h3d_body)
  const int l31 = lane & 31, hi = lane >> 5;
  int aoff[2][2], boff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
      aoff[kk][h] = (wid * 32 + l31) * 128 + (((4 * kk + 2 * hi + h) ^ ((l31 >> 1) & 7)) << 4);
    boff[kk] = G::AB + l31 * 64 + (((2 * kk + hi) ^ ((l31 >> 2) & 3)) << 4);
  }
  auto mf = [](u32x4 x, u32x4 y, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, x), __builtin_bit_cast(f16x8, y), c, 0, 0, 0);
  };
  f32x16 acc[FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  using Frag = H3Frag<FJ>;
  auto read_b = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int p = 0; p < 2; ++p) f.b[p][j] = ld16(st + boff[kk] + p * PB + j * 2048);
  };
  auto read_a = [&](const char* st, int kk, Frag& f) {
#pragma unroll
    for (int h = 0; h < 2; ++h) f.raw[h] = ld16(st + aoff[kk][h]);
  };
  auto split_a = [&](Frag& f, int h) { split2h(f.raw[h], sa, f.ph[h], f.pl[h]); };
  // transposed product: C^T[n][m] += W[n][k] A[m][k]
  auto mma1 = [&](const Frag& f, int q) {
    const int j = q / 3, t = q % 3;
    const u32x4 xa = t == 0 ? cat2(f.pl[0], f.pl[1]) : cat2(f.ph[0], f.ph[1]);
    const u32x4 xb = t == 1 ? f.b[1][j] : f.b[0][j];
    if constexpr (TR) acc[j] = mf(xb, xa, acc[j]);
    else acc[j] = mf(xa, xb, acc[j]);
  };
#define H3P_MMA(F, LO, HI)                               \
  _Pragma("unroll") for (int q = LO; q < HI; ++q) mma1(F, q); \
  __builtin_amdgcn_sched_barrier(0);

  // ---- epilogue state: the computing tile
  int cord = 0, cks = 0;
  float runmax = 0.f;
  u32x4 rres[RES ? FJ * 4 : 1];
  auto tile_mn = [&](int ord, int& m0, int& n0) {
    const int t = w0 + ord * GR;
    m0 = (t / tilesN) * BM;
    n0 = (t % tilesN) * BNH;
  };
  auto load_res = [&]() {
    if constexpr (RES) {
      int m0, n0;
      tile_mn(cord, m0, n0);
      const int m = m0 + wid * 32 + l31;
      const size_t rrow = (size_t)(g.r_period > 0 ? (m < g.M ? m : 0) % g.r_period : (m < g.M ? m : 0)) * g.ldr;
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + 32 * j + 8 * q + 4 * hi;
          rres[4 * j + q] = n < g.N ? ld16((const float*)g.R + rrow + n) : u32x4{0, 0, 0, 0};
        }
    }
  };
  auto epilogue = [&]() {
    int m0, n0;
    tile_mn(cord, m0, n0);
    const int m = m0 + wid * 32 + l31;
    const float* eb = reinterpret_cast<const float*>(smem + NS * STG + (cord & 1) * H3P_EPI);
    auto hilo = [](const float* v, u32x2& h, u32x2& l) {   // the RNE bf16 split of store_tile's S path
      h = u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      const float r0 = v[0] - __uint_as_float(h.x << 16), r1 = v[1] - __uint_as_float(h.x & 0xffff0000u);
      const float r2 = v[2] - __uint_as_float(h.y << 16), r3 = v[3] - __uint_as_float(h.y & 0xffff0000u);
      l = u32x2{pack_bf16x2(r0, r1), pack_bf16x2(r2, r3)};
    };
    if constexpr (EPI == 3) {
      // head-transposed fp32 at any token count: the lane's four rows may straddle images, one
      // 4-byte store each
      const int mb = m0 + wid * 32 + 4 * hi;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int c = 32 * j + l31, n = n0 + c;
        const float sv = eb[c] * inv_sa, bv = eb[128 + c];
        const int grp = n >> 8, hd = n & 255;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int mr = mb + 8 * q + e;
            const bool ok = mr < g.M && n < g.N;
            const int b = mr / g.vt_T, tok = mr - b * g.vt_T;
            const int idx = ok ? ((grp * g.vt_B + b) * 256 + hd) * g.vt_T + tok : 0;
            float v = acc[j][4 * q + e] * sv + bv;
            if (g.act) v = apply_act(v, g.act);
            if (ok) runmax = fmaxf(runmax, fabsf(v));
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsc, ok ? idx * 4 : D6_BAD, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
      return;
    }
    if constexpr (EPI == 2) {
      const int mb = m0 + wid * 32 + 4 * hi;         // + 8 q: four consecutive tokens of one image
      const long long lo = (long long)g.vt_B * g.N * g.vt_T;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int c = 32 * j + l31, n = n0 + c;
        const float sv = eb[c] * inv_sa, bv = eb[128 + c];
        const int grp = n >> 8, hd = n & 255;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int mr = mb + 8 * q;
          const bool ok = mr < g.M && n < g.N;
          const int b = mr / g.vt_T, tok = mr - b * g.vt_T;
          const int idx = ok ? ((grp * g.vt_B + b) * 256 + hd) * g.vt_T + (g.vt_swz ? vt_pos(tok) : tok) : 0;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[j][4 * q + e] * sv + bv;
            if (g.act) v[e] = apply_act(v[e], g.act);
          }
          if (ok) runmax = fmaxf(runmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
          if (g.S) {
            u32x2 h, l;
            if (g.s_f16) {
              float w[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) w[e] = v[e] * vsf;
              split_f16x4(w, h, l);
            } else {
              hilo(v, h, l);
            }
            __builtin_amdgcn_raw_buffer_store_b64(h, rss, ok ? idx * 2 : D6_BAD, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(l, rss, ok ? (int)((lo + idx) * 2) : D6_BAD, 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(pack16<float>(v), rsc, ok ? idx * 4 : D6_BAD, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{0, 0}, rsc, D6_BAD, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
      return;
    }
    const bool splanes = EPI == 1 && g.S && n0 >= g.s_col0;   // whole tile in the planes
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int c = 32 * j + 8 * q + 4 * hi, n = n0 + c;
        const f32x4 sv = *reinterpret_cast<const f32x4*>(eb + c);
        const f32x4 bv = *reinterpret_cast<const f32x4*>(eb + 128 + c);
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[j][4 * q + e] * (sv[e] * inv_sa) + bv[e];
        if constexpr (RES) {
          float rv[4];
          unpack16<float>(rres[4 * j + q], rv);
          if (!g.res_post) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += rv[e];
          }
          if (g.act) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], g.act);
          }
          if (g.res_post) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += rv[e];
          }
        } else if (g.act) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], g.act);
        }
        const bool ok = m < g.M && n < g.N;
        if (ok) runmax = fmaxf(runmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        if (EPI == 1 && splanes) {
          u32x2 h, l;
          hilo(v, h, l);
          const int so = m * ns + (n - g.s_col0);
          __builtin_amdgcn_raw_buffer_store_b64(h, rss, ok ? so * 2 : D6_BAD, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b64(l, rss, ok ? (g.M * ns + so) * 2 : D6_BAD, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(pack16<float>(v), rsc, ok ? (m * g.ldc + n) * 4 : D6_BAD, 0, 0);
          if constexpr (EPI == 1) __builtin_amdgcn_raw_buffer_store_b64(u32x2{0, 0}, rsc, D6_BAD, 0, 0);
        }
      }
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  };

  setup(w0);
#pragma unroll
  for (int i = 0; i < NS; ++i) issue_next(i);
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm((NS - 1) * D));   // step 0's DMA (the bias pieces are older)
  __syncthreads();
  Frag X, Y;
  read_b(smem, 0, X);
  read_a(smem, 0, X);
  split_a(X, 0);
  split_a(X, 1);
  constexpr int QA = NQ / 3;
  constexpr int Q1 = NQ / 6 > 0 ? NQ / 6 : 1, Q2 = Q1 + NQ / 4, Q3 = Q2 + NQ / 4;
  int sc = 0;                                        // gs % NS
  int since = 1 << 20;                               // steps since the last epilogue
  for (int gs = 0; gs < total; ++gs) {
    const int sn_i = sc + 1 == NS ? 0 : sc + 1;
    const char* st = smem + sc * STG;
    const char* sn = smem + sn_i * STG;
    const bool last = cks == nk - 1;
    __builtin_amdgcn_sched_barrier(0);
    read_b(st, 1, Y);
    read_a(st, 1, Y);
    H3P_MMA(X, 0, QA)
    split_a(Y, 0);
    H3P_MMA(X, QA, 2 * QA)
    split_a(Y, 1);
    H3P_MMA(X, 2 * QA, NQ)
    // wait for step gs + 1's DMA: the younger operations are the later DMA steps (NS - 2 of them)
    // and, when a tile ended within the last NS - 1 steps, its S stores
    if (since < NS - 1) __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm((NS - 2) * D + S_ST) & ~(15 << 8));
    else __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm((NS - 2) * D) & ~(15 << 8));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (RES && last) load_res();
    __builtin_amdgcn_sched_barrier(0);
    issue_next(sc);                                  // step gs + NS into the stage just consumed
    H3P_MMA(Y, 0, Q1)
    read_b(sn, 0, X);
    read_a(sn, 0, X);
    H3P_MMA(Y, Q1, Q2)
    split_a(X, 0);
    H3P_MMA(Y, Q2, Q3)
    split_a(X, 1);
    H3P_MMA(Y, Q3, NQ)
    ++since;
    if (last) {
      epilogue();
      ++cord;
      cks = 0;
      since = 0;
    } else {
      ++cks;
    }
    sc = sn_i;
  }
#undef H3P_MMA
  __builtin_amdgcn_s_waitcnt(d6_waitcnt_vm0());
  if (g.amax_c) amax_publish_block(runmax, g.amax_c, g.amax_c_mul, reinterpret_cast<float*>(smem));
}

#define H3P_KERNELS(SUF, WM, NS, OCC)                                                                                  \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_linear##SUF(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 4, false, false, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_linear_n64##SUF(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, false, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_linear_r##SUF(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 4, false, true, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_linear_r_n64##SUF(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, true, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 4, false, false, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv_n64##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 2, false, false, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv_r##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 4, false, true, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv_r_n64##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 2, false, true, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv_pl##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 4, true, false, WM, NS>(g); } \
  __global__ __launch_bounds__(64 * WM, OCC) void gemm_h3p_conv_pl_n64##SUF(GemmArgs g) { gemm_h3p_body<GEMM_CONV, 2, true, false, WM, NS>(g); }
H3P_KERNELS(, 4, 2, 2)
#undef H3P_KERNELS
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_s(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 4, false, false, 4, 2, 1>(g); }
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_s_r(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 4, false, true, 4, 2, 1>(g); }
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_vt(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 4, false, false, 4, 2, 2>(g); }
// few-row problems (the decoder's B*Q rows): 64-column tiles -- twice the work-groups on a grid that
// leaves most CUs idle -- with a third stage (74 KB of LDS); measured 1.19 -> 1.02 ms for the fp32h3
// decoder's 42 GEMMs, and slower on the full-size launches (q/k 1.60 -> 1.80 ms: DESIGN.md section 0)
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_fr(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, false, 4, 3>(g); }
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_r_fr(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, true, 4, 3>(g); }
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_vt_fr(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, false, 4, 3, 2>(g); }
__global__ __launch_bounds__(256, 2) void gemm_h3p_linear_vte_fr(GemmArgs g) { gemm_h3p_body<GEMM_LINEAR, 2, false, false, 4, 3, 3>(g); }
// long-K few-row problems (the decoder's linear2, K = 2048, on 24 work-groups: a chain of 64 K-steps
// per work-group, each waiting on its DMA): six stages, five K-steps in flight, one work-group per CU
// (148 KB of LDS).  The MFMA sequence per output is the one of every h3 kernel (K-steps in order; per
// 16-wide chunk lo.hi, hi.lo, hi.hi), so the results are the same bits as the non-persistent kernel's.
#ifndef SPE_FRD_NS
#define SPE_FRD_NS 6
#endif
#ifndef SPE_FRD_FJ
#define SPE_FRD_FJ 1
#endif
#ifndef SPE_FRD_WM
#define SPE_FRD_WM 2
#endif
__global__ __launch_bounds__(64 * SPE_FRD_WM, 1) void gemm_h3p_linear_frd(GemmArgs g) {
  gemm_h3p_body<GEMM_LINEAR, SPE_FRD_FJ, false, false, SPE_FRD_WM, SPE_FRD_NS>(g);
}
__global__ __launch_bounds__(64 * SPE_FRD_WM, 1) void gemm_h3p_linear_r_frd(GemmArgs g) {
  gemm_h3p_body<GEMM_LINEAR, SPE_FRD_FJ, false, true, SPE_FRD_WM, SPE_FRD_NS>(g);
}
constexpr int H3_FRD_MIN_K = 1281;
constexpr int H3_FEW_ROWS = 4096;

// 1 = not a problem for the h3 kernel (the caller runs the x6 path)
int launch_h3d(const GemmArgs& g, int mode, hipStream_t s) {
  if (!g.H3 || !g.h3_sinv || (mode != GEMM_LINEAR && mode != GEMM_CONV) || (g.lda & 3)) return 1;
  const bool pl = mode == GEMM_CONV && (g.Cin & 31);
  if (pl ? ((g.Cin & 3) || (g.K & 3) || g.K != g.Cin * g.KH * g.KW) : (g.K & 31)) return 1;
  if ((reinterpret_cast<uintptr_t>(g.A) & 15) || (reinterpret_cast<uintptr_t>(g.H3) & 15) || (g.ldb & 7)) return 1;
  constexpr long long LIM = (1LL << 31) - (1LL << 24);
  if ((long long)2 * g.h3_rows * g.ldb * 2 >= LIM || g.h3_rows < g.N) return 1;
  if (mode == GEMM_CONV) {
    if ((long long)(g.M / (g.Ho * g.Wo)) * g.H * g.W * g.Cin * 4 >= LIM) return 1;
  } else if ((long long)(g.M + H3_BM) * g.lda * 4 + (long long)g.K * 4 >= LIM) {
    return 1;
  }
  const bool narrow = g.N <= 64;
  const int bn = narrow ? 64 : 128;
  const int tiles = ((g.M + H3_BM - 1) / H3_BM) * ((g.N + bn - 1) / bn);
  if (tiles <= 0) return 0;
  const dim3 grid(tiles), block(H3_NT);
  // the persistent form for plain row stores (gemm_h3p_body)
  const bool res = g.R != nullptr;
  {
    // persistent S-plane (EPI 1) and head-transposed (EPI 2) forms: 128-column tiles
    const int ncu = spe_cu_count();
    const dim3 pg(tiles < 2 * ncu || ncu <= 0 ? tiles : 2 * ncu), pb(256);
    const bool rok = !res || (!(g.ldr & 3) && !(reinterpret_cast<uintptr_t>(g.R) & 15));
    if (mode == GEMM_LINEAR && !narrow && g.K >= 64 && g.S && g.vt_T <= 0 && rok && g.s_col0 % 128 == 0 &&
        g.s_col0 < g.N && !(g.N & 3) && !(g.ldc & 3) && !(reinterpret_cast<uintptr_t>(g.C) & 15) &&
        (long long)g.M * g.ldc * 4 < LIM && (long long)g.M * (g.N - g.s_col0) * 4 < LIM) {
      if (res) hipLaunchKernelGGL(gemm_h3p_linear_s_r, pg, pb, 0, s, g);
      else hipLaunchKernelGGL(gemm_h3p_linear_s, pg, pb, 0, s, g);
      spe_gemm_last_path = 8;
      return (int)hipGetLastError();
    }
    if (mode == GEMM_LINEAR && !narrow && g.K >= 64 && g.vt_T > 0 && !res && !g.out_f16 &&
        (!g.vt_swz || (g.S && g.vt_T % 16 == 0)) && (!g.s_f16 || g.S) &&
        g.vt_T % 4 == 0 && g.M == g.vt_B * g.vt_T && !(g.N & 255) && (!g.S || g.s_col0 == 0) &&
        (long long)g.vt_B * g.N * g.vt_T * 4 < LIM && !(reinterpret_cast<uintptr_t>(g.C) & 15)) {
      if (g.M <= H3_FEW_ROWS && g.K >= 96) {
        const int t2 = ((g.M + H3_BM - 1) / H3_BM) * ((g.N + 63) / 64);
        hipLaunchKernelGGL(gemm_h3p_linear_vt_fr, dim3(t2 < 2 * ncu || ncu <= 0 ? t2 : 2 * ncu), pb, 0, s, g);
      } else {
        hipLaunchKernelGGL(gemm_h3p_linear_vt, pg, pb, 0, s, g);
      }
      spe_gemm_last_path = 8;
      return (int)hipGetLastError();
    }
    // few-row head-transposed fp32 at a token count the 16-byte form cannot take (the decoder's
    // self-attention V^T, T = Q = 11)
    if (mode == GEMM_LINEAR && !narrow && g.M <= H3_FEW_ROWS && g.K >= 96 && g.vt_T > 0 && !res && !g.S &&
        !g.out_f16 && !g.vt_swz && g.M == g.vt_B * g.vt_T && !(g.N & 255) &&
        (long long)g.vt_B * g.N * g.vt_T * 4 < LIM) {
      const int t2 = ((g.M + H3_BM - 1) / H3_BM) * ((g.N + 63) / 64);
      hipLaunchKernelGGL(gemm_h3p_linear_vte_fr, dim3(t2 < 2 * ncu || ncu <= 0 ? t2 : 2 * ncu), pb, 0, s, g);
      spe_gemm_last_path = 8;
      return (int)hipGetLastError();
    }
  }
  // (also the N <= 512 ones: 13 -> 11 us a launch for the decoder's 256-column projections; the
  // 2048-column ones are slower on it, 704 tiles)
  if (mode == GEMM_LINEAR && !narrow && g.M <= H3_FEW_ROWS && (g.K >= H3_FRD_MIN_K || g.N <= 512) && g.vt_T <= 0 && !g.S &&
      (g.K >> 5) >= SPE_FRD_NS && !(g.N & 3) && !(g.ldc & 3) && !(reinterpret_cast<uintptr_t>(g.C) & 15) &&
      (long long)g.M * g.ldc * 4 < LIM && (!res || (!(g.ldr & 3) && !(reinterpret_cast<uintptr_t>(g.R) & 15)))) {
    const int ncu = spe_cu_count();
    constexpr int FBM = 32 * SPE_FRD_WM, FBN = 32 * SPE_FRD_FJ;
    const int t2 = ((g.M + FBM - 1) / FBM) * ((g.N + FBN - 1) / FBN);
    const int slots = SPE_FRD_WM == 2 ? 2 * ncu : ncu;   // 76 KB (two waves) / 148 KB (four) of LDS
    const dim3 pg(t2 < slots || ncu <= 0 ? t2 : slots), pb(64 * SPE_FRD_WM);
    if (res) hipLaunchKernelGGL(gemm_h3p_linear_r_frd, pg, pb, 0, s, g);
    else hipLaunchKernelGGL(gemm_h3p_linear_frd, pg, pb, 0, s, g);
    spe_gemm_last_path = 8;
    return (int)hipGetLastError();
  }
  // (long-K problems keep the non-persistent kernel: the layer-3 3x3, K = 2304, measured 0.213 vs
  // 0.245 ms and the neck, K = 4608, 1.35 vs 1.39 ms; up to K = 1152 the persistent form is as fast
  // or faster)
  if (g.vt_T <= 0 && !g.S && g.K >= 64 && g.K <= 1280 && !(g.N & 3) && !(g.ldc & 3) && !(reinterpret_cast<uintptr_t>(g.C) & 15) &&
      (long long)g.M * g.ldc * 4 < LIM && (!res || (!pl && !(g.ldr & 3) && !(reinterpret_cast<uintptr_t>(g.R) & 15)))) {
    const int ncu = spe_cu_count();
    // (the 256-row, three-stage, 8-wave form -- H3PGeo<4, 8, 3> -- measured 0-5 % slower on every
    // shape of scripts/x6_bench.py: the slack it gives the stores is not what these launches lack)
    const dim3 pg(tiles < 2 * ncu || ncu <= 0 ? tiles : 2 * ncu), pb(256);
#define H3P_GO(K) hipLaunchKernelGGL(K, pg, pb, 0, s, g)
#define H3P_SEL(NAME) H3P_GO(NAME)
    if (mode == GEMM_LINEAR && !narrow && g.M <= H3_FEW_ROWS && g.K >= 96) {
      const int t2 = ((g.M + H3_BM - 1) / H3_BM) * ((g.N + 63) / 64);
      const dim3 pg2(t2 < 2 * ncu || ncu <= 0 ? t2 : 2 * ncu);
      if (res) hipLaunchKernelGGL(gemm_h3p_linear_r_fr, pg2, pb, 0, s, g);
      else hipLaunchKernelGGL(gemm_h3p_linear_fr, pg2, pb, 0, s, g);
    } else if (mode == GEMM_CONV && pl) {
      if (narrow) H3P_SEL(gemm_h3p_conv_pl_n64);
      else H3P_SEL(gemm_h3p_conv_pl);
    } else if (mode == GEMM_CONV) {
      if (res) {
        if (narrow) H3P_SEL(gemm_h3p_conv_r_n64);
        else H3P_SEL(gemm_h3p_conv_r);
      } else {
        if (narrow) H3P_SEL(gemm_h3p_conv_n64);
        else H3P_SEL(gemm_h3p_conv);
      }
    } else if (res) {
      if (narrow) H3P_SEL(gemm_h3p_linear_r_n64);
      else H3P_SEL(gemm_h3p_linear_r);
    } else {
      if (narrow) H3P_SEL(gemm_h3p_linear_n64);
      else H3P_SEL(gemm_h3p_linear);
    }
#undef H3P_SEL
#undef H3P_GO
    spe_gemm_last_path = 8;
    return (int)hipGetLastError();
  }
  if (mode == GEMM_CONV && pl) {
    if (narrow) hipLaunchKernelGGL(gemm_h3d_conv_pl_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_h3d_conv_pl, grid, block, 0, s, g);
  } else if (mode == GEMM_CONV) {
    if (narrow) hipLaunchKernelGGL(gemm_h3d_conv_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_h3d_conv, grid, block, 0, s, g);
  } else {
    if (narrow) hipLaunchKernelGGL(gemm_h3d_linear_n64, grid, block, 0, s, g);
    else hipLaunchKernelGGL(gemm_h3d_linear, grid, block, 0, s, g);
  }
  return (int)hipGetLastError();
}

template <typename T, bool X3 = false>
int launch_t(const GemmArgs& g, int mode, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  if (tiles <= 0) return 0;
  dim3 grid(tiles), block(NT);
  switch (mode) {
    case GEMM_LINEAR: hipLaunchKernelGGL((gemm_kernel<T, GEMM_LINEAR, X3>), grid, block, 0, s, g); break;
    case GEMM_LINEAR_ADD: hipLaunchKernelGGL((gemm_kernel<T, GEMM_LINEAR_ADD, X3>), grid, block, 0, s, g); break;
    case GEMM_CONV: hipLaunchKernelGGL((gemm_kernel<T, GEMM_CONV, X3>), grid, block, 0, s, g); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

}  // namespace

thread_local int spe_gemm_last_path = 0;

int spe_launch_gemm(const GemmArgs& g, int dtype, int mode, hipStream_t s) {
  constexpr int CEb = 8, CEf = 4;
  const int ce = dtype == SPE_DTYPE_BF16 ? CEb : CEf;
  if (g.K % ce) return -2;                                   // K must be whole 16-byte chunks
  // (Cin == 4 pairs: see spe_launch_gemm2 -- a chunk is two adjacent in-range pixels)
  const bool pairs = mode == GEMM_CONV && ce == 8 && g.Cin == 4 && g.pad == 0 && g.KW % 2 == 0 &&
                     (g.Wo - 1) * g.stride + g.KW <= g.W && (g.Ho - 1) * g.stride + g.KH <= g.H;
  if (mode == GEMM_CONV && (g.Cin % ce) && !pairs) return -3;
  if (g.ldb % 64) return -4;                                 // weights padded to 64 elements
  if ((g.lda % ce) || (g.ldc % (g.out_f32 ? 4 : ce)) || (g.R && (g.ldr % ce))) return -5;
  // fused LayerNorm: the large-tile bf16 kernel only
  if (g.ln_g && dtype != SPE_DTYPE_BF16) return -5;
  if (dtype == SPE_DTYPE_BF16) {                 // 256-row tiles when they fill the chip
    spe_gemm_last_path = 1;
    const int rc = spe_launch_gemm2(g, mode, s);
    if (rc != 1) return rc;
  }
  spe_gemm_last_path = 0;
  if (dtype == SPE_DTYPE_F32X3) return launch_t<float, true>(g, mode, s);
  if (dtype == SPE_DTYPE_F32H3) {
    spe_gemm_last_path = 7;
    const int rc = launch_h3d(g, mode, s);
    if (rc != 1) return rc;
    dtype = SPE_DTYPE_F32X6;                     // shapes the h3 kernel does not serve: the x6 path
  }
  if (dtype == SPE_DTYPE_F32X6) {
    // few-row problems (the decoder's B*Q rows) would leave most CUs idle on 256 x 128 tiles:
    // they take the 128 x 128 geometry (at 2.7x the exact-f32 kernel's matrix rate per tile)
    const int tiles6 = ((g.M + BM6 - 1) / BM6) * ((g.N + BN6 - 1) / BN6);
    spe_gemm_last_path = 6;
    const int rc = launch_x6d(g, mode, s);
    if (rc != 1) return rc;
    spe_gemm_last_path = 5;
    return tiles6 >= 128 ? launch_x6(g, mode, s) : launch_x6_geo<128>(g, mode, s);
  }
  return dtype == SPE_DTYPE_BF16 ? launch_t<bf16>(g, mode, s) : launch_t<float>(g, mode, s);
}

int spe_launch_gemm_h3(const GemmArgs& g, int mode, hipStream_t s) {
  if ((g.K & 3) || (g.ldb % 64) || (g.lda & 3) || (g.ldc & 3) || (g.R && (g.ldr & 3)) || g.ln_g) return -5;
  spe_gemm_last_path = 7;
  return launch_h3d(g, mode, s);                 // 1: not served (nothing launched)
}
