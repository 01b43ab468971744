// Attention lab (development only): times the production encoder attention kernel
// (csrc/attention.hip, included verbatim) beside candidate variants on the bench shape
// (B=64, H=8, T=2704, head_dim 32, bf16) and compares their outputs.
//
// usage: attn_lab [iters] [B]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "attention.hip"
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

namespace {

// ---------------------------------------------------------------- variant v2
// Tile 0 (and any partial tile) computes the exact running max as before.  Every later full
// tile skips the max chain: p = exp2(s - m) against the stale running max, the tile's row sums
// come from a fresh ones . P^T MFMA chain, and only if some lane's tile sum reaches 2^64
// (p may have grown past 2^64, or overflowed) is the tile recomputed with the exact max and
// the accumulators rescaled.  m only ever grows on that path, so P stays within [0, 2^64].
constexpr float SUM_LIMIT = 18446744073709551616.0f;   // 2^64

template <typename TI>
__global__ __launch_bounds__(NT, SPE_ATTN_OCC) void attn_v2_kernel(AttnArgs a) {
  typedef AT<TI> A;
  typedef typename A::v8 v8;
  constexpr int KBYTES = KT * KROW, VBYTES = 32 * VROW;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;

  v8 qf[2];
  {
    const float sl2 = a.scale * LOG2E;
    const TI* qp = (const TI*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<TI>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[i] = __builtin_bit_cast(v8, pack16<TI>(f));
    }
  }
  u32x4 ones_u{A::ONE2, A::ONE2, A::ONE2, A::ONE2};
  asm volatile("" : "+v"(ones_u));
  const v8 ones = __builtin_bit_cast(v8, ones_u);
  f32x16 zero;
#pragma unroll
  for (int r = 0; r < 16; ++r) zero[r] = 0.f;

  f32x16 o, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, ls = 0.f;

  const int ntiles = (a.Tk + KT - 1) / KT;
  constexpr int SLOT = KBYTES + VBYTES;
  Stage<TI, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + (kt & 1) * SLOT;
    const char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if (more) st.load(a, b, h, kt + 1, tid);
    if (wave_live) {
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + k_off_bf16(sub * 32 + r32, hh));
        kf[sub][1] = ld16(kl + k_off_bf16(sub * 32 + r32, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          vf[sub][ks] = ld16(vl + r32 * VROW + (2 * sub + ks) * 32 + hh * 16);
      const bool exact = kt == 0 || (kt + 1) * KT > a.Tk;     // first or partial tile
      f32x16 s0, s1;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], exact ? zero : negm);
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
      }
      v8 pb[4];
      f32x16 lt;
      bool redo = exact;
      if (!exact) {
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x16& p = (i >> 1) ? s1 : s0;
          const int ks = i & 1;
          u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                   A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
          pb[i] = __builtin_bit_cast(v8, pw);
        }
        lt = A::mfma(ones, pb[0], zero);
        lt = A::mfma(ones, pb[1], lt);
        lt = A::mfma(ones, pb[2], lt);
        lt = A::mfma(ones, pb[3], lt);
        redo = __any(!(lt[0] < SUM_LIMIT));
        if (redo) {           // recompute the raw scores for the exact path
#pragma unroll
          for (int sub = 0; sub < 2; ++sub) {
            f32x16& s = sub ? s1 : s0;
            s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], zero);
            s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
          }
        }
      }
      if (redo) {
        // exact path: s0/s1 hold raw scores (exp2 domain)
        const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
        const float mn = kt == 0 ? mx : __builtin_fmaxf(m, mx);
        if (kt != 0) {
          const float alpha = __builtin_amdgcn_exp2f(m - mn);
#pragma unroll
          for (int r = 0; r < 16; ++r) o[r] *= alpha;
          ls *= alpha;
        }
        m = mn;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          negm[r] = -m;
          s0[r] = __builtin_amdgcn_exp2f(s0[r] - m);
          s1[r] = __builtin_amdgcn_exp2f(s1[r] - m);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x16& p = (i >> 1) ? s1 : s0;
          const int ks = i & 1;
          u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                   A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
          pb[i] = __builtin_bit_cast(v8, pw);
        }
        lt = A::mfma(ones, pb[0], zero);
        lt = A::mfma(ones, pb[1], lt);
        lt = A::mfma(ones, pb[2], lt);
        lt = A::mfma(ones, pb[3], lt);
      }
      ls += lt[0];
#pragma unroll
      for (int i = 0; i < 4; ++i) o = A::mfma(__builtin_bit_cast(v8, vf[i >> 1][i & 1]), pb[i], o);
    }
    if (more) st.store(smem + ((kt + 1) & 1) * SLOT, smem + ((kt + 1) & 1) * SLOT + KBYTES, tid);
    __syncthreads();
  }

  if (!wave_live || q >= a.Tq) return;
  const float inv = 1.f / ls;
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}



// ---------------------------------------------------------------- variant v4 (row sums)
// The production kernel with the row sums taken off the matrix pipe: LSM 1 = f32 adds of p
// before packing, LSM 2 = v_dot2_f32_bf16 on the packed P (the exact bf16 values PV uses),
// LSM 3 = no row sums at all (ablation: wrong output, timing only).
template <int LSM>
__global__ __launch_bounds__(NT, SPE_ATTN_OCC) void attn_v4_kernel(AttnArgs a) {
  typedef AT<bf16> A;
  typedef A::v8 v8;
  constexpr int KBYTES = KT * KROW, VBYTES = 32 * VROW;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;
  v8 qf[2];
  {
    const float sl2 = a.scale * LOG2E;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<bf16>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[i] = __builtin_bit_cast(v8, pack16<bf16>(f));
    }
  }
  f32x16 o, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, ls = 0.f;
  const int ntiles = (a.Tk + KT - 1) / KT;
  constexpr int SLOT = KBYTES + VBYTES;
  Stage<bf16, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + (kt & 1) * SLOT;
    const char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if (more) st.load(a, b, h, kt + 1, tid);
    if (wave_live) {
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + k_off_bf16(sub * 32 + r32, hh));
        kf[sub][1] = ld16(kl + k_off_bf16(sub * 32 + r32, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          vf[sub][ks] = ld16(vl + r32 * VROW + (2 * sub + ks) * 32 + hh * 16);
      f32x16 s0, s1;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], negm);
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
      }
      const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
      if (kt == 0 || __any(mx > RESCALE_SLACK)) {
        const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
        if (kt != 0) {
          const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int r = 0; r < 16; ++r) o[r] *= alpha;
          ls *= alpha;
        }
        m += d;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
      if constexpr (LSM == 1) {
        float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) { t0 += s0[r]; t1 += s0[r + 1]; t2 += s1[r]; t3 += s1[r + 1]; }
        ls += (t0 + t1) + (t2 + t3);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x16& p = (i >> 1) ? s1 : s0;
        const int ks = i & 1;
        u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                 A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
        if constexpr (LSM == 2) {
          const uint32_t one2 = 0x3F803F80u;
#pragma unroll
          for (int j = 0; j < 4; ++j)
            ls = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, pw[j]), __builtin_bit_cast(bf16x2_t, one2), ls, false);
        }
        const v8 pb = __builtin_bit_cast(v8, pw);
        o = A::mfma(__builtin_bit_cast(v8, vf[i >> 1][i & 1]), pb, o);
      }
    }
    if (more) st.store(smem + ((kt + 1) & 1) * SLOT, smem + ((kt + 1) & 1) * SLOT + KBYTES, tid);
    __syncthreads();
  }
  if (!wave_live || q >= a.Tq) return;
  const float lt = LSM == 3 ? 1.f : ls + __shfl_xor(ls, 32, 64);
  const float inv = 1.f / lt;
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}

// ---------------------------------------------------------------- variant v5 (G query groups per wave)
// v4.add (row sums as f32 adds) with each wave owning G groups of 32 queries that share the
// K / V^T fragments it reads from LDS: per query, G times fewer LDS fragment reads and (with
// the workgroup covering 128*G queries) G times less K/V staging.
template <int G, int OCC>
__global__ __launch_bounds__(NT, OCC) void attn_v5_kernel(AttnArgs a) {
  typedef AT<bf16> A;
  typedef A::v8 v8;
  constexpr int KBYTES = KT * KROW, VBYTES = 32 * VROW, QW = 32 * G, QB = 4 * QW;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + QB - 1) / QB;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q0 = qb * QB + wid * QW + r32;      // group g: q0 + 32 g
  const bool wave_live = qb * QB + wid * QW < a.Tq;
  v8 qf[G][2];
  const float sl2 = a.scale * LOG2E;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = q0 + 32 * g;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<bf16>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[g][i] = __builtin_bit_cast(v8, pack16<bf16>(f));
    }
  }
  f32x16 o[G], negm[G];
  float m[G], ls[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { o[g][r] = 0.f; negm[g][r] = 0.f; }
    m[g] = 0.f; ls[g] = 0.f;
  }
  const int ntiles = (a.Tk + KT - 1) / KT;
  constexpr int SLOT = KBYTES + VBYTES;
  Stage<bf16, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + (kt & 1) * SLOT;
    const char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if (more) st.load(a, b, h, kt + 1, tid);
    if (wave_live) {
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + k_off_bf16(sub * 32 + r32, hh));
        kf[sub][1] = ld16(kl + k_off_bf16(sub * 32 + r32, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          vf[sub][ks] = ld16(vl + r32 * VROW + (2 * sub + ks) * 32 + hh * 16);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        f32x16 s0, s1;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x16& s = sub ? s1 : s0;
          s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[g][0], negm[g]);
          s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[g][1], s);
        }
        const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
        if (kt == 0 || __any(mx > RESCALE_SLACK)) {
          const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
          if (kt != 0) {
            const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
            for (int r = 0; r < 16; ++r) o[g][r] *= alpha;
            ls[g] *= alpha;
          }
          m[g] += d;
#pragma unroll
          for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[g][r] = -m[g]; }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
        float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
        for (int r = 0; r < 16; r += 2) { t0 += s0[r]; t1 += s0[r + 1]; t2 += s1[r]; t3 += s1[r + 1]; }
        ls[g] += (t0 + t1) + (t2 + t3);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x16& p = (i >> 1) ? s1 : s0;
          const int ks = i & 1;
          u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                   A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
          o[g] = A::mfma(__builtin_bit_cast(v8, vf[i >> 1][i & 1]), __builtin_bit_cast(v8, pw), o[g]);
        }
      }
    }
    if (more) st.store(smem + ((kt + 1) & 1) * SLOT, smem + ((kt + 1) & 1) * SLOT + KBYTES, tid);
    __syncthreads();
  }
  if (!wave_live) return;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int q = q0 + 32 * g;
    const float inv = 1.f / (ls[g] + __shfl_xor(ls[g], 32, 64));
    if (q >= a.Tq) continue;
    bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int d0 = 8 * j + 4 * hh;
      st8(op + d0, u32x2{pack_bf16x2(o[g][4 * j] * inv, o[g][4 * j + 1] * inv),
                         pack_bf16x2(o[g][4 * j + 2] * inv, o[g][4 * j + 3] * inv)});
    }
  }
}

// ---------------------------------------------------------------- variant v6
// Row sums off the matrix pipe (LSM 1: f32 adds, 2: v_dot2_f32_bf16 on the packed P) and, with
// STALE, no max chain on full tiles after the first: p = exp2(s - m) against the running max,
// and only if a lane's partial row sum of the tile reaches 2^64 (or is not finite) the tile is
// recomputed exactly and the accumulators rescaled.
template <int LSM, bool STALE, int OCC>
__global__ __launch_bounds__(NT, OCC) void attn_v6_kernel(AttnArgs a) {
  typedef AT<bf16> A;
  typedef A::v8 v8;
  constexpr int KBYTES = KT * KROW, VBYTES = 32 * VROW;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;
  v8 qf[2];
  {
    const float sl2 = a.scale * LOG2E;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<bf16>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[i] = __builtin_bit_cast(v8, pack16<bf16>(f));
    }
  }
  f32x16 o, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, ls = 0.f;
  const int ntiles = (a.Tk + KT - 1) / KT;
  const int nfull = a.Tk / KT;
  constexpr int SLOT = KBYTES + VBYTES;
  Stage<bf16, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + (kt & 1) * SLOT;
    const char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if (more) st.load(a, b, h, kt + 1, tid);
    if (wave_live) {
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + k_off_bf16(sub * 32 + r32, hh));
        kf[sub][1] = ld16(kl + k_off_bf16(sub * 32 + r32, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          vf[sub][ks] = ld16(vl + r32 * VROW + (2 * sub + ks) * 32 + hh * 16);
      f32x16 s0, s1;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], negm);
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
      }
      u32x4 pw[4];
      float tsum = 0.f;
      auto finish = [&]() {       // exp2, pack, partial row sum of this lane's 32 keys
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
        if constexpr (LSM == 1) {
          float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
          for (int r = 0; r < 16; r += 2) { t0 += s0[r]; t1 += s0[r + 1]; t2 += s1[r]; t3 += s1[r + 1]; }
          tsum = (t0 + t1) + (t2 + t3);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x16& p = (i >> 1) ? s1 : s0;
          const int ks = i & 1;
          pw[i] = u32x4{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                        A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
        }
        if constexpr (LSM == 2) {
          // inline asm: hipcc (ROCm 7.2) folds __builtin_amdgcn_fdot2_f32_bf16 calls on different
          // vector elements into one (observed: half the dot2s read the same register)
          float t0 = 0.f, t1 = 0.f;
          const uint32_t one2 = 0x3F803F80u;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; j += 2) {
              asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(t0) : "v"(pw[i][j]), "v"(one2));
              asm volatile("v_dot2_f32_bf16 %0, %1, %2, %0" : "+v"(t1) : "v"(pw[i][j + 1]), "v"(one2));
            }
          tsum = t0 + t1;
        }
      };
      bool exact = !STALE || kt == 0 || kt >= nfull;
      if (!exact) {
        finish();
        if (__any(!(tsum < SUM_LIMIT))) {      // rare: recompute this tile with the exact max
          exact = true;
#pragma unroll
          for (int sub = 0; sub < 2; ++sub) {
            f32x16& s = sub ? s1 : s0;
            s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], negm);
            s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
          }
        }
      }
      if (exact) {
        const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);     // relative to m
        if (kt == 0 || __any(mx > (STALE ? 0.f : RESCALE_SLACK))) {
          const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
          if (kt != 0) {
            const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
            for (int r = 0; r < 16; ++r) o[r] *= alpha;
            ls *= alpha;
          }
          m += d;
#pragma unroll
          for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
        }
        finish();
      }
      ls += tsum;
#pragma unroll
      for (int i = 0; i < 4; ++i) o = A::mfma(__builtin_bit_cast(v8, vf[i >> 1][i & 1]), __builtin_bit_cast(v8, pw[i]), o);
    }
    if (more) st.store(smem + ((kt + 1) & 1) * SLOT, smem + ((kt + 1) & 1) * SLOT + KBYTES, tid);
    __syncthreads();
  }
  if (!wave_live || q >= a.Tq) return;
  const float inv = 1.f / (ls + __shfl_xor(ls, 32, 64));
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}

// ---------------------------------------------------------------- variant v7
// v4.add with one barrier per TWO 64-key tiles: the LDS slot of a step holds tiles 2j and 2j+1;
// tile 2j+2 is loaded before tile 2j's compute and stored after it, tile 2j+3 likewise around
// tile 2j+1's compute (the other slot was released by the previous barrier), then one barrier.
template <int OCC>
__global__ __launch_bounds__(NT, OCC) void attn_v7_kernel(AttnArgs a) {
  typedef AT<bf16> A;
  typedef A::v8 v8;
  constexpr int KBYTES = KT * KROW, VBYTES = 32 * VROW, TILE = KBYTES + VBYTES, SLOT = 2 * TILE;
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;
  v8 qf[2];
  {
    const float sl2 = a.scale * LOG2E;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<bf16>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[i] = __builtin_bit_cast(v8, pack16<bf16>(f));
    }
  }
  f32x16 o, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, ls = 0.f;
  const int ntiles = (a.Tk + KT - 1) / KT;
  Stage<bf16, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  if (ntiles > 1) {
    st.load(a, b, h, 1, tid);
    st.store(smem + TILE, smem + TILE + KBYTES, tid);
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + ((kt >> 1) & 1) * SLOT + (kt & 1) * TILE;
    const char* vl = kl + KBYTES;
    const bool more = kt + 2 < ntiles;
    if (more) st.load(a, b, h, kt + 2, tid);
    if (wave_live) {
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + k_off_bf16(sub * 32 + r32, hh));
        kf[sub][1] = ld16(kl + k_off_bf16(sub * 32 + r32, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          vf[sub][ks] = ld16(vl + r32 * VROW + (2 * sub + ks) * 32 + hh * 16);
      f32x16 s0, s1;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], negm);
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
      }
      const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
      if (kt == 0 || __any(mx > RESCALE_SLACK)) {
        const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
        if (kt != 0) {
          const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int r = 0; r < 16; ++r) o[r] *= alpha;
          ls *= alpha;
        }
        m += d;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
      float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r += 2) { t0 += s0[r]; t1 += s0[r + 1]; t2 += s1[r]; t3 += s1[r + 1]; }
      ls += (t0 + t1) + (t2 + t3);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x16& p = (i >> 1) ? s1 : s0;
        const int ks = i & 1;
        u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
                 A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
        o = A::mfma(__builtin_bit_cast(v8, vf[i >> 1][i & 1]), __builtin_bit_cast(v8, pw), o);
      }
    }
    if (more) {
      char* dst = smem + (((kt + 2) >> 1) & 1) * SLOT + (kt & 1) * TILE;
      st.store(dst, dst + KBYTES, tid);
    }
    if (kt & 1) __syncthreads();
  }
  if (!wave_live || q >= a.Tq) return;
  const float inv = 1.f / (ls + __shfl_xor(ls, 32, 64));
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}
// ---------------------------------------------------------------- variant v3 (no LDS)
// K and V^T pre-tiled in global memory in MFMA fragment order: per (b, h, 64-key tile) eight
// 1 KiB chunks [sub][c][lane][8] (K) and [sub][ks][lane][8] (V^T); every wave streams its own
// fragments with fully coalesced 16-B loads one tile ahead (L1/L2 shared by the workgroup's
// waves), so there is no LDS staging and no barrier.
struct TiledArgs { const void* kt; const void* vt; };
__global__ __launch_bounds__(NT, SPE_ATTN_OCC) void attn_v3_kernel(AttnArgs a, TiledArgs t) {
  typedef AT<bf16> A;
  typedef A::v8 v8;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  if (qb * 128 + wid * 32 >= a.Tq) return;
  v8 qf[2];
  {
    const float sl2 = a.scale * LOG2E;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      unpack16<bf16>(q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0}, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] *= sl2;
      qf[i] = __builtin_bit_cast(v8, pack16<bf16>(f));
    }
  }
  u32x4 ones_u{A::ONE2, A::ONE2, A::ONE2, A::ONE2};
  asm volatile("" : "+v"(ones_u));
  const v8 ones = __builtin_bit_cast(v8, ones_u);
  f32x16 o, ls, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; ls[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f;
  const int ntiles = (a.Tk + KT - 1) / KT;
  const u32x4* kg = (const u32x4*)t.kt + (size_t)(b * a.H + h) * ntiles * 4 * 64 + lane;
  const u32x4* vg = (const u32x4*)t.vt + (size_t)(b * a.H + h) * ntiles * 4 * 64 + lane;
  u32x4 kf[4], vf[4], kn[4], vn[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { kf[i] = kg[i * 64]; vf[i] = vg[i * 64]; }
  for (int kt = 0; kt < ntiles; ++kt) {
    if (kt + 1 < ntiles) {
#pragma unroll
      for (int i = 0; i < 4; ++i) { kn[i] = kg[(kt + 1) * 256 + i * 64]; vn[i] = vg[(kt + 1) * 256 + i * 64]; }
    }
    f32x16 s0, s1;
    s0 = A::mfma(__builtin_bit_cast(v8, kf[0]), qf[0], negm);
    s0 = A::mfma(__builtin_bit_cast(v8, kf[1]), qf[1], s0);
    s1 = A::mfma(__builtin_bit_cast(v8, kf[2]), qf[0], negm);
    s1 = A::mfma(__builtin_bit_cast(v8, kf[3]), qf[1], s1);
    const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
    if (kt == 0 || __any(mx > RESCALE_SLACK)) {
      const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
      if (kt != 0) {
        const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
        for (int r = 0; r < 16; ++r) { o[r] *= alpha; ls[r] *= alpha; }
      }
      m += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) { s0[r] = __builtin_amdgcn_exp2f(s0[r]); s1[r] = __builtin_amdgcn_exp2f(s1[r]); }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const f32x16& p = (i >> 1) ? s1 : s0;
      const int ks = i & 1;
      u32x4 pw{A::pk(p[8 * ks + 0], p[8 * ks + 1]), A::pk(p[8 * ks + 2], p[8 * ks + 3]),
               A::pk(p[8 * ks + 4], p[8 * ks + 5]), A::pk(p[8 * ks + 6], p[8 * ks + 7])};
      const v8 pb = __builtin_bit_cast(v8, pw);
      o = A::mfma(__builtin_bit_cast(v8, vf[i]), pb, o);
      ls = A::mfma(ones, pb, ls);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) { kf[i] = kn[i]; vf[i] = vn[i]; }
  }
  if (q >= a.Tq) return;
  const float inv = 1.f / ls[0];
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}

}  // namespace

// ---------------------------------------------------------------- host
static uint32_t lcg(uint64_t& s) {
  s = s * 6364136223846793005ull + 1442695040888963407ull;
  return (uint32_t)(s >> 33);
}
static float gauss(uint64_t& s) {
  float u1 = (lcg(s) + 1.0f) / 2147483649.0f, u2 = lcg(s) / 2147483648.0f;
  return std::sqrt(-2.f * std::log(u1)) * std::cos(6.2831853f * u2);
}
static uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}
static float from_bf16(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

typedef void (*Launch)(const AttnArgs&, hipStream_t);
static void launch_prod(const AttnArgs& a, hipStream_t s) { spe_launch_attention(a, SPE_DTYPE_BF16, s); }
static TiledArgs g_tiled;
static void launch_v3(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(attn_v3_kernel, dim3(a.B * a.H * ((a.Tq + 127) / 128)), dim3(NT), 0, s, a, g_tiled);
}
template <int LSM> static void launch_v4(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(attn_v4_kernel<LSM>, dim3(a.B * a.H * ((a.Tq + 127) / 128)), dim3(NT), 0, s, a);
}
template <int G, int OCC> static void launch_v5(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_v5_kernel<G, OCC>), dim3(a.B * a.H * ((a.Tq + 128 * G - 1) / (128 * G))), dim3(NT), 0, s, a);
}
template <int LSM, bool STALE, int OCC> static void launch_v6(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_v6_kernel<LSM, STALE, OCC>), dim3(a.B * a.H * ((a.Tq + 127) / 128)), dim3(NT), 0, s, a);
}
template <int OCC> static void launch_v7(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((attn_v7_kernel<OCC>), dim3(a.B * a.H * ((a.Tq + 127) / 128)), dim3(NT), 0, s, a);
}
static void launch_v2(const AttnArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(attn_v2_kernel<bf16>, dim3(a.B * a.H * ((a.Tq + 127) / 128)), dim3(NT), 0, s, a);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 20;
  const int B = argc > 2 ? std::atoi(argv[2]) : 64;
  const int H = 8, T = 2704, D = 256;
  struct Variant { const char* name; Launch fn; };
  std::vector<Variant> vars = {{"prod", launch_prod}, {"v4.add", launch_v4<1>},
                               {"v7.o4", launch_v7<4>}, {"v7.o3", launch_v7<3>}};
  // scenarios: score scale (q multiplier) and whether keys are sorted by increasing score
  struct Scen { const char* name; float qmul; bool ramp; };
  std::vector<Scen> scens = {{"randn", 1.f, false}, {"wide x8", 8.f, false}, {"ramp x40", 40.f, true}};
  const size_t nqk = (size_t)B * T * 512, nv = (size_t)B * H * 32 * T, no = (size_t)B * T * D;
  std::vector<uint16_t> hqk(nqk), hv(nv);
  void *dqk, *dv, *dref, *dout;
  CHECK(hipMalloc(&dqk, nqk * 2));
  CHECK(hipMalloc(&dv, nv * 2));
  CHECK(hipMalloc(&dref, no * 2));
  CHECK(hipMalloc(&dout, no * 2));
  std::vector<uint16_t> href(no), hout(no);
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (const Scen& sc : scens) {
    uint64_t seed = 12345;
    for (size_t i = 0; i < nqk; ++i) {
      const size_t col = i % 512;
      float g = gauss(seed);
      if (sc.ramp && col >= 256) {          // keys: a shared direction growing along the sequence
        const size_t row = i / 512, t = row % T;
        g = 0.1f * g + (float)t / T * ((col & 31) == 0 ? 1.f : 0.f);
      }
      hqk[i] = to_bf16(col < 256 ? g * sc.qmul * (sc.ramp ? ((col & 31) == 0 ? 1.f : 0.02f) : 1.f) : g);
    }
    for (size_t i = 0; i < nv; ++i) hv[i] = to_bf16(gauss(seed));
    CHECK(hipMemcpy(dqk, hqk.data(), nqk * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dv, hv.data(), nv * 2, hipMemcpyHostToDevice));
    {   // fragment-ordered copies for v3 (zero-padded past T)
      const int ntiles = (T + 63) / 64;
      const size_t per = (size_t)ntiles * 4 * 64 * 8;
      std::vector<uint16_t> tk((size_t)B * H * per, 0), tv((size_t)B * H * per, 0);
      for (int bb = 0; bb < B; ++bb)
        for (int hd = 0; hd < H; ++hd)
          for (int kt = 0; kt < ntiles; ++kt)
            for (int i = 0; i < 4; ++i)
              for (int ln = 0; ln < 64; ++ln)
                for (int e = 0; e < 8; ++e) {
                  const int r32 = ln & 31, hh = ln >> 5, sub = i >> 1, c = i & 1;
                  const size_t dst = (((size_t)(bb * H + hd) * ntiles + kt) * 4 + i) * 512 + ln * 8 + e;
                  const int key = kt * 64 + sub * 32 + r32, dim = (2 * c + hh) * 8 + e;
                  if (key < T) tk[dst] = hqk[((size_t)bb * T + key) * 512 + 256 + hd * 32 + dim];
                  const int g = i, vkey = kt * 64 + g * 16 + (e & 3) + 8 * (e >> 2) + 4 * hh;
                  if (vkey < T) tv[dst] = hv[((size_t)(bb * H + hd) * 32 + r32) * T + vkey];
                }
      if (!g_tiled.kt) {
        CHECK(hipMalloc((void**)&g_tiled.kt, tk.size() * 2));
        CHECK(hipMalloc((void**)&g_tiled.vt, tv.size() * 2));
      }
      CHECK(hipMemcpy((void*)g_tiled.kt, tk.data(), tk.size() * 2, hipMemcpyHostToDevice));
      CHECK(hipMemcpy((void*)g_tiled.vt, tv.data(), tv.size() * 2, hipMemcpyHostToDevice));
    }
    AttnArgs a{};
    a.q = dqk; a.ldq = 512; a.k = (char*)dqk + 512; a.ldk = 512; a.vt = dv; a.ldo = D;
    a.B = B; a.H = H; a.Tq = T; a.Tk = T; a.scale = 1.f / std::sqrt(32.f);
    std::printf("== %s (B=%d)\n", sc.name, B);
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      a.o = vi == 0 ? dref : dout;
      CHECK(hipMemsetAsync(a.o, 0xFF, no * 2, st));
      vars[vi].fn(a, st);
      CHECK(hipStreamSynchronize(st));
      CHECK(hipGetLastError());
      double err = 0, mean = 0;
      long nan = 0;
      if (vi > 0) {
        CHECK(hipMemcpy(hout.data(), dout, no * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < no; ++i) {
          const float x = from_bf16(hout[i]), r = from_bf16(href[i]);
          if (!std::isfinite(x)) { ++nan; continue; }
          const double d = std::fabs(x - r);
          err = std::max(err, d);
          mean += d;
        }
        mean /= no;
      } else {
        CHECK(hipMemcpy(href.data(), dref, no * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < no; ++i) nan += !std::isfinite(from_bf16(href[i]));
      }
      CHECK(hipEventRecord(e0, st));
      for (int it = 0; it < iters; ++it) vars[vi].fn(a, st);
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      ms /= iters;
      const double fl = 4.0 * B * H * (double)T * T * 32;
      std::printf("%-8s %.4f ms  %7.1f TF/s  max|d|=%.3g mean|d|=%.3g nonfinite=%ld\n", vars[vi].name, ms,
                  fl / ms / 1e9, err, mean, nan);
    }
  }
  return 0;
}
