// Decoder cross-attention of the bf16 path, computed against the encoder memory itself.
//
// Reference: TransformerDecoderLayer.forward_post, multihead_attn(query = tgt + query_pos,
// key = memory + pos, value = memory) (REV/models/transformer.py:230-233), i.e. per head h
//     o_h = softmax(scale . q_h . K_h^T) V_h,   q_h = Wq_h x + bq_h, K_h = Wk_h (mem + pos) + bk_h,
//                                               V_h = Wv_h mem + bv_h.
// The memory is the same for all six decoder layers and has T = (S/8)^2 = 2704 tokens, while
// the queries are only Q = 11 per image, so instead of projecting the memory to K and V for
// every layer (2 x 6 x T x 256 x 256 MACs per image), both projections move to the query side:
//     scores_h = (Wk_h^T q_h) . (mem + pos)      (the bk term is constant per row: softmax-invariant)
//     o_h      = Wv_h (sum_t p_t mem_t) + bv_h   (sum_t p_t = 1)
// so a layer needs q'_h = Wk_h^T q_h (256 wide, per query and head: one small GEMM with
// Wq/Wk folded, registry.cpp fold_cross_attention) and u_h = softmax(q'_h . (mem+pos)^T) . mem,
// which is this file, followed by o_h = Wv_h u_h + bv_h (in the split-merge kernel) and the
// layer's unchanged output projection.
//
// xattn_kernel: one workgroup = (image, key split, group of up to 96 attention rows), rows
// r = q * 8 + h; 8 waves: two loader waves stage each 32-key tile (the K rows [32][256] of
// memory+pos and the V rows [32][256] of the memory, contiguous 16 KB reads, global_load_lds
// into XOR-swizzled LDS through a four-stage ring: three tiles in flight while one is consumed,
// one barrier per tile), and three wave pairs each own 32 rows, each wave of a pair 128 of the
// 256 value dims.  Per tile every compute wave runs
//   S^T = K . Q'^T (32x32x16 bf16 MFMAs, K = 256, two accumulation chains), online softmax in
//   the exp2 domain (q' is pre-scaled by scale * log2 e), and U^T[d][row] += V^T[d][keys] . P^T
//   for its dims, P^T taken straight from the score registers (its key order is the
//   accumulator's) and V^T read transposed out of the row-major V tile by ds_read_b64_tr_b16
//   in that same key order.
// Each key split writes fp32 partials (m, l, unnormalised U) that a merge kernel combines.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int NT = 512, KT = 32, RG = 96, D = 256;   // RG: rows per workgroup (3 wave pairs)
constexpr int KTILE = KT * D * 2;               // 16 KB: K rows [key][256] (512 B rows)
constexpr int VTILE = KT * D * 2;               // 16 KB: V rows [key][256] (512 B rows)
constexpr int STAGE = KTILE + VTILE;
#ifndef SPE_XATTN_STAGES
#define SPE_XATTN_STAGES 4
#endif
constexpr int NSTAGE = SPE_XATTN_STAGES;        // ring: tile t in use, t+1 .. t+NSTAGE-1 in flight
constexpr int LDS_BYTES = NSTAGE * STAGE;
static_assert(NSTAGE >= 3 && NSTAGE <= 5, "ring: 3..5 slots (160 KB of LDS)");
constexpr int LOADS = STAGE / 1024 / 2;         // glds per loader wave per tile
constexpr int DB = 4;                           // 32-dim blocks of U per wave
constexpr float NEG_BIG = -1.0e30f;
constexpr float SLACK = 8.0f;                   // lazy rescale threshold (log2 units), as attention.hip

__device__ __attribute__((aligned(64))) uint32_t g_xzero[16];

typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int N>
SPE_DEV void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// K tile: chunk c of key row k at slot c ^ (k & 15) (the 16 keys of a ds_read_b128 lane group
// hit distinct bank groups).  V tile: chunk c at slot c ^ ((k & 3) << 2), so the four key rows
// of every ds_read_b64_tr_b16 block fall in four different 64-byte bank segments.
SPE_DEV int kkey(int key) { return key & 15; }
SPE_DEV int vkey(int key) { return (key & 3) << 2; }
SPE_DEV int k_off(int key, int c) { return key * 512 + ((c ^ kkey(key)) << 4); }
SPE_DEV int v_off(int key, int c) { return key * 512 + ((c ^ vkey(key)) << 4); }

// 4 keys x 16 dims of the V tile, delivered transposed: lane i of each 16-lane group gets dim
// d0 + i of keys k0 .. k0+3 (cdna_hip_programming.md T10); lane 4q+p addresses key k0+q, dims
// d0 + 4p .. +3 (d0 % 16 == 0).  LDS byte address of this lane's block row:
SPE_DEV uint32_t v_tr_addr(uint32_t vbase, int k0, int d0, int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  return vbase + v_off(k0 + q, (d0 >> 3) + (p >> 1)) + 8 * (p & 1);
}
// Issued as inline asm: the compiler treats the ds_read_b64_tr_b16 builtin as aliasing the
// tiles still in flight by LDS-DMA and drains them (vmcnt(0)) before it; the waits for these
// reads are therefore explicit (lgkmcnt + sched_barrier, cdna_hip_programming.md rule 18).
SPE_DEV u32x2 ds_read_tr(uint32_t addr) {
  u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

__global__ __launch_bounds__(NT, 1) void xattn_kernel(XattnArgs a) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hh = lane >> 5, r32 = lane & 31, l16 = lane & 15, dg = 16 * ((lane >> 4) & 1);
  const int R = 8 * a.Q, ngroups = (R + RG - 1) / RG;
  int bid = blockIdx.x;
  const int grp = bid % ngroups; bid /= ngroups;
  const int split = bid % a.splits;
  const int b = bid / a.splits;
  const int row0 = grp * RG, nrows = min(RG, R - row0);
  const int ntiles = (a.T + KT - 1) / KT;
  const int tb = split * a.tiles_per_split, te = min(ntiles, tb + a.tiles_per_split);

  // ---- roles.  Waves 6 and 7 only stage the K and V tiles (the DMA issue is not cheap beside
  // LDS reads and MFMAs).  Compute wave pair (2 rb, 2 rb + 1): rows 32 rb .. +32, dims
  // 128 dh .. +128 of U; each wave of the pair computes the scores of its rows itself (two
  // waves per SIMD, no P exchange).  q' B fragments for all 16 K-steps of 16 dims.
  const bool loader = wid >= 6;
  const int rb = wid >> 1, dh = wid & 1;
  const bool live_wave = !loader && rb * 32 < nrows;
  const int my_row = rb * 32 + r32;             // row within the group
  bf16x8 qf[16];
  {
    const int r = row0 + my_row;
    const bool live = live_wave && my_row < nrows;
    const bf16* qp = (const bf16*)a.q + (size_t)(b * a.Q + (live ? r >> 3 : 0)) * a.ldq + (live ? (r & 7) : 0) * D;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      qf[ks] = __builtin_bit_cast(bf16x8, live ? ld16(qp + 16 * ks + 8 * hh) : u32x4{0, 0, 0, 0});
  }

  // ---- staging (loader waves): wave 6 the K tile, wave 7 the V tile,
  // 16 x 1 KB each (2 key rows per instruction)
  const char* zero = reinterpret_cast<const char*>(g_xzero);
  const bool isv = wid == 7;
  const char* src0 = isv ? (const char*)a.v : (const char*)a.k;
  const int ldsrc = isv ? a.ldv : a.ldk;
  auto issue = [&](int t, int buf) {
    char* st = lds + buf * STAGE + (isv ? KTILE : 0);
    const int key0 = t * KT;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = 2 * i + (lane >> 5), s = lane & 31;
      const int c = s ^ (isv ? vkey(key) : kkey(key));
      const int row = b * a.T + key0 + key;
      const char* src = key0 + key < a.T ? src0 + ((size_t)row * ldsrc + c * 8) * 2 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + i * 1024), 16, 0, 0);
    }
  };

  // ---- state: negm (-m in every element: the score MFMAs start from it), m, l per row, and
  // U^T[32 db + i][row] for the 8 blocks of 32 dims
  f32x16 negm, acc[DB];
#pragma unroll
  for (int r = 0; r < 16; ++r) negm[r] = 0.f;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;
  float m = 0.f, l = 0.f;

  // the q' loads must retire before the DMA stream starts (vmcnt is in-order; see ffn.hip)
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) asm volatile("" ::"v"(qf[ks]));
  const int nt = te - tb;
  auto tile_at = [&](int i) { return tb + i; };
  // NSTAGE-slot ring: tiles t+1..t+NSTAGE-1 stay in flight while tile t is consumed; the slot of
  // tile t+NSTAGE-1 is refilled once every wave has passed tile t's barrier (it held tile t-1).
  if (loader) {
#pragma unroll
    for (int i = 0; i < NSTAGE - 1; ++i)
      if (tb + i < te) issue(tile_at(i), i);
  }
  for (int it = 0; it < nt; ++it) {
    const int t = tile_at(it), buf = it % NSTAGE;
    if (loader) {
      // tile t landed; the (up to NSTAGE - 2) newer tiles may stay in flight
      const int newer = min(NSTAGE - 2, nt - 1 - it);
      if (newer >= 3) wait_vmcnt<3 * LOADS>();
      else if (newer == 2) wait_vmcnt<2 * LOADS>();
      else if (newer == 1) wait_vmcnt<LOADS>();
      else wait_vmcnt<0>();
    }
    // raw barrier (__syncthreads' fence would drain the tiles in flight): tile t visible to
    // all, every wave done with tile t-1
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (loader) {
      if (it + NSTAGE - 1 < nt) issue(tile_at(it + NSTAGE - 1), (buf + NSTAGE - 1) % NSTAGE);
      continue;
    }
    if (!live_wave) continue;
    const char* kl = lds + buf * STAGE;
    const char* vl = kl + KTILE;

    // S^T - m: lane (row r32, hh) register r <-> key (r & 3) + 8 (r >> 2) + 4 hh
    f32x16 s;
    {
      f32x16 sa, sb;
#pragma unroll
      for (int ks = 0; ks < 16; ks += 2) {
        const bf16x8 k0 = __builtin_bit_cast(bf16x8, ld16(kl + k_off(r32, 2 * ks + hh)));
        const bf16x8 k1 = __builtin_bit_cast(bf16x8, ld16(kl + k_off(r32, 2 * ks + 2 + hh)));
        if (ks == 0) {
          sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, qf[ks], negm, 0, 0, 0);
          sb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, qf[ks + 1], f32x16{}, 0, 0, 0);
        } else {
          sa = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k0, qf[ks], sa, 0, 0, 0);
          sb = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k1, qf[ks + 1], sb, 0, 0, 0);
        }
      }
      s = sa + sb;
    }
    const int key_base = t * KT;
    if (key_base + KT > a.T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key_base + (r & 3) + 8 * (r >> 2) + 4 * hh >= a.T) s[r] = NEG_BIG;
    }
    float mq[4];                                // max tree (v_max3), then lane <-> lane^32
#pragma unroll
    for (int i = 0; i < 4; ++i)
      mq[i] = __builtin_fmaxf(__builtin_fmaxf(s[4 * i], s[4 * i + 1]), __builtin_fmaxf(s[4 * i + 2], s[4 * i + 3]));
    float mx = __builtin_fmaxf(__builtin_fmaxf(mq[0], mq[1]), __builtin_fmaxf(mq[2], mq[3]));
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
      mx = __builtin_fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    if (it == 0 || __any(mx > SLACK)) {
      const float d = it == 0 ? mx : __builtin_fmaxf(mx, 0.f);
      if (it != 0) {
        const float alpha = __builtin_amdgcn_exp2f(-d);
        l *= alpha;
#pragma unroll
        for (int db = 0; db < DB; ++db)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[db][r] *= alpha;
      }
      m += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s[r] -= d; negm[r] = -m; }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(s[r]);
    {
      float lq[4];                              // row-sum tree
#pragma unroll
      for (int i = 0; i < 4; ++i) lq[i] = (s[4 * i] + s[4 * i + 1]) + (s[4 * i + 2] + s[4 * i + 3]);
      l += (lq[0] + lq[1]) + (lq[2] + lq[3]);
    }
    // P^T B operands: element e of K-step ks is register 8 ks + e, i.e. key
    // 16 ks + 4 hh + 8 (e >> 2) + (e & 3); the V^T A operand is read in that order
    bf16x8 pb[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      pb[ks] = __builtin_bit_cast(bf16x8, u32x4{pack_bf16x2(s[8 * ks], s[8 * ks + 1]), pack_bf16x2(s[8 * ks + 2], s[8 * ks + 3]),
                                                pack_bf16x2(s[8 * ks + 4], s[8 * ks + 5]), pack_bf16x2(s[8 * ks + 6], s[8 * ks + 7])});
    // V^T fragments of dim block db: reads [ks][lo/hi]; block db+1's reads are in flight while
    // block db multiplies
    const uint32_t vbase = (uint32_t)(uintptr_t)(lds_ptr_t)vl;
    u32x2 vr[2][4];
    auto read_v = [&](u32x2 (&r)[4], int db) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        r[2 * ks] = ds_read_tr(v_tr_addr(vbase, 16 * ks + 4 * hh, 128 * dh + 32 * db + dg, l16));
        r[2 * ks + 1] = ds_read_tr(v_tr_addr(vbase, 16 * ks + 8 + 4 * hh, 128 * dh + 32 * db + dg, l16));
      }
    };
    read_v(vr[0], 0);
#pragma unroll
    for (int db = 0; db < DB; ++db) {
      if (db < DB - 1) {
        read_v(vr[(db + 1) & 1], db + 1);
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      const u32x2(&r)[4] = vr[db & 1];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        acc[db] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            __builtin_bit_cast(bf16x8, u32x4{r[2 * ks].x, r[2 * ks].y, r[2 * ks + 1].x, r[2 * ks + 1].y}), pb[ks],
            acc[db], 0, 0, 0);
    }
  }
  if (!live_wave) return;
  // ---- partials: m, l (summed over the two lane halves) and the unnormalised U^T rows; lane
  // holds U^T[d = 32 db + 8 (r>>2) + 4 hh + (r&3)][row r32]
  l += __shfl_xor(l, 32, 64);
  if (my_row >= nrows) return;
  const size_t pr = ((size_t)b * a.splits + split) * R + row0 + my_row;
  if (hh == 0 && dh == 0) {
    a.pm[pr] = m;
    a.pl[pr] = l;
  }
  float* pu = a.pu + pr * D;
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = {acc[db][4 * g], acc[db][4 * g + 1], acc[db][4 * g + 2], acc[db][4 * g + 3]};
      st16(pu + 128 * dh + 32 * db + 8 * g + 4 * hh, __builtin_bit_cast(u32x4, v));
    }
}

// merge of the key splits for one row: weight of split s = 2^(m_s - M)
struct Merge {
  float M, L;
};
SPE_DEV Merge merge_stats(const XattnArgs& a, int b, int r, int R) {
  float M = NEG_BIG;
  for (int s = 0; s < a.splits; ++s) M = fmaxf(M, a.pm[((size_t)b * a.splits + s) * R + r]);
  float L = 0.f;
  for (int s = 0; s < a.splits; ++s) {
    const size_t pr = ((size_t)b * a.splits + s) * R + r;
    L += __builtin_amdgcn_exp2f(a.pm[pr] - M) * a.pl[pr];
  }
  return {M, L};
}

// u = sum_s 2^(m_s - M) U_s / sum_s 2^(m_s - M) l_s, stored as is (one wave per row)
__global__ __launch_bounds__(256) void xattn_merge_u_kernel(XattnArgs a) {
  const int lane = threadIdx.x & 63, R = 8 * a.Q;
  const int br = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (br >= a.B * R) return;
  const int b = br / R, r = br - b * R;
  const Merge mg = merge_stats(a, b, r, R);
  f32x4 u = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < a.splits; ++s) {
    const size_t pr = ((size_t)b * a.splits + s) * R + r;
    u += __builtin_amdgcn_exp2f(a.pm[pr] - mg.M) * *reinterpret_cast<const f32x4*>(a.pu + pr * D + 4 * lane);
  }
  u *= 1.f / mg.L;
  bf16* up = (bf16*)a.u + (size_t)(b * a.Q + (r >> 3)) * a.ldu + (r & 7) * D + 4 * lane;
  st8(up, u32x2{pack_bf16x2(u[0], u[1]), pack_bf16x2(u[2], u[3])});
}

// Merge + value projection, o_h[j] = Wv[h*32 + j] . u_h + bv[h*32 + j] (the reference's V
// projection moved past the probability-weighted sum, which it commutes with since the
// probabilities sum to one).  Block = (16 query rows (b, q), head h): Wv_h [32][256] and the
// 16 merged u_h rows staged in LDS as fp32 (rows padded to 257 floats: the 16 threads sharing a
// u row read 16 different Wv rows on 16 different banks), 2 outputs per thread.
constexpr int MR = 16, WP = D + 1;
__global__ __launch_bounds__(256) void xattn_merge_wv_kernel(XattnArgs a) {
  __shared__ float wvs[32 * WP];
  __shared__ float us[MR * WP];
  const int tid = threadIdx.x, R = 8 * a.Q, h = blockIdx.y, bq0 = blockIdx.x * MR;
  const bf16* wv = (const bf16*)a.wv + (size_t)h * 32 * D;
#pragma unroll
  for (int i = 0; i < 4; ++i) {                 // 32 x 256 bf16 = 1024 chunks of 8
    const int idx = tid + i * 256, j = idx >> 5, c = idx & 31;
    float f[8];
    unpack16<bf16>(ld16(wv + (size_t)j * D + 8 * c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) wvs[j * WP + 8 * c + e] = f[e];
  }
  {
    const int i = tid >> 4, d0 = 16 * (tid & 15), bq = bq0 + i;
    float u[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) u[e] = 0.f;
    if (bq < a.B * a.Q) {
      const int b = bq / a.Q, r = (bq - b * a.Q) * 8 + h;
      const Merge mg = merge_stats(a, b, r, R);
      for (int s = 0; s < a.splits; ++s) {
        const size_t pr = ((size_t)b * a.splits + s) * R + r;
        const float w = __builtin_amdgcn_exp2f(a.pm[pr] - mg.M);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(a.pu + pr * D + d0 + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) u[4 * g + e] += w * v[e];
        }
      }
      const float inv = 1.f / mg.L;
#pragma unroll
      for (int e = 0; e < 16; ++e) u[e] *= inv;
    }
#pragma unroll
    for (int e = 0; e < 16; ++e) us[i * WP + d0 + e] = u[e];
  }
  __syncthreads();
  const int i = tid >> 4, j = 2 * (tid & 15), bq = bq0 + i;
  float o0 = a.bv[h * 32 + j], o1 = a.bv[h * 32 + j + 1];
  const float* ur = us + i * WP;
  const float* w0 = wvs + j * WP;
  const float* w1 = w0 + WP;
#pragma unroll 8
  for (int n = 0; n < D; ++n) {
    const float x = ur[n];
    o0 += x * w0[n];
    o1 += x * w1[n];
  }
  if (bq < a.B * a.Q)
    *reinterpret_cast<uint32_t*>((bf16*)a.o + (size_t)bq * a.ldo + h * 32 + j) = pack_bf16x2(o0, o1);
}

}  // namespace

int spe_xattn_splits(int B, int Q, int T) {
  const int groups = (8 * Q + RG - 1) / RG, ntiles = (T + KT - 1) / KT;
  int s = 1;
  while (s < ntiles && B * groups * s < 256) s *= 2;
  const int tps = (ntiles + s - 1) / s;
  return (ntiles + tps - 1) / tps;              // every split non-empty
}

int spe_xattn_launch_splits(int T, int splits) {
  const int ntiles = (T + KT - 1) / KT, tps = (ntiles + splits - 1) / splits;
  return (ntiles + tps - 1) / tps;              // no empty split (<= requested)
}

int spe_launch_xattn(const XattnArgs& a0, hipStream_t s) {
  XattnArgs a = a0;
  if (a.B <= 0) return 0;
  if (a.ldq % 8 || a.ldk % 8 || a.ldv % 8 || a.ldu % 8 || a.splits < 1 || a.T < 1) return -5;
  const int ntiles = (a.T + KT - 1) / KT;
  a.tiles_per_split = (ntiles + a.splits - 1) / a.splits;
  a.splits = spe_xattn_launch_splits(a.T, a.splits);
  if (!a.pm || !a.pl || !a.pu || (!a.partials_only && (a.wv ? !a.o || !a.bv || a.ldo % 2 : !a.u))) return -5;
  const int groups = (8 * a.Q + RG - 1) / RG;
  hipLaunchKernelGGL(xattn_kernel, dim3(a.B * a.splits * groups), dim3(NT), 0, s, a);
  if (a.partials_only) return (int)hipGetLastError();
  if (a.wv)
    hipLaunchKernelGGL(xattn_merge_wv_kernel, dim3((a.B * a.Q + MR - 1) / MR, 8), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(xattn_merge_u_kernel, dim3((a.B * 8 * a.Q + 3) / 4), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
