// Decoder cross-attention of the fp32h3 accuracy-contract model, computed against the encoder
// memory itself -- the fold of xattn.hip (header there) at fp32-level products.
//
// Reference: TransformerDecoderLayer.forward_post, multihead_attn(query = tgt + query_pos,
// key = memory + pos, value = memory) (REV/models/transformer.py:230-233).  Per head h
//     scores_h = (Wk_h^T q_h) . (mem + pos)     o_h = Wv_h (sum_t p_t mem_t) + bv_h
// with q'_h = Wk_h^T q_h from one GEMM over the folded Wqk (registry.cpp fold_cross_attention; the
// fp32h3 model keeps it fp32 and runs it on the h3 GEMM).  Before fold, the fp32h3 decoder projected
// the memory to K and V^T for all six layers (2 x 6 x T x 256 x 256 MACs per image, 2.1 GB written
// and read back per step at B = 64) and ran the exact-f32 attention over them.
//
// Operands.  xattn_h3_split_kernel writes the memory once per batch as fp16 planes, rows of 1 KB
// (hi 256 | lo 256): kp = (mem + pos) * 2^sk and vp = mem * 2^sv, hi = RNE(x), lo = RNE(x - hi)
// (x - hi exact in fp32), the powers of two from the memory's bound (the last encoder norm2's
// LayerNorm bound, vplane_scale: |mem + pos| <= bound + 1, every scaled |x| < 2^14).  q' is split in
// registers per row and per 128-dim half with its own 2^(13 - e).  Every product is three fp16
// MFMAs (hi.hi + hi.lo + lo.hi): ~2^-22 relative per product, the fp32h3 GEMMs' rule.
//
// xattn_h3_kernel: one work-group = (image, key split, group of up to 96 attention rows r = 8q + h);
// 8 waves: two loader waves stage each 32-key tile (K and V rows of 1 KB, global_load_lds into
// XOR-swizzled images, a two-stage ring: 2 x 64 KB), three wave pairs own 32 rows each.  Wave dh of a
// pair forms the partial scores S^T over dims [128 dh, 128 dh + 128) (8 K-steps x 3 MFMAs, its q'
// half as B fragments in registers), unscales them and trades them with its partner through LDS
// (one extra barrier per tile); both then hold the same sum (fp32 addition commutes), run the same
// online softmax (exp2 domain, lazy rescale) and U^T[d][row] += V^T . P^T for their 128 value dims,
// P split in registers (RTZ fp16 hi + RNE remainder, attn_split.hip), V^T read transposed by
// ds_read_b64_tr_b16 in the score accumulator's key order.  Each key split writes fp32 partials
// (m, l, unnormalised U); xattn_h3_merge_wv_kernel merges them, applies Wv_h / bv_h in fp32 and
// raises max |o| for the out-projection GEMM's scale.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int NT = 512, KT = 32, RG = 96, D = 256;
constexpr int ROW = 1024;                       // one key row of a plane image: hi 512 B | lo 512 B
constexpr int KTILE = KT * ROW;                 // 32 KB
constexpr int STAGE = 2 * KTILE;                // [K | V]
constexpr int NSTAGE = 2;
constexpr int XCH = 4096;                       // per-wave partial-score exchange: 16 floats x 64 lanes
constexpr int LDS_BYTES = NSTAGE * STAGE + 6 * XCH;   // 152 KB
constexpr int DB = 4;                           // 32-dim blocks of U per wave
constexpr float NEG_BIG = -1.0e30f;
constexpr float SLACK = 8.0f;                   // lazy rescale threshold (log2 units), as xattn.hip

__device__ __attribute__((aligned(64))) uint32_t g_x3zero[16];

typedef __attribute__((address_space(3))) void* lds_ptr_t;
SPE_DEV void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// K image: chunk c (16 B; hi 0-31, lo 32-63) of key row k at slot c ^ (k & 15); V image at slot
// c ^ ((k & 3) << 2) (xattn.hip's swizzles: the XOR leaves bit 5, so lo = hi + 512 B)
SPE_DEV int k_off(int key, int c) { return key * ROW + ((c ^ (key & 15)) << 4); }
SPE_DEV int v_off(int key, int c) { return key * ROW + ((c ^ ((key & 3) << 2)) << 4); }
SPE_DEV uint32_t v_tr_addr(uint32_t vbase, int k0, int d0, int lane16) {
  const int q = lane16 >> 2, p = lane16 & 3;
  return vbase + v_off(k0 + q, (d0 >> 3) + (p >> 1)) + 8 * (p & 1);
}
SPE_DEV u32x2 ds_read_tr(uint32_t addr) {
  u32x2 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
SPE_DEV f32x16 mfma_h(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// the memory planes' powers of two (producer and consumer evaluate the same expressions)
SPE_DEV float k_scale(const float* mem_amax) { return vplane_scale(mem_amax, 1.f, 1.f); }
SPE_DEV float v_scale(const float* mem_amax) { return vplane_scale(mem_amax, 1.f, 0.f); }

__global__ __launch_bounds__(256) void xattn_h3_split_kernel(const float* __restrict__ mem, const float* __restrict__ pos,
                                                             const float* mem_amax, uint16_t* __restrict__ kp,
                                                             uint16_t* __restrict__ vp, int B, int T) {
  const float sk = k_scale(mem_amax), sv = v_scale(mem_amax);
  const size_t n4 = (size_t)B * T * (D / 4);
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const size_t row = i / (D / 4);
    const int c = (int)(i % (D / 4)), t = (int)(row % T);
    float x[4], p[4], kx[4], vx[4];
    unpack16<float>(ld16(mem + row * D + 4 * c), x);
    unpack16<float>(ld16(pos + (size_t)t * D + 4 * c), p);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      kx[e] = (x[e] + p[e]) * sk;                 // the reference's fp32 memory + pos, then 2^sk (exact)
      vx[e] = x[e] * sv;
    }
    u32x2 h, l;
    split_f16x4(kx, h, l);
    st8(kp + row * 2 * D + 4 * c, h);
    st8(kp + row * 2 * D + D + 4 * c, l);
    split_f16x4(vx, h, l);
    st8(vp + row * 2 * D + 4 * c, h);
    st8(vp + row * 2 * D + D + 4 * c, l);
  }
}

__global__ __launch_bounds__(NT, 1) void xattn_h3_kernel(XattnArgs a) {
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

  // ---- roles: waves 6 (K) and 7 (V) stage the tiles; compute pair (2 rb, 2 rb + 1) owns rows
  // 32 rb .. +32, wave dh the dims 128 dh .. +128 of both its partial scores and its U
  const bool loader = wid >= 6;
  const int rb = wid >> 1, dh = wid & 1;
  const bool live_wave = !loader && rb * 32 < nrows;
  const int my_row = rb * 32 + r32;

  // q' B fragments (S^T = K . Q'^T): lane (row r32, hh) holds dims 128 dh + 16 ks + 8 hh + (0..7),
  // scaled by 2^(13 - e) (max |q'| of the row's half in [2^(e-1), 2^e)) and split into fp16 hi / lo
  u32x4 qh[8], ql[8];
  float sinv = 1.f;                             // 2^-(sq + sk): the partial scores' unscale
  {
    const int r = row0 + my_row;
    const bool live = live_wave && my_row < nrows;
    const float* qp = (const float*)a.q + (size_t)(b * a.Q + (live ? r >> 3 : 0)) * a.ldq + (live ? (r & 7) : 0) * D + 128 * dh;
    float f[8][8];
    float am = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      unpack16<float>(live ? ld16(qp + 16 * ks + 8 * hh) : u32x4{0, 0, 0, 0}, f[ks]);
      unpack16<float>(live ? ld16(qp + 16 * ks + 8 * hh + 4) : u32x4{0, 0, 0, 0}, f[ks] + 4);
#pragma unroll
      for (int e = 0; e < 8; ++e) am = __builtin_fmaxf(am, __builtin_fabsf(f[ks][e]));
    }
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(am), __float_as_uint(am), false, false);
      am = __builtin_fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
    }
    float sq = 1.f;
    if (am > 0.f && am <= 3.0e38f) {
      const int e = __builtin_amdgcn_frexp_expf(am);
      sq = __builtin_ldexpf(1.f, 13 - e);
      sinv = __builtin_ldexpf(1.f, e - 13);
    }
    sinv *= 1.f / k_scale(a.mem_amax);          // (a power of two)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f[ks][e] * sq;
      u32x2 h0, l0, h1, l1;
      split_f16x4(v, h0, l0);
      split_f16x4(v + 4, h1, l1);
      qh[ks] = u32x4{h0.x, h0.y, h1.x, h1.y};
      ql[ks] = u32x4{l0.x, l0.y, l1.x, l1.y};
    }
  }

  // ---- staging (loader waves): one 1 KB key row per global_load_lds, lane -> slot `lane` holding
  // source chunk lane ^ swizzle (the swizzle on the source address, the LDS side lane-linear)
  const char* zero = reinterpret_cast<const char*>(g_x3zero);
  const bool isv = wid == 7;
  const char* src0 = isv ? (const char*)a.v : (const char*)a.k;
  const size_t ldsrc = (size_t)(isv ? a.ldv : a.ldk) * 2;
  auto issue = [&](int t, int buf) {
    char* st = lds + buf * STAGE + (isv ? KTILE : 0);
    const int key0 = t * KT;
    // (a rolled loop: the loader waves' addresses must not add to the compute waves' live registers)
#pragma unroll 2
    for (int key = 0; key < KT; ++key) {
      const int c = lane ^ (isv ? ((key & 3) << 2) : (key & 15));
      const char* src = key0 + key < a.T ? src0 + (size_t)(b * a.T + key0 + key) * ldsrc + c * 16 : zero;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)(st + key * ROW), 16, 0, 0);
    }
  };

  f32x16 acc[DB];
#pragma unroll
  for (int db = 0; db < DB; ++db)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[db][r] = 0.f;
  float m = 0.f, l = 0.f;

  // the q' loads retire before the DMA stream starts (vmcnt is in-order)
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) asm volatile("" ::"v"(qh[ks]), "v"(ql[ks]));
  const int nt = te - tb;
  if (loader && nt > 0) issue(tb, 0);
  float* const xown = reinterpret_cast<float*>(lds + NSTAGE * STAGE + (loader ? 0 : wid) * XCH);
  const float* const xoth = reinterpret_cast<const float*>(lds + NSTAGE * STAGE + (loader ? 0 : wid ^ 1) * XCH);
  for (int it = 0; it < nt; ++it) {
    const int t = tb + it, buf = it & 1;
    if (loader) wait_vm0();
    // barrier A (raw: __syncthreads' fence would drain the tile in flight): tile t visible to all,
    // every wave done with tile t-1 and with the previous exchange
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (loader) {
      if (it + 1 < nt) issue(t + 1, buf ^ 1);
      __builtin_amdgcn_s_barrier();             // barrier B (the pairs' exchange)
      continue;
    }
    const char* kl = lds + buf * STAGE;
    f32x16 sp;
#pragma unroll
    for (int r = 0; r < 16; ++r) sp[r] = 0.f;
    if (live_wave) {
      // partial S^T over this wave's 128 dims: lane (row r32, hh) register r <-> key
      // (r & 3) + 8 (r >> 2) + 4 hh
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int o = k_off(r32, 16 * dh + 2 * ks + hh);
        const u32x4 kh = ld16(kl + o), klo = ld16(kl + o + 512);
        sp = mfma_h(klo, qh[ks], sp);
        sp = mfma_h(kh, ql[ks], sp);
        sp = mfma_h(kh, qh[ks], sp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sp[r] *= sinv;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        st16(xown + j * 256 + 4 * lane, u32x4{__float_as_uint(sp[4 * j]), __float_as_uint(sp[4 * j + 1]),
                                              __float_as_uint(sp[4 * j + 2]), __float_as_uint(sp[4 * j + 3])});
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();               // barrier B: both halves written
    asm volatile("" ::: "memory");
    if (!live_wave) continue;
    f32x16 s;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[4];
      unpack16<float>(ld16(xoth + j * 256 + 4 * lane), o);
#pragma unroll
      for (int e = 0; e < 4; ++e) s[4 * j + e] = sp[4 * j + e] + o[e];   // the same sum in both waves
    }
    const int key_base = t * KT;
    if (key_base + KT > a.T) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (key_base + (r & 3) + 8 * (r >> 2) + 4 * hh >= a.T) s[r] = NEG_BIG;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] -= m;
    float mq[4];
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
      for (int r = 0; r < 16; ++r) s[r] -= d;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = __builtin_amdgcn_exp2f(s[r]);
    {
      float lq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) lq[i] = (s[4 * i] + s[4 * i + 1]) + (s[4 * i + 2] + s[4 * i + 3]);
      l += (lq[0] + lq[1]) + (lq[2] + lq[3]);
    }
    // P^T B operands of K-step ks: registers 8 ks + e (key 16 ks + 4 hh + 8 (e >> 2) + (e & 3)),
    // hi = RTZ fp16 pair, lo = RNE(p - hi) by v_fma_mix
    u32x4 ph[2], pl[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v0 = s[8 * ks + 2 * e], v1 = s[8 * ks + 2 * e + 1];
        hw[e] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v0, v1));
        uint32_t lo;
        asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hw[e]), "v"(v0));
        asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hw[e]), "v"(v1));
        lw[e] = lo;
      }
      ph[ks] = u32x4{hw[0], hw[1], hw[2], hw[3]};
      pl[ks] = u32x4{lw[0], lw[1], lw[2], lw[3]};
    }
    // V^T fragments (hi and lo planes) of step j = (dim block db = j / 2, K-step ks = j % 2): step j+1's
    // four reads in flight while step j's three MFMAs run
    const uint32_t vbase = (uint32_t)(uintptr_t)(lds_ptr_t)(kl + KTILE);
    u32x2 vr[2][4];
    auto read_v = [&](u32x2 (&r)[4], int j) {
      const int db = j >> 1, ks = j & 1;
      const uint32_t a0 = v_tr_addr(vbase, 16 * ks + 4 * hh, 128 * dh + 32 * db + dg, l16);
      const uint32_t a1 = v_tr_addr(vbase, 16 * ks + 8 + 4 * hh, 128 * dh + 32 * db + dg, l16);
      r[0] = ds_read_tr(a0);
      r[1] = ds_read_tr(a1);
      r[2] = ds_read_tr(a0 + 512);
      r[3] = ds_read_tr(a1 + 512);
    };
    read_v(vr[0], 0);
#pragma unroll
    for (int j = 0; j < 2 * DB; ++j) {
      if (j < 2 * DB - 1) {
        read_v(vr[(j + 1) & 1], j + 1);
        asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      const u32x2(&r)[4] = vr[j & 1];
      const int db = j >> 1, ks = j & 1;
      const u32x4 ah{r[0].x, r[0].y, r[1].x, r[1].y};
      const u32x4 al{r[2].x, r[2].y, r[3].x, r[3].y};
      acc[db] = mfma_h(al, ph[ks], acc[db]);
      acc[db] = mfma_h(ah, pl[ks], acc[db]);
      acc[db] = mfma_h(ah, ph[ks], acc[db]);
    }
  }
  if (!live_wave) return;
  // ---- partials: m, l (summed over the two lane halves), U^T unscaled by 2^-sv; lane holds
  // U^T[d = 32 db + 8 (r>>2) + 4 hh + (r&3)][row r32] of its 128 dims
  l += __shfl_xor(l, 32, 64);
  if (my_row >= nrows) return;
  const float vinv = 1.f / v_scale(a.mem_amax);
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
      const f32x4 v = {acc[db][4 * g] * vinv, acc[db][4 * g + 1] * vinv, acc[db][4 * g + 2] * vinv, acc[db][4 * g + 3] * vinv};
      st16(pu + 128 * dh + 32 * db + 8 * g + 4 * hh, __builtin_bit_cast(u32x4, v));
    }
}

// Merge of the key splits (weight of split s = 2^(m_s - M)) and the value projection in fp32,
// o_h[j] = Wv[h*32 + j] . u_h + bv[h*32 + j]: block = (16 query rows (b, q), head h), Wv_h [32][256]
// and the 16 merged u_h rows staged in LDS (rows padded to 257 floats), 2 outputs per thread; max |o|
// raised into o_amax.
constexpr int MR = 16, WP = D + 1;
__global__ __launch_bounds__(256) void xattn_h3_merge_wv_kernel(XattnArgs a) {
  __shared__ float wvs[32 * WP];
  __shared__ float us[MR * WP];
  const int tid = threadIdx.x, R = 8 * a.Q, h = blockIdx.y, bq0 = blockIdx.x * MR;
  const float* wv = (const float*)a.wv + (size_t)h * 32 * D;
#pragma unroll
  for (int i = 0; i < 8; ++i) {                 // 32 x 256 floats = 2048 chunks of 4
    const int idx = tid + i * 256, j = idx >> 6, c = idx & 63;
    float f[4];
    unpack16<float>(ld16(wv + (size_t)j * D + 4 * c), f);
#pragma unroll
    for (int e = 0; e < 4; ++e) wvs[j * WP + 4 * c + e] = f[e];
  }
  {
    const int i = tid >> 4, d0 = 16 * (tid & 15), bq = bq0 + i;
    float u[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) u[e] = 0.f;
    if (bq < a.B * a.Q) {
      const int b = bq / a.Q, r = (bq - b * a.Q) * 8 + h;
      float M = NEG_BIG;
      for (int s = 0; s < a.splits; ++s) M = fmaxf(M, a.pm[((size_t)b * a.splits + s) * R + r]);
      float L = 0.f;
      for (int s = 0; s < a.splits; ++s) {
        const size_t pr = ((size_t)b * a.splits + s) * R + r;
        const float w = __builtin_amdgcn_exp2f(a.pm[pr] - M);
        L += w * a.pl[pr];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = *reinterpret_cast<const f32x4*>(a.pu + pr * D + d0 + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) u[4 * g + e] += w * v[e];
        }
      }
      const float inv = 1.f / L;
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
    o0 = __builtin_fmaf(x, w0[n], o0);
    o1 = __builtin_fmaf(x, w1[n], o1);
  }
  float mx = 0.f;
  if (bq < a.B * a.Q) {
    st8((float*)a.o + (size_t)bq * a.ldo + h * 32 + j, u32x2{__float_as_uint(o0), __float_as_uint(o1)});
    mx = __builtin_fmaxf(__builtin_fabsf(o0), __builtin_fabsf(o1));
  }
  if (a.o_amax) amax_publish_block(mx, a.o_amax, 1.f, us);
}

}  // namespace

int spe_launch_xattn_h3_split(const float* mem, const float* pos, const float* mem_amax, void* kp, void* vp, int B,
                              int T, hipStream_t s) {
  if (B <= 0 || T <= 0) return 0;
  if (!mem || !pos || !kp || !vp) return -5;
  const size_t n4 = (size_t)B * T * (D / 4);
  const size_t blocks = (n4 + 255) / 256;
  const int grid = blocks < 8192 ? (int)blocks : 8192;
  hipLaunchKernelGGL(xattn_h3_split_kernel, dim3(grid), dim3(256), 0, s, mem, pos, mem_amax, (uint16_t*)kp,
                     (uint16_t*)vp, B, T);
  return (int)hipGetLastError();
}

int spe_launch_xattn_h3(const XattnArgs& a0, hipStream_t s) {
  XattnArgs a = a0;
  if (a.B <= 0) return 0;
  if (a.ldq % 4 || a.ldk != 2 * D || a.ldv != 2 * D || a.ldo % 2 || a.splits < 1 || a.T < 1) return -5;
  if (!a.q || !a.k || !a.v || !a.pm || !a.pl || !a.pu || !a.wv || !a.bv || !a.o) return -5;
  const int ntiles = (a.T + KT - 1) / KT;
  a.tiles_per_split = (ntiles + a.splits - 1) / a.splits;
  a.splits = spe_xattn_launch_splits(a.T, a.splits);
  const int groups = (8 * a.Q + RG - 1) / RG;
  hipLaunchKernelGGL(xattn_h3_kernel, dim3(a.B * a.splits * groups), dim3(NT), 0, s, a);
  hipLaunchKernelGGL(xattn_h3_merge_wv_kernel, dim3((a.B * a.Q + MR - 1) / MR, 8), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
