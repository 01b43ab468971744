// Fused multi-head attention (flash-style, online softmax) for head_dim = 32 on gfx950.
//
// Replaces nn.MultiheadAttention's score/softmax/value product in
//   encoder self-attention   REV/models/transformer.py:158-161  (Tq = Tk = (S/8)^2)
//   decoder self-attention   REV/models/transformer.py:225-227  (Tq = Tk = num_queries)
//   decoder cross-attention  REV/models/transformer.py:230-233  (Tq = num_queries, Tk = tokens)
// The reference materialises the full head-averaged probability tensor (need_weights=True);
// the outputs do not depend on it, so it is never formed here.  key_padding_mask is all-False
// for fixed-size inputs (REV/utils/misc.py:311-322) and is therefore not an input.
//
// Workgroup = 4 waves = 128 queries of one (image, head); each wave owns 32 queries.
// Scores are computed transposed (S^T = K . Q^T) with 32x32 MFMAs so that each lane holds the
// scores of ONE query: the row max needs a single lane<->lane^32 exchange, and the probability
// tile is fed straight back as the B operand of O^T = V^T . P^T without leaving registers.
// K tiles [64 keys][32] and V^T tiles [32][64 keys] are staged through XOR-swizzled LDS,
// double-buffered (register prefetch of tile t+1 overlaps the MFMAs of tile t).
//
// head_dim 32 makes the softmax the bottleneck (one exp per 128 MFMA flops), so the bf16 path
// spends as little VALU per score as possible: Q is pre-scaled by softmax_scale*log2(e) (scores
// come out in the exp2 domain), the running max only triggers an O/l rescale when some lane's
// max actually grew (wave-uniform branch), and the row sums l are f32 adds of p (each lane sums
// its 32 keys, the lane pair is combined once at the end).  The chip runs this loop at its
// power limit (~1.75-1.8 GHz), so what pays is energy per tile, not issue slots: a ones . P^T
// MFMA for the sums (4 of 12 MFMAs) cost more than the 35 VALU adds that replace it
// (scripts/lab/attn_lab.hip: 0.86 -> 0.81 ms at B = 64 on random inputs).
// bf16: v_mfma_f32_32x32x16_bf16; fp16 operands (config 5): v_mfma_f32_32x32x16_f16 (same
// kernel, AT<f16> traits).  fp32 (parity mode): v_mfma_f32_32x32x2_f32, exact f32.
#include "spe_common.h"
#include <type_traits>
#include "spe_kernels.h"

namespace {

constexpr int NT = 256;
constexpr int KT = 64;                 // keys per softmax step (and per staged tile, fp32)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;    // finite "minus infinity" (exp2 of it underflows to 0)
constexpr float RESCALE_SLACK = 8.0f;  // log2 units (bf16 path)
constexpr float LAZY_LIMIT = 4096.0f;  // fp16-P tiles: a lane's 32-key sum that forces the max path
#ifndef SPE_ATTN_PACK
#define SPE_ATTN_PACK 1
#endif
#ifndef SPE_ATTN_LAZY
#define SPE_ATTN_LAZY 1
#endif
// DMA kernel: waves per workgroup (4: 128 queries, two DMA pieces per wave per tile; 8: 256
// queries, one piece per wave -- the piece's issue cost halves -- and two workgroups per CU)
#ifndef SPE_ATTN_DMA_WAVES
#define SPE_ATTN_DMA_WAVES 8
#endif
constexpr int DMA_WAVES = SPE_ATTN_DMA_WAVES;
static_assert(DMA_WAVES == 4 || DMA_WAVES == 8, "DMA waves");
#ifndef SPE_ATTN_OCC
#define SPE_ATTN_OCC 4
#endif

// ---------------------------------------------------------------- bf16 LDS image
// Padded (not XOR-swizzled) rows, so every fragment read is lane base + immediate offset with
// no per-read address VALU.  K tile: rows of 64 B + 16 B pad: the 16 keys of one ds_read_b128
// lane group start 20 banks apart mod 64 -> 16 distinct 4-bank groups (conflict-free).
constexpr int KROW = 80;
SPE_DEV int k_off_bf16(int key, int c) { return key * KROW + (c << 4); }
// V^T tile: 32 rows (d) of KT keys + 16 B pad (row = 36 dwords: the 16 rows of each
// ds_read_b128 lane group start on distinct 4-bank groups).  Within every 16-key group the two
// middle quads are swapped (keys 0-3, 8-11, 4-7, 12-15), which is the k order the P^T operand
// has straight out of the S^T accumulator: each PV MFMA's A operand is ONE 16-byte read.
constexpr int VROW = KT * 2 + 16;
SPE_DEV int v_quad_off(int d, int quad) {            // quad = 4-key unit index within the row
  const int g = quad >> 2, qi = quad & 3;
  const int pos = (qi == 1) ? 2 : (qi == 2) ? 1 : qi;
  return d * VROW + g * 32 + pos * 8;
}
// ---------------------------------------------------------------- fp32 LDS image
SPE_DEV int k_off_f32(int key, int c) { return key * 128 + ((c ^ (key & 7)) << 4); }       // 8 chunks
SPE_DEV int v_off_f32(int d, int c) { return d * 256 + ((c ^ (d & 15)) << 4); }            // 16 chunks

template <typename T, int KTT>
struct Stage {
  static constexpr int ES = sizeof(T);
  static constexpr int KCH = KTT * 32 * ES / 16 / NT;  // K chunks per thread
  static constexpr int VCH = 32 * KTT * ES / 16 / NT;  // V^T chunks per thread
  u32x4 kr[KCH], vr[VCH];

  SPE_DEV void load(const AttnArgs& a, int b, int h, int kt, int tid) {
    constexpr int CE = 16 / ES;
    constexpr int KCPR = 32 / CE;     // K chunks per key row
    constexpr int VCPR = KTT / CE;    // V^T chunks per d row
    const T* kbase = (const T*)a.k + (size_t)b * a.Tk * a.ldk + h * 32;
    const T* vbase = (const T*)a.vt + (size_t)(b * a.H + h) * 32 * a.Tk;
    if ((kt + 1) * KTT <= a.Tk && (a.Tk % CE) == 0) {     // whole tile in range (wave-uniform)
#pragma unroll
      for (int i = 0; i < KCH; ++i) {
        const int idx = tid + i * NT, key = idx / KCPR, c = idx % KCPR;
        kr[i] = ld16(kbase + (size_t)(kt * KTT + key) * a.ldk + c * CE);
      }
#pragma unroll
      for (int i = 0; i < VCH; ++i) {
        const int idx = tid + i * NT, d = idx / VCPR, c = idx % VCPR;
        vr[i] = ld16(vbase + (size_t)d * a.Tk + kt * KTT + c * CE);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      int idx = tid + i * NT;
      int key = idx / KCPR, c = idx % KCPR;
      int kk = kt * KTT + key;
      kr[i] = kk < a.Tk ? ld16(kbase + (size_t)kk * a.ldk + c * CE) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      int idx = tid + i * NT;
      int d = idx / VCPR, c = idx % VCPR;
      int k0 = kt * KTT + c * CE;
      const T* src = vbase + (size_t)d * a.Tk + k0;
      if (k0 + CE <= a.Tk && ((a.Tk % CE) == 0)) {
        vr[i] = ld16(src);
      } else {
        T tmp[CE];
#pragma unroll
        for (int e = 0; e < CE; ++e) tmp[e] = (k0 + e < a.Tk) ? src[e] : from_f32<T>(0.f);
        vr[i] = *reinterpret_cast<const u32x4*>(tmp);
      }
    }
  }

  SPE_DEV void store(char* kl, char* vl, int tid) const {
    constexpr int CE = 16 / ES;
    constexpr int KCPR = 32 / CE;
    constexpr int VCPR = KTT / CE;
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      int idx = tid + i * NT;
      int key = idx / KCPR, c = idx % KCPR;
      st16(kl + (ES == 2 ? k_off_bf16(key, c) : k_off_f32(key, c)), kr[i]);
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      int idx = tid + i * NT;
      int d = idx / VCPR, c = idx % VCPR;
      if constexpr (ES == 2) {
        st8(vl + v_quad_off(d, 2 * c), u32x2{vr[i].x, vr[i].y});
        st8(vl + v_quad_off(d, 2 * c + 1), u32x2{vr[i].z, vr[i].w});
      } else {
        st16(vl + v_off_f32(d, c), vr[i]);
      }
    }
  }
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
// s_waitcnt immediate (gfx9: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8]) for a vmcnt-only
// wait, issued through the builtin so the compiler's own wait insertion accounts for it
constexpr int attn_waitcnt_vm(int vm) { return (vm & 15) | ((vm >> 4) << 14) | (7 << 4) | (15 << 8); }

// mask keys past Tk (last tile only)
SPE_DEV void tile_mask(f32x16& s0, f32x16& s1, int key_base, int Tk, int hh) {
  if (key_base + KT > Tk) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (key_base + kr >= Tk) s0[r] = NEG_BIG;
      if (key_base + 32 + kr >= Tk) s1[r] = NEG_BIG;
    }
  }
}

// Tk % 16 == 0 (the DMA kernel): the lane's scores r = 0-7 of s0 are keys 0-15 of the tile, r =
// 8-15 keys 16-31, and s1 the next 32 -- each register group is one whole 16-key group, so the
// mask is four wave-uniform tests
SPE_DEV void tile_mask16(f32x16& s0, f32x16& s1, int key_base, int Tk) {
  if (key_base + KT > Tk) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
      if (key_base + 16 * g >= Tk) {
        f32x16& s = g < 2 ? s0 : s1;
#pragma unroll
        for (int r = 0; r < 8; ++r) s[8 * (g & 1) + r] = NEG_BIG;
      }
  }
}

// mask keys past Tk (last tile only; MASK = false: done by the caller) and return the lane-pair
// max of the 32 scores
template <bool MASK = true>
SPE_DEV float tile_max(f32x16& s0, f32x16& s1, int key_base, int Tk, int hh) {
  if constexpr (MASK) tile_mask(s0, s1, key_base, Tk, hh);
  // two independent v_max3 chains (the file is built with -fno-honor-nans, so no canonicalizes)
  float ma = __builtin_fmaxf(s0[0], s1[0]), mb = __builtin_fmaxf(s0[1], s1[1]);
#pragma unroll
  for (int r = 2; r < 16; r += 2) {
    ma = __builtin_fmaxf(__builtin_fmaxf(ma, s0[r]), s1[r]);
    mb = __builtin_fmaxf(__builtin_fmaxf(mb, s0[r + 1]), s1[r + 1]);
  }
  const float mx = __builtin_fmaxf(ma, mb);
  // lane <-> lane^32 exchange without an LDS round trip
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
  return __builtin_fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}

// 16-bit operand traits: bf16 (default) or fp16 (BASELINE config 5's "fp16 MFMA attention":
// the encoder q/k projection and V^T are then stored as fp16 by their GEMM epilogues).  P is
// packed with v_cvt_pkrtz_f16_f32 for fp16 (one instruction per two values, like
// v_cvt_pk_bf16_f32; round-toward-zero costs < 1 fp16 ulp = 2^-10, below bf16's RNE 2^-9).
template <typename TI> struct AT;
template <> struct AT<bf16> {
  typedef bf16x8 v8;
  static SPE_DEV uint32_t pk(float a, float b) { return pack_bf16x2(a, b); }
  static SPE_DEV f32x16 mfma(v8 a, v8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0); }
};
template <> struct AT<f16> {
  typedef f16x8 v8;
  static SPE_DEV uint32_t pk(float a, float b) { return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b)); }
  static SPE_DEV f32x16 mfma(v8 a, v8 b, f32x16 c) { return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0); }
};

// ------------------------------------------------------------------ bf16 kernel
// ROLE only separates the symbols of the token-query (encoder self-attention) and the
// object-query (decoder) launches so profiler summaries report them apart; the code is shared.
// TV: type of V^T and of P (the value product).  TV = fp16 also under bf16 q/k (the bf16
// model's encoder, V^T stored fp16 by the v-projection epilogue): P is then packed as fp16
// pairs, and the row sums are packed-fp16 adds of those same words (15 v_pk_add_f16 + one
// v_dot2_f32_f16 per 64-key tile instead of 32 f32 adds; the tile's partial sum <= 32 * 2^8
// fits fp16, and it is the rounded P the value product uses).
// DMA: K and V^T tiles go global -> LDS by buffer_load ... lds (V^T stored in vt_pos order by the
// v projection, so each 16-byte chunk lands verbatim), through a three-slot ring with two tiles
// in flight: no staging registers, no ds_write, no per-tile vmcnt(0) before a store.  Each
// wave issues exactly two 1 KB pieces per tile (unpadded XOR-swizzled images: K 4, V^T 4; the
// padded images took 10 pieces, 3 per wave with two duplicates), so one immediate vmcnt retires
// a tile.  Needs Tk % 16 == 0 (the quad swap stays inside a row).
template <int ROLE, typename TI, typename TV = TI, bool DMA = false>
__global__ __launch_bounds__(DMA ? 64 * DMA_WAVES : NT, DMA ? 16 / DMA_WAVES : SPE_ATTN_OCC) void attn16_kernel(AttnArgs a) {
  typedef AT<TI> A;
  typedef AT<TV> AV;
  typedef typename A::v8 v8;
  typedef typename AV::v8 vv8;
  constexpr bool HSUM = sizeof(TV) == 2 && !std::is_same<TV, bf16>::value;   // fp16 P: packed sums
  constexpr bool LAZY = HSUM && DMA && SPE_ATTN_LAZY;   // no per-tile max (below)
  // PACK (DMA): unpadded tiles, XOR-swizzled instead -- K 4 KB + V^T 4 KB = 8 pieces, 8 / DMA_WAVES per wave
  constexpr bool PACK = DMA && SPE_ATTN_PACK;
  constexpr int KBYTES = PACK ? KT * 64 : KT * KROW, VBYTES = PACK ? 32 * KT * 2 : 32 * VROW;
  constexpr int DSLOT = PACK ? 8192 : 10240;       // DMA slot (padded: K 5 KB + V^T 4.5 KB + 0.5 KB spill room)
  constexpr int NPC = PACK ? 8 / DMA_WAVES : 3;    // DMA pieces per wave per tile
  static_assert(KBYTES + VBYTES <= DSLOT, "DMA slot");
  static_assert(!DMA || PACK || DMA_WAVES == 4, "padded DMA images: 4 waves");
  __shared__ __attribute__((aligned(1024))) char smem[DMA ? 3 * DSLOT : 2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  constexpr int QB = 32 * (DMA ? DMA_WAVES : 4);   // queries per workgroup
  const int qblocks = (a.Tq + QB - 1) / QB;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * QB + wid * 32 + r32;
  const bool wave_live = qb * QB + wid * 32 < a.Tq;

  // query fragment (B operand of S^T = K . Q^T), pre-scaled into the exp2 domain
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
  // the query fragments are formed here, before the DMA stream starts: left to the compiler it
  // re-forms them inside the key loop, and its wait for the q loads (vmcnt is in-order) then
  // drains the next tile's DMA every iteration
  if constexpr (DMA) asm volatile("" ::"v"(qf[0]), "v"(qf[1]));
  // o: O^T accumulator; ls: this lane's running sum of p over its half of the keys.
  f32x16 o;
  float ls = 0.f;
  // negm: -m in every element, the accumulator the score MFMAs start from, so the scores come
  // out already shifted by the running max (s - m) and p = exp2 of them costs no subtract.
  f32x16 negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f;                        // set from the first tile (forced rescale at kt == 0)

  // Two-slot LDS ring, one barrier per 64-key step: tile kt+1 travels global -> registers
  // during step kt and is written to the other slot after it.  (A three-slot ring that
  // prefetches the next step's K fragments measured slower: its extra live registers cost
  // either spills or a wave of occupancy.)
  const int ntiles = (a.Tk + KT - 1) / KT;
  constexpr int SLOT = KBYTES + VBYTES;
  Stage<TI, KT> st;
  // DMA pieces of this wave: slots wid, wid + 4 (PACK: of {K 0-3, V^T 0-3}), or wid, wid + 4,
  // wid + 8 (padded: of {K 0-4, V^T 0-4, K 0-1 again}).  Per lane a fixed voffset; the tile moves
  // the scalar soffset.  PACK images (conflict-free for ds_read_b128's 16-lane groups): key row
  // of 64 B with 16-byte chunk c at slot c ^ ((key >> 2) & 3); V^T row of 128 B with chunk c at
  // slot c ^ ((d >> 1) & 7) -- a lane-linear DMA piece gets the swizzle on its source addresses.  Rows past Tk read as zero through
  // the descriptors' ranges (this image's K rows, this (image, head)'s V^T block).
  // (b, h and the wave index are wave-uniform; readfirstlane lets the compiler keep the
  // descriptors and the piece selection scalar instead of waterfalling over lanes)
  const int bu = __builtin_amdgcn_readfirstlane(b), hu = __builtin_amdgcn_readfirstlane(h);
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const TI*)a.k + (size_t)bu * a.Tk * a.ldk + hu * 32), (short)0, a.Tk * a.ldk * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((const TV*)a.vt + (size_t)(bu * a.H + hu) * 32 * a.Tk), (short)0, 32 * a.Tk * 2, 0x00020000);
  int dvo[3] = {0, 0, 0}, dlo[3] = {0, 0, 0};
  bool dv[3] = {false, false, false};
  if constexpr (DMA) {
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      const int slot = wu + DMA_WAVES * j;
      if constexpr (PACK) {
        const int isv = slot >= 4, pc = slot & 3;
        if (!isv) {
          const int key = pc * 16 + (lane >> 2), c = (lane & 3) ^ ((key >> 2) & 3);
          dvo[j] = key * a.ldk * 2 + c * 16;
          dlo[j] = pc * 1024;
        } else {
          const int d = pc * 8 + (lane >> 3), c = (lane & 7) ^ ((d >> 1) & 7);
          dvo[j] = (d * a.Tk + c * 8) * 2;
          dlo[j] = KBYTES + pc * 1024;
        }
        dv[j] = isv;
        continue;
      }
      const int piece = slot < 10 ? slot : slot - 10;
      const int isv = piece >= 5, pc = isv ? piece - 5 : piece;
      const int o = pc * 1024 + lane * 16;
      if (!isv) {
        const int key = o / KROW, c = (o - key * KROW) >> 4;
        dvo[j] = key * a.ldk * 2 + (c < 4 ? c : 0) * 16;
        dlo[j] = pc * 1024;
      } else {
        const int d = o / VROW, c = (o - d * VROW) >> 4;
        dvo[j] = (d < 32 && c < 8) ? (d * a.Tk + c * 8) * 2 : 0;
        dlo[j] = KBYTES + pc * 1024;
      }
      dv[j] = isv;
    }
  }
  auto issue = [&](int kt, int slot) {
    char* base = smem + slot * DSLOT;
#pragma unroll
    for (int j = 0; j < NPC; ++j) {
      // (the LDS address is per wave-instruction: lane 0's; lanes follow at 16-byte steps)
      lds_ptr_t dst = (lds_ptr_t)(base + dlo[j]);
      if (dv[j]) __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, dst, 16, dvo[j], kt * KT * 2, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rk, dst, 16, dvo[j], kt * KT * a.ldk * 2, 0, 0);
    }
  };
  if constexpr (DMA) {
    issue(0, 0);
    if (ntiles > 1) issue(1, 1);
  } else {
    st.load(a, b, h, 0, tid);
    st.store(smem, smem + KBYTES, tid);
    __syncthreads();
  }
  // fragment offsets in a staged tile: K (key sub * 32 + r32, 16-byte chunk c), V^T (row r32, the
  // chunk of keys sub * 32 + 16 ks + 8 hh)
  auto koff = [&](int sub, int c) {
    return PACK ? (sub * 32 + r32) * 64 + ((c ^ ((r32 >> 2) & 3)) << 4) : k_off_bf16(sub * 32 + r32, c);
  };
  auto voff = [&](int sub, int ks) {
    const int ch = (2 * sub + ks) * 2 + hh;
    return PACK ? r32 * 128 + ((ch ^ ((r32 >> 1) & 7)) << 4) : r32 * VROW + ch * 16;
  };
  // one 64-key step; SC = the DMA ring slot as a compile-time constant (the DMA loop below is
  // unrolled by the ring's three slots, so every fragment read is a lane base + immediate
  // offset: no per-step address VALU), -1 for the register-staged kernel
  auto step = [&](int kt, auto SC) {
    constexpr int S = decltype(SC)::value;
    const char* kl = smem + (DMA ? S * DSLOT : (kt & 1) * SLOT);
    const char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if constexpr (DMA) {
      // tile kt landed (tile kt+1 may stay in flight), then the barrier: tile kt visible to all,
      // every wave done with tile kt-1, whose slot takes tile kt+2
      if (more) __builtin_amdgcn_s_waitcnt(attn_waitcnt_vm(NPC));
      else __builtin_amdgcn_s_waitcnt(attn_waitcnt_vm(0));
      __builtin_amdgcn_s_barrier();
      // (live waves issue tile kt+2 after their score MFMAs: a DMA issued ahead of the fragment
      // reads made the compiler wait for every read, V included, before the first MFMA)
      if (!wave_live && kt + 2 < ntiles) issue(kt + 2, (S + 2) % 3);
    } else {
      if (more) st.load(a, b, h, kt + 1, tid);
    }
    if (wave_live) {
      // every fragment read of this step is issued up front; V lands during QK^T + softmax
      u32x4 kf[2][2], vf[2][2];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        kf[sub][0] = ld16(kl + koff(sub, hh));
        kf[sub][1] = ld16(kl + koff(sub, 2 + hh));
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)      // keys sub*32 + 16ks + {4hh..+3, 8+4hh..+3}
          vf[sub][ks] = ld16(vl + voff(sub, ks));
      f32x16 s0, s1;                    // s - m
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][0]), qf[0], negm);
        s = A::mfma(__builtin_bit_cast(v8, kf[sub][1]), qf[1], s);
      }
      if constexpr (DMA) {
        if (kt + 2 < ntiles) issue(kt + 2, (S + 2) % 3);
      }
      // LAZY (fp16 P): no per-tile max at all.  The tile is exponentiated against the stale
      // running max and its packed-fp16 row sum, formed anyway, is the overflow test: only if
      // some lane's 32-key sum passes LAZY_LIMIT (any p > 2^12, or an fp16 overflow) are the
      // scores recomputed from the K tile still in LDS and taken through the max/rescale path.
      bool full = !LAZY || kt == 0;
      u32x4 pw[2][2];
      float tsum = 0.f;
      for (;;) {
        if constexpr (DMA) tile_mask16(s0, s1, kt * KT, a.Tk);
        if (full) {
          const float mx = tile_max<!DMA>(s0, s1, kt * KT, a.Tk, hh);   // relative to m
          // Lazy rescale (wave-uniform): keep the stale max until some lane's max grew by more
          // than RESCALE_SLACK (p <= 2^8 then, harmless in fp32 accumulators and 16-bit P).  With
          // an exact "grew at all" test, 32 queries per wave re-fire the rescale on about half the
          // tiles.  The first tile always sets m to its own max (o and l are still zero then).
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
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s0[r] = __builtin_amdgcn_exp2f(s0[r]);
          s1[r] = __builtin_amdgcn_exp2f(s1[r]);
        }
        if constexpr (!HSUM) {
          float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
          for (int r = 0; r < 16; r += 2) { t0 += s0[r]; t1 += s0[r + 1]; t2 += s1[r]; t3 += s1[r + 1]; }
          tsum = (t0 + t1) + (t2 + t3);
        }
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          const f32x16& p = sub ? s1 : s0;
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
            pw[sub][ks] = u32x4{AV::pk(p[8 * ks + 0], p[8 * ks + 1]), AV::pk(p[8 * ks + 2], p[8 * ks + 3]),
                                AV::pk(p[8 * ks + 4], p[8 * ks + 5]), AV::pk(p[8 * ks + 6], p[8 * ks + 7])};
        }
        if constexpr (HSUM) {
          typedef _Float16 h2 __attribute__((ext_vector_type(2)));
          auto H2 = [](uint32_t w) { return __builtin_bit_cast(h2, w); };
          h2 u[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            u[e] = (H2(pw[0][0][e]) + H2(pw[0][1][e])) + (H2(pw[1][0][e]) + H2(pw[1][1][e]));
          tsum = __builtin_amdgcn_fdot2((u[0] + u[1]) + (u[2] + u[3]), h2{(_Float16)1.f, (_Float16)1.f}, 0.f, false);
        }
        if (full || !__any(tsum > LAZY_LIMIT)) break;
        full = true;
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
          f32x16& s = sub ? s1 : s0;
          s = A::mfma(__builtin_bit_cast(v8, ld16(kl + koff(sub, hh))), qf[0], negm);
          s = A::mfma(__builtin_bit_cast(v8, ld16(kl + koff(sub, 2 + hh))), qf[1], s);
        }
      }
      ls += tsum;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          o = AV::mfma(__builtin_bit_cast(vv8, vf[sub][ks]), __builtin_bit_cast(vv8, pw[sub][ks]), o);
    }
    if constexpr (!DMA) {
      if (more) st.store(smem + ((kt + 1) & 1) * SLOT, smem + ((kt + 1) & 1) * SLOT + KBYTES, tid);
      __syncthreads();
    }
  };
  if constexpr (DMA) {
    for (int kt = 0; kt < ntiles; kt += 3) {
      step(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < ntiles) step(kt + 1, std::integral_constant<int, 1>{});
      if (kt + 2 < ntiles) step(kt + 2, std::integral_constant<int, 2>{});
    }
  } else {
    for (int kt = 0; kt < ntiles; ++kt) step(kt, std::integral_constant<int, -1>{});
  }

  if (!wave_live || q >= a.Tq) return;
  const float inv = 1.f / (ls + __shfl_xor(ls, 32, 64));   // the lane pair's two key halves
  bf16* op = (bf16*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int d0 = 8 * g + 4 * hh;
    st8(op + d0, u32x2{pack_bf16x2(o[4 * g] * inv, o[4 * g + 1] * inv), pack_bf16x2(o[4 * g + 2] * inv, o[4 * g + 3] * inv)});
  }
}

// ------------------------------------------------------------------ fp32 (parity) kernel
__global__ __launch_bounds__(NT, 2) void attn_f32_kernel(AttnArgs a) {
  constexpr int KBYTES = KT * 32 * 4, VBYTES = 32 * KT * 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * (KBYTES + VBYTES)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;
  const float sl2 = a.scale * LOG2E;

  u32x4 qf[4];
  {
    const float* qp = (const float*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) qf[i] = q < a.Tq ? ld16(qp + 16 * hh + 4 * i) : u32x4{0, 0, 0, 0};
  }
  f32x16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  float m = NEG_BIG, l = 0.f;

  const int ntiles = (a.Tk + KT - 1) / KT;
  Stage<float, KT> st;
  st.load(a, b, h, 0, tid);
  st.store(smem, smem + KBYTES, tid);
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    char* kl = smem + (kt & 1) * (KBYTES + VBYTES);
    char* vl = kl + KBYTES;
    const bool more = kt + 1 < ntiles;
    if (more) st.load(a, b, h, kt + 1, tid);
    if (wave_live) {
      f32x16 s0, s1;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] = 0.f; s1[r] = 0.f; }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int key = sub * 32 + r32;
        f32x16& s = sub ? s1 : s0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          f32x4 kv = __builtin_bit_cast(f32x4, ld16(kl + k_off_f32(key, 4 * hh + c)));
          f32x4 qv = __builtin_bit_cast(f32x4, qf[c]);
#pragma unroll
          for (int e = 0; e < 4; ++e) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[e], qv[e], s, 0, 0, 0);
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] *= sl2; s1[r] *= sl2; }
      const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
      const float mn = __builtin_fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mn);   // (bare v_exp_f32: exp2f's denormal scaling buys nothing here)
      float sum = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s0[r] = __builtin_amdgcn_exp2f(s0[r] - mn);
        s1[r] = __builtin_amdgcn_exp2f(s1[r] - mn);
        sum += s0[r] + s1[r];
      }
      l = l * alpha + sum;
      m = mn;
#pragma unroll
      for (int r = 0; r < 16; ++r) o[r] *= alpha;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const f32x16& p = sub ? s1 : s0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // keys 8i + 4hh + (0..3) of this sub-tile = chunk 2i + hh
          f32x4 vv = __builtin_bit_cast(f32x4, ld16(vl + v_off_f32(r32, sub * 8 + 2 * i + hh)));
#pragma unroll
          for (int e = 0; e < 4; ++e) o = __builtin_amdgcn_mfma_f32_32x32x2f32(vv[e], p[4 * i + e], o, 0, 0, 0);
        }
      }
    }
    if (more) st.store(smem + ((kt + 1) & 1) * (KBYTES + VBYTES), smem + ((kt + 1) & 1) * (KBYTES + VBYTES) + KBYTES, tid);
    __syncthreads();
  }

  if (!wave_live || q >= a.Tq) return;
  const float lt = l + __shfl_xor(l, 32, 64);    // each lane of the pair summed its 32 keys
  const float inv = 1.f / lt;
  float* op = (float*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    float v[4] = {o[4 * g] * inv, o[4 * g + 1] * inv, o[4 * g + 2] * inv, o[4 * g + 3] * inv};
    st16(op + 8 * g + 4 * hh, pack16<float>(v));
  }
}

// ------------------------------------------------------------------ fp32x3 (parity) kernel
// fp32 q, k, V^T in and fp32 out like attn_f32_kernel, computed with split-bf16 MFMAs: every
// fp32 operand x = hi + lo (hi = bf16(x), lo = bf16(x - hi)) and each product as hi.hi + hi.lo
// + lo.hi on v_mfma_f32_32x32x16_bf16 (relative error ~2^-17 per product instead of fp32's
// 2^-24, at a sixth of the matrix cycles of v_mfma_f32_32x32x2_f32).  K and V^T are split once
// per tile as they are staged (the bf16 kernel's LDS images, one for hi and one for lo); q is
// scaled into the exp2 domain in fp32 and split in registers; the probabilities stay fp32 for
// the running max, the exp2 and the row sums, and are split only as the value-product operand.
// PS (AttnArgs::presplit): K and V^T arrive as bf16 hi / lo planes written by the projection
// epilogues (GemmArgs::S) -- the same RNE split, done once per element instead of once per
// (element, query block) -- and are staged as plain 16-byte copies.
template <bool PS>
__global__ __launch_bounds__(NT, 2) void attn_x3_kernel(AttnArgs a) {
  constexpr int KB = KT * KROW, VB = 32 * VROW, SLOT = 2 * (KB + VB);   // [K hi | K lo | V hi | V lo]
  __shared__ __attribute__((aligned(16))) char smem[2 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  const bool wave_live = qb * 128 + wid * 32 < a.Tq;
  auto mf = [](u32x4 x, u32x4 y, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, x), __builtin_bit_cast(bf16x8, y), c, 0, 0, 0);
  };
  // query fragments: dims 16i + 8hh + (0..7), scaled by softmax_scale * log2(e) in fp32, split
  u32x4 qh[2], ql[2];
  {
    const float sl2 = a.scale * LOG2E;
    const float* qp = (const float*)a.q + (size_t)(b * a.Tq + (q < a.Tq ? q : 0)) * a.ldq + h * 32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float f[8];
      const u32x4 x0 = q < a.Tq ? ld16(qp + 16 * i + 8 * hh) : u32x4{0, 0, 0, 0};
      const u32x4 x1 = q < a.Tq ? ld16(qp + 16 * i + 8 * hh + 4) : u32x4{0, 0, 0, 0};
      unpack16<float>(x0, f);
      unpack16<float>(x1, f + 4);
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v0 = f[2 * e] * sl2, v1 = f[2 * e + 1] * sl2;
        hw[e] = pack_bf16x2(v0, v1);
        lw[e] = pack_bf16x2(v0 - __uint_as_float(hw[e] << 16), v1 - __uint_as_float(hw[e] & 0xffff0000u));
      }
      qh[i] = u32x4{hw[0], hw[1], hw[2], hw[3]};
      ql[i] = u32x4{lw[0], lw[1], lw[2], lw[3]};
    }
  }
  // negm: -m in every element, the accumulator the score MFMAs start from (scores come out
  // shifted by the running max), as in the bf16 kernel; m is set by the first tile
  f32x16 o, negm;
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, l = 0.f;

  // staging: fp32 tiles through registers (Stage<float>), split into the hi / lo images; PS:
  // one 16-byte K chunk (8 dims of a key) and one V^T chunk (8 keys of a d row) per plane
  Stage<float, KT> st;
  u32x4 pk[2], pv[2];
  const size_t klo = (size_t)a.B * a.Tk * a.ldk, vlo = (size_t)a.B * a.H * 32 * a.Tk;
  auto load_ps = [&](int kt) {
    const int key = kt * KT + (tid >> 2), c = tid & 3;
    const bf16* kp = (const bf16*)a.k + (size_t)(b * a.Tk + (key < a.Tk ? key : 0)) * a.ldk + h * 32 + c * 8;
    pk[0] = key < a.Tk ? ld16(kp) : u32x4{0, 0, 0, 0};
    pk[1] = key < a.Tk ? ld16(kp + klo) : u32x4{0, 0, 0, 0};
    const int d = tid >> 3, k0 = kt * KT + (tid & 7) * 8;
    const bf16* vp = (const bf16*)a.vt + ((size_t)(b * a.H + h) * 32 + d) * a.Tk + (k0 < a.Tk ? k0 : 0);
    pv[0] = k0 < a.Tk ? ld16(vp) : u32x4{0, 0, 0, 0};
    pv[1] = k0 < a.Tk ? ld16(vp + vlo) : u32x4{0, 0, 0, 0};
  };
  auto store_ps = [&](char* sl) {
    const int key = tid >> 2, c = tid & 3, d = tid >> 3, cv = tid & 7;
    st16(sl + k_off_bf16(key, c), pk[0]);
    st16(sl + KB + k_off_bf16(key, c), pk[1]);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      st8(sl + 2 * KB + p * VB + v_quad_off(d, 2 * cv), u32x2{pv[p].x, pv[p].y});
      st8(sl + 2 * KB + p * VB + v_quad_off(d, 2 * cv + 1), u32x2{pv[p].z, pv[p].w});
    }
  };
  auto store = [&](char* sl) {
    constexpr int KCPR = 8, VCPR = KT / 4;
#pragma unroll
    for (int i = 0; i < Stage<float, KT>::KCH; ++i) {
      const int idx = tid + i * NT, key = idx / KCPR, c = idx % KCPR;   // dims 4c..4c+3
      const f32x4 f = __builtin_bit_cast(f32x4, st.kr[i]);
      const uint32_t h0 = pack_bf16x2(f[0], f[1]), h1 = pack_bf16x2(f[2], f[3]);
      const uint32_t l0 = pack_bf16x2(f[0] - __uint_as_float(h0 << 16), f[1] - __uint_as_float(h0 & 0xffff0000u));
      const uint32_t l1 = pack_bf16x2(f[2] - __uint_as_float(h1 << 16), f[3] - __uint_as_float(h1 & 0xffff0000u));
      const int off = k_off_bf16(key, c >> 1) + (c & 1) * 8;
      st8(sl + off, u32x2{h0, h1});
      st8(sl + KB + off, u32x2{l0, l1});
    }
#pragma unroll
    for (int i = 0; i < Stage<float, KT>::VCH; ++i) {
      const int idx = tid + i * NT, d = idx / VCPR, c = idx % VCPR;     // keys 4c..4c+3
      const f32x4 f = __builtin_bit_cast(f32x4, st.vr[i]);
      const uint32_t h0 = pack_bf16x2(f[0], f[1]), h1 = pack_bf16x2(f[2], f[3]);
      const uint32_t l0 = pack_bf16x2(f[0] - __uint_as_float(h0 << 16), f[1] - __uint_as_float(h0 & 0xffff0000u));
      const uint32_t l1 = pack_bf16x2(f[2] - __uint_as_float(h1 << 16), f[3] - __uint_as_float(h1 & 0xffff0000u));
      st8(sl + 2 * KB + v_quad_off(d, c), u32x2{h0, h1});
      st8(sl + 2 * KB + VB + v_quad_off(d, c), u32x2{l0, l1});
    }
  };
  const int ntiles = (a.Tk + KT - 1) / KT;
  if constexpr (PS) {
    load_ps(0);
    store_ps(smem);
  } else {
    st.load(a, b, h, 0, tid);
    store(smem);
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const char* kl = smem + (kt & 1) * SLOT;
    const char* vl = kl + 2 * KB;
    const bool more = kt + 1 < ntiles;
    if (more) {
      if constexpr (PS) load_ps(kt + 1);
      else st.load(a, b, h, kt + 1, tid);
    }
    if (wave_live) {
      // (fragments read at their use: reading all 16 up front measured 1.85 vs 1.76 ms per
      // B = 64 launch -- 172 instead of 164 VGPRs, a wave per SIMD less)
      f32x16 s0, s1;
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        f32x16& s = sub ? s1 : s0;
        s = negm;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int ko = k_off_bf16(sub * 32 + r32, 2 * i + hh);
          const u32x4 kh = ld16(kl + ko), klo = ld16(kl + KB + ko);
          s = mf(klo, qh[i], s);
          s = mf(kh, ql[i], s);
          s = mf(kh, qh[i], s);
        }
      }
      // lazy rescale (the bf16 kernel's rule): the running max moves only when some lane's tile
      // max passed it by more than RESCALE_SLACK, so p <= 2^8 -- exact-range fp32 for p, l, o and
      // the hi / lo split; the first tile sets m.  p = exp2 by the bare v_exp_f32 (exp2f's
      // denormal-range scaling costs 4 VALU per score; p < 2^-126 is below any sum's ulp).
      const float mx = tile_max(s0, s1, kt * KT, a.Tk, hh);
      if (kt == 0 || __any(mx > RESCALE_SLACK)) {
        const float d = kt == 0 ? mx : __builtin_fmaxf(mx, 0.f);
        if (kt != 0) {
          const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
          for (int r = 0; r < 16; ++r) o[r] *= alpha;
          l *= alpha;
        }
        m += d;
#pragma unroll
        for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
      }
      float t0 = 0.f, t1 = 0.f, t2 = 0.f, t3 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        s0[r] = __builtin_amdgcn_exp2f(s0[r]);
        s0[r + 1] = __builtin_amdgcn_exp2f(s0[r + 1]);
        s1[r] = __builtin_amdgcn_exp2f(s1[r]);
        s1[r + 1] = __builtin_amdgcn_exp2f(s1[r + 1]);
        t0 += s0[r];
        t1 += s0[r + 1];
        t2 += s1[r];
        t3 += s1[r + 1];
      }
      l += (t0 + t1) + (t2 + t3);
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const f32x16& p = sub ? s1 : s0;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          uint32_t hw[4], lw[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v0 = p[8 * ks + 2 * e], v1 = p[8 * ks + 2 * e + 1];
            hw[e] = pack_bf16x2(v0, v1);
            lw[e] = pack_bf16x2(v0 - __uint_as_float(hw[e] << 16), v1 - __uint_as_float(hw[e] & 0xffff0000u));
          }
          const u32x4 ph{hw[0], hw[1], hw[2], hw[3]}, pl{lw[0], lw[1], lw[2], lw[3]};
          const int vo = r32 * VROW + (2 * sub + ks) * 32 + hh * 16;
          const u32x4 vh = ld16(vl + vo), vlo = ld16(vl + VB + vo);
          o = mf(vlo, ph, o);
          o = mf(vh, pl, o);
          o = mf(vh, ph, o);
        }
      }
    }
    if (more) {
      if constexpr (PS) store_ps(smem + ((kt + 1) & 1) * SLOT);
      else store(smem + ((kt + 1) & 1) * SLOT);
    }
    __syncthreads();
  }

  if (!wave_live || q >= a.Tq) return;
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = 1.f / lt;
  float* op = (float*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    // O^T accumulator rows: dims 8g + 4hh + (0..3), the bf16 kernel's output order
    float v[4] = {o[4 * g] * inv, o[4 * g + 1] * inv, o[4 * g + 2] * inv, o[4 * g + 3] * inv};
    st16(op + 8 * g + 4 * hh, pack16<float>(v));
  }
}

}  // namespace

int spe_launch_attention(const AttnArgs& a, int dtype, hipStream_t s) {
  if (a.B <= 0 || a.Tq <= 0 || a.Tk <= 0) return 0;
  const int ce = (dtype == SPE_DTYPE_F32 || dtype == SPE_DTYPE_F32X3) ? 4 : 8;
  if ((a.ldq % ce) || (a.ldk % ce) || (a.ldo % 4)) return -5;
  if (a.presplit && (dtype != SPE_DTYPE_F32X3 || a.Tk % 8 || a.ldk % 8)) return -5;
  if (a.v_f16 && !(a.presplit && a.vt_swz)) return -5;
  if (a.presplit && a.vt_swz) {                    // V^T planes in vt_pos order: the LDS-DMA split kernel
    const int rc = spe_launch_attention_split(a, s);
    return rc == 1 ? -5 : rc;
  }
  dim3 grid(a.B * a.H * ((a.Tq + 127) / 128)), block(NT);
  if (a.vt_swz && (a.Tk % 16 || (dtype != SPE_DTYPE_F16 && dtype != SPE_DTYPE_BF16 && dtype != SPE_DTYPE_BF16_F16V)))
    return -5;                                     // (swizzled V^T: 16-bit operands, whole quads per row)
  if (a.vt_swz) {                                  // LDS-DMA staging (the only reader of that layout)
    grid = dim3(a.B * a.H * ((a.Tq + 32 * DMA_WAVES - 1) / (32 * DMA_WAVES)));
    block = dim3(64 * DMA_WAVES);
    if (dtype == SPE_DTYPE_F16) {
      if (a.Tq >= 128) hipLaunchKernelGGL((attn16_kernel<0, f16, f16, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((attn16_kernel<1, f16, f16, true>), grid, block, 0, s, a);
    } else if (dtype == SPE_DTYPE_BF16_F16V) {
      if (a.Tq >= 128) hipLaunchKernelGGL((attn16_kernel<0, bf16, f16, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((attn16_kernel<1, bf16, f16, true>), grid, block, 0, s, a);
    } else {
      if (a.Tq >= 128) hipLaunchKernelGGL((attn16_kernel<0, bf16, bf16, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((attn16_kernel<1, bf16, bf16, true>), grid, block, 0, s, a);
    }
    return (int)hipGetLastError();
  }
  if (dtype == SPE_DTYPE_F16)
    if (a.Tq >= 128)
      hipLaunchKernelGGL((attn16_kernel<0, f16>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((attn16_kernel<1, f16>), grid, block, 0, s, a);
  else if (dtype == SPE_DTYPE_BF16_F16V)
    if (a.Tq >= 128)
      hipLaunchKernelGGL((attn16_kernel<0, bf16, f16>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((attn16_kernel<1, bf16, f16>), grid, block, 0, s, a);
  else if (dtype == SPE_DTYPE_BF16)
    if (a.Tq >= 128)
      hipLaunchKernelGGL((attn16_kernel<0, bf16>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((attn16_kernel<1, bf16>), grid, block, 0, s, a);
  else if (dtype == SPE_DTYPE_F32X3 && a.presplit)
    hipLaunchKernelGGL(attn_x3_kernel<true>, grid, block, 0, s, a);
  else if (dtype == SPE_DTYPE_F32X3)
    hipLaunchKernelGGL(attn_x3_kernel<false>, grid, block, 0, s, a);
  else
    hipLaunchKernelGGL(attn_f32_kernel, grid, block, 0, s, a);
  return (int)hipGetLastError();
}
