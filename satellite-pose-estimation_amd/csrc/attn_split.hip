// Encoder self-attention of the fp32 accuracy modes (fp32h3, fp32x3, fp32x6) on split operands,
// REV/models/transformer.py:158-161 (nn.MultiheadAttention's score / softmax / value product at
// head_dim 32), fp32 q in, fp32 out.
//
// Operands arrive pre-split by the projection epilogues (gemm.hip, GemmArgs::S): K as bf16 hi / lo
// planes [B*Tk][ldk], V^T as hi / lo planes [B][H][32][Tk] in vt_pos key order -- bf16 (fp32x3 /
// fp32x6) or, in the fp32h3 model, fp16 of V * 2^-ev with the power of two from a bound on |V|
// (vplane_scale, spe_common.h).  Scores: S^T = K.Q^T as three bf16 32x32x16 MFMAs per product
// (klo.qhi + khi.qlo + khi.qhi, q split in registers after the exp2-domain prescale); value product:
// three MFMAs per product on the P split -- fp16 with fp16 V planes (P <= 2^12, hi = RTZ(p),
// lo = RNE(p - hi): 2^-21 relative per p), bf16 otherwise.
//
// Against the register-staged attn_x3_kernel (attention.hip) this kernel: stages the four planes of a
// 64-key tile global -> LDS by buffer_load ... lds through a ring of NSLOT = 4 slots (each wave issues
// one 1 KB piece of each plane per tile, two tiles ahead, one barrier per tile, no staging registers
// or ds_writes); reads every fragment at a per-lane base + immediate offset (the loop unrolled by the
// ring's slots); masks keys only in a tile that reaches past Tk; skips the per-tile max (lazy softmax,
// the bf16 DMA kernel's rule: a tile is exponentiated against the stale running max and its fp32 row
// sum is the overflow test -- only a lane sum above LAZY_LIMIT, i.e. some p > 2^12, recomputes the
// scores from the K tile still in LDS and takes the max / rescale path); splits P to fp16 with one
// v_cvt_pkrtz_f16_f32 per pair and v_fma_mix for the remainders (3 VALU per pair against 6 for the
// bf16 split); and software-pipelines the tiles: step kt issues tile kt+1's score MFMAs with tile kt's
// exp2 / row sums in their gaps (sched_group_barrier), then tile kt's value product with the P split
// in its gaps.  Built with -fno-slp-vectorize: the row sums stay scalar v_add_f32 (packed f32 adds
// beside MFMAs cost more issue than they save, MI355X_MICROARCH.md).
//
// Measured (kbench, B = 64, 2704 tokens, fp16 V planes): 1.74 ms for attn_x3_kernel -> 1.50 ms; the
// PMC passes put the SIMD's instruction issue at ~87 % busy (2 waves x 1066 issue cycles per 2453-cycle
// wave-tile), MFMA 57 % at 1.51 GHz.  Per 64-key tile and wave the issue floor is ~24 MFMA x 8 + 32
// v_exp x 8 + 32 sums + 48 split VALU = ~830 cycles against 768 matrix cycles.  P as one RNE fp16 term
// (no lo part: 20 instead of 24 MFMAs, 1.26 ms) moved the bench keypoints 1.7e-4 from exact f32 and
// failed the precision gate (tests/test_gpu_precision.py): the split stays.
#include "spe_common.h"
#include "spe_kernels.h"
#include <type_traits>

namespace {

constexpr int NT = 256;                 // 4 waves x 32 queries
constexpr int KT = 64;                  // keys per tile
constexpr int PLANE = 4096;             // one plane of a tile: K 64 keys x 64 B / V^T 32 rows x 128 B
constexpr int SLOT = 4 * PLANE;         // [K hi | K lo | V^T hi | V^T lo]
#ifndef SPE_SPLIT_SLOTS
#define SPE_SPLIT_SLOTS 4
#endif
constexpr int NSLOT = SPE_SPLIT_SLOTS;  // LDS ring depth: 3 (48 KB, three work-groups per CU) or 4
static_assert(NSLOT == 3 || NSLOT == 4, "ring");
constexpr float LOG2E = 1.4426950408889634f;
constexpr float NEG_BIG = -1.0e30f;
constexpr float RESCALE_SLACK = 8.0f;
constexpr float LAZY_LIMIT = 4096.0f;

constexpr int waitcnt_vm(int vm) { return (vm & 15) | ((vm >> 4) << 14) | (7 << 4) | (15 << 8); }
typedef __attribute__((address_space(3))) void* lds_ptr_t;

SPE_DEV f32x16 mfma_bf(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
SPE_DEV f32x16 mfma_h(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// Keys past Tk (the last tile; Tk % 16 == 0): registers 0-7 of s0 hold keys 0-15 of the tile, 8-15
// keys 16-31, s1 the next 32 -- whole 16-key groups, four wave-uniform tests
SPE_DEV void mask16(f32x16& s0, f32x16& s1, int key_base, int Tk) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
    if (key_base + 16 * g >= Tk) {
      f32x16& s = g < 2 ? s0 : s1;
#pragma unroll
      for (int r = 0; r < 8; ++r) s[8 * (g & 1) + r] = NEG_BIG;
    }
}

// the lane pair's max over its 32 scores (v_max3 chains, one permlane32 exchange)
SPE_DEV float pair_max(const f32x16& s0, const f32x16& s1) {
  float ma = __builtin_fmaxf(s0[0], s1[0]), mb = __builtin_fmaxf(s0[1], s1[1]);
#pragma unroll
  for (int r = 2; r < 16; r += 2) {
    ma = __builtin_fmaxf(__builtin_fmaxf(ma, s0[r]), s1[r]);
    mb = __builtin_fmaxf(__builtin_fmaxf(mb, s0[r + 1]), s1[r + 1]);
  }
  const float mx = __builtin_fmaxf(ma, mb);
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
  return __builtin_fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
}

template <bool F16V>
__global__ __launch_bounds__(NT, NSLOT == 3 ? 3 : 2) void attn_split_kernel(AttnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hh = lane >> 5, r32 = lane & 31;
  const int qblocks = (a.Tq + 127) / 128;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = bid / qblocks, qb = bid - bh * qblocks;
  const int b = bh / a.H, h = bh - b * a.H;
  const int q = qb * 128 + wid * 32 + r32;
  // (wave-uniform, made scalar so the tile loop branches instead of running both sides under exec)
  const bool wave_live = __builtin_amdgcn_readfirstlane(qb * 128 + wid * 32 < a.Tq ? 1 : 0) != 0;

  // query fragments (B operand of S^T = K . Q^T): dims 16i + 8hh + (0..7), scaled into the exp2
  // domain in fp32, split into bf16 hi / lo
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
  // formed before the DMA stream starts (vmcnt is in-order: a q load left for the loop would drain
  // the ring at its first use)
  asm volatile("" ::"v"(qh[0]), "v"(qh[1]), "v"(ql[0]), "v"(ql[1]));

  // ---- DMA: per (image, head) descriptors over the four planes (reads past Tk return zeros);
  // this wave issues piece `wid` of each plane per tile.  K image: key rows of 64 B, chunk c at slot
  // c ^ ((key >> 2) & 3); V^T image: rows of 128 B, chunk c at slot c ^ ((d >> 1) & 7) -- the
  // swizzle on the source address, the LDS side lane-linear.
  const int bu = __builtin_amdgcn_readfirstlane(b), hu = __builtin_amdgcn_readfirstlane(h);
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const size_t klo = (size_t)a.B * a.Tk * a.ldk * 2, vlo = (size_t)a.B * a.H * 32 * a.Tk * 2;   // bytes
  const char* kb = (const char*)a.k + ((size_t)bu * a.Tk * a.ldk + hu * 32) * 2;
  const char* vb = (const char*)a.vt + (size_t)(bu * a.H + hu) * 32 * a.Tk * 2;
  const __amdgpu_buffer_rsrc_t rkh = __builtin_amdgcn_make_buffer_rsrc((void*)kb, (short)0, a.Tk * a.ldk * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rkl = __builtin_amdgcn_make_buffer_rsrc((void*)(kb + klo), (short)0, a.Tk * a.ldk * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rvh = __builtin_amdgcn_make_buffer_rsrc((void*)vb, (short)0, 32 * a.Tk * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rvl = __builtin_amdgcn_make_buffer_rsrc((void*)(vb + vlo), (short)0, 32 * a.Tk * 2, 0x00020000);
  int kvo, vvo;
  {
    const int key = wu * 16 + (lane >> 2), c = (lane & 3) ^ ((key >> 2) & 3);
    kvo = key * a.ldk * 2 + c * 16;
    const int d = wu * 8 + (lane >> 3), cv = (lane & 7) ^ ((d >> 1) & 7);
    vvo = (d * a.Tk + cv * 8) * 2;
  }
  auto issue = [&](int kt, int slot) {
    char* base = smem + slot * SLOT + wu * 1024;
    const int ks = kt * KT * a.ldk * 2, vs = kt * KT * 2;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rkh, (lds_ptr_t)(base), 16, kvo, ks, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rkl, (lds_ptr_t)(base + PLANE), 16, kvo, ks, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rvh, (lds_ptr_t)(base + 2 * PLANE), 16, vvo, vs, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rvl, (lds_ptr_t)(base + 3 * PLANE), 16, vvo, vs, 0, 0);
  };

  // fragment offsets in a slot: K (key sub*32 + r32, chunk 2i + hh), V^T (row r32, the chunk of keys
  // sub*32 + 16ks + 8hh in vt_pos order = chunk 2(2sub + ks) + hh); sub / plane / slot are immediates
  const int ks2 = (r32 >> 2) & 3;
  const int ko0 = r32 * 64 + ((hh ^ ks2) << 4), ko1 = r32 * 64 + (((2 + hh) ^ ks2) << 4);
  int vo[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) vo[j] = r32 * 128 + (((2 * j + hh) ^ ((r32 >> 1) & 7)) << 4);

  f32x16 o, negm;                       // O^T accumulator; -m in every element (score MFMAs start there)
#pragma unroll
  for (int r = 0; r < 16; ++r) { o[r] = 0.f; negm[r] = 0.f; }
  float m = 0.f, l = 0.f;
  const int ntiles = (a.Tk + KT - 1) / KT;
  issue(0, 0);
  if (ntiles > 1) issue(1, 1);
  if (NSLOT == 4 && ntiles > 2) issue(2, 2);

  auto scores = [&](const char* sl, f32x16& s0, f32x16& s1) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16& s = sub ? s1 : s0;
      const u32x4 kh0 = ld16(sl + sub * 2048 + ko0), kl0 = ld16(sl + PLANE + sub * 2048 + ko0);
      const u32x4 kh1 = ld16(sl + sub * 2048 + ko1), kl1 = ld16(sl + PLANE + sub * 2048 + ko1);
      s = mfma_bf(kl0, qh[0], negm);
      s = mfma_bf(kh0, ql[0], s);
      s = mfma_bf(kh0, qh[0], s);
      s = mfma_bf(kl1, qh[1], s);
      s = mfma_bf(kh1, ql[1], s);
      s = mfma_bf(kh1, qh[1], s);
    }
  };
  // keys past Tk (only a last tile that reaches past it; wave-uniform tests)
  auto mask = [&](int kt, f32x16& s0, f32x16& s1) {
    if ((kt + 1) * KT > a.Tk) mask16(s0, s1, kt * KT, a.Tk);
  };
  // the max path: the first tile sets m; later ones move it (rescaling o and l) only when some lane's
  // tile max passed it by more than RESCALE_SLACK.  Returns the shift d applied to m.
  auto maxpath = [&](bool first, f32x16& s0, f32x16& s1) {
    const float mx = pair_max(s0, s1);     // relative to m
    float d = 0.f;
    if (first || __any(mx > RESCALE_SLACK)) {
      d = first ? mx : __builtin_fmaxf(mx, 0.f);
      if (!first) {
        const float alpha = __builtin_amdgcn_exp2f(-d);
#pragma unroll
        for (int r = 0; r < 16; ++r) o[r] *= alpha;
        l *= alpha;
      }
      m += d;
#pragma unroll
      for (int r = 0; r < 16; ++r) { s0[r] -= d; s1[r] -= d; negm[r] = -m; }
    }
    return d;
  };
  // exp2 of the shifted scores in place and the lane's row sum over its 32 keys
  auto expsum = [&](f32x16& s0, f32x16& s1) {
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
    return (t0 + t1) + (t2 + t3);
  };
  // value product O^T += V^T . P^T of one tile, P split in registers
  auto pv = [&](const char* sl, const f32x16& s0, const f32x16& s1) {
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const f32x16& p = sub ? s1 : s0;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        uint32_t hw[4], lw[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v0 = p[8 * ks + 2 * e], v1 = p[8 * ks + 2 * e + 1];
          if constexpr (F16V) {
            // hi = RTZ pair; lo = RNE(p - hi) from the fp16 halves directly (v_fma_mix: -hi * 1 + p in
            // fp32, rounded to fp16 into one half of lo)
            hw[e] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v0, v1));
            uint32_t lo;
            asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hw[e]), "v"(v0));
            asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hw[e]), "v"(v1));
            lw[e] = lo;
          } else {
            hw[e] = pack_bf16x2(v0, v1);
            lw[e] = pack_bf16x2(v0 - __uint_as_float(hw[e] << 16), v1 - __uint_as_float(hw[e] & 0xffff0000u));
          }
        }
        const u32x4 ph{hw[0], hw[1], hw[2], hw[3]}, pl{lw[0], lw[1], lw[2], lw[3]};
        const u32x4 vh = ld16(sl + 2 * PLANE + vo[2 * sub + ks]), vl = ld16(sl + 3 * PLANE + vo[2 * sub + ks]);
        if constexpr (F16V) {
          o = mfma_h(vl, ph, o);
          o = mfma_h(vh, pl, o);
          o = mfma_h(vh, ph, o);
        } else {
          o = mfma_bf(vl, ph, o);
          o = mfma_bf(vh, pl, o);
          o = mfma_bf(vh, ph, o);
        }
      }
    }
  };

  // Software pipeline over the tiles: step kt issues the score MFMAs of tile kt+1 (into the other
  // score buffer) and, independent of them, exponentiates tile kt's scores computed one step earlier,
  // so the in-order wave fills the MFMA gaps with that VALU; then tile kt's value product.  Ring of
  // NSLOT slots, tile j in slot j % NSLOT: step kt reads K of tile kt+1 and V^T of tile kt; after its
  // barrier (every wave done with step kt-1) tile kt+NSLOT-1 goes into tile kt-1's slot.
  f32x16 sa0, sa1, sb0, sb1;
  {
    if (NSLOT == 4 && ntiles > 2) __builtin_amdgcn_s_waitcnt(waitcnt_vm(8));
    else if (ntiles > 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm(4));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    if (wave_live) {
      scores(smem, sa0, sa1);
      mask(0, sa0, sa1);
      maxpath(true, sa0, sa1);
    }
  }
  // SC: the slot of tile kt (compile-time: every fragment read is base + immediate offset)
  auto step = [&](int kt, auto SC, f32x16& c0, f32x16& c1, f32x16& n0, f32x16& n1) {
    constexpr int S = decltype(SC)::value;
    const char* sl = smem + S * SLOT;
    // tile kt+1 landed (NSLOT 4: tile kt+2's pieces may stay in flight); after the barrier tile kt+1 is
    // visible to all and tile kt-1's slot takes tile kt+NSLOT-1 (no fragment read of this step
    // touches that slot: the DMA goes out first)
    if (NSLOT == 4 && kt + 2 < ntiles) __builtin_amdgcn_s_waitcnt(waitcnt_vm(4));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    if (kt + NSLOT - 1 < ntiles) issue(kt + NSLOT - 1, (S + NSLOT - 1) % NSLOT);
    if (wave_live) {
      // tile kt+1's score MFMAs (the last step's read a stale slot: 12 MFMAs per work-group
      // row, unused) with tile kt's exp2 / row sums in their gaps: two v_exp_f32 and two v_add_f32
      // (24 issue cycles) per 32-cycle MFMA
      scores(smem + ((S + 1) % NSLOT) * SLOT, n0, n1);
      float t = expsum(c0, c1);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int i = 0; i < 12; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i == 1) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      }
      // lazy softmax: tile kt was shifted by the running max as it stood when its scores were
      // formed; a lane sum past LAZY_LIMIT (some p > 2^12) recomputes them from the K tile still in
      // its slot and takes the max path (tile kt+1's scores, formed with the old m, move by the
      // same shift)
      if (__any(t > LAZY_LIMIT)) {
        scores(sl, c0, c1);
        mask(kt, c0, c1);
        const float d = maxpath(false, c0, c1);
#pragma unroll
        for (int r = 0; r < 16; ++r) { n0[r] -= d; n1[r] -= d; }
        t = expsum(c0, c1);
      }
      l += t;
      pv(sl, c0, c1);
      constexpr int PM = 3, PS = 12;     // MFMAs / split VALU per 16-key group
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, PS, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < PM; ++j) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          if (j == 0 && g < 3) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
          if (g < 3) __builtin_amdgcn_sched_group_barrier(0x002, PS / PM, 0);
        }
      if (kt + 1 < ntiles) mask(kt + 1, n0, n1);
    }
  };
  using C0 = std::integral_constant<int, 0>;
  using C1 = std::integral_constant<int, 1>;
  using C2 = std::integral_constant<int, 2>;
  using C3 = std::integral_constant<int, NSLOT == 4 ? 3 : 0>;
  using C4 = std::integral_constant<int, NSLOT == 4 ? 0 : 1>;
  using C5 = std::integral_constant<int, NSLOT == 4 ? 1 : 2>;
  // unrolled by lcm(2, NSLOT) (score buffers alternate, ring slots cycle), slots as immediates
  constexpr int U = NSLOT == 4 ? 4 : 6;
  int kt = 0;
  for (; kt + U <= ntiles; kt += U) {
    step(kt, C0{}, sa0, sa1, sb0, sb1);
    step(kt + 1, C1{}, sb0, sb1, sa0, sa1);
    step(kt + 2, C2{}, sa0, sa1, sb0, sb1);
    step(kt + 3, C3{}, sb0, sb1, sa0, sa1);
    if constexpr (U == 6) {
      step(kt + 4, C4{}, sa0, sa1, sb0, sb1);
      step(kt + 5, C5{}, sb0, sb1, sa0, sa1);
    }
  }
  const int rest = ntiles - kt;
  if (rest >= 1) step(kt, C0{}, sa0, sa1, sb0, sb1);
  if (rest >= 2) step(kt + 1, C1{}, sb0, sb1, sa0, sa1);
  if (rest >= 3) step(kt + 2, C2{}, sa0, sa1, sb0, sb1);
  if (U == 6 && rest >= 4) step(kt + 3, C3{}, sb0, sb1, sa0, sa1);
  if (U == 6 && rest >= 5) step(kt + 4, C4{}, sa0, sa1, sb0, sb1);

  if (!wave_live || q >= a.Tq) return;
  const float lt = l + __shfl_xor(l, 32, 64);   // the lane pair's two key halves
  float inv = 1.f / lt;
  if constexpr (F16V) inv *= 1.f / vplane_scale(a.v_amax, a.v_l1, a.v_bmax);   // (a power of two)
  float* op = (float*)a.o + (size_t)(b * a.Tq + q) * a.ldo + h * 32;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    // O^T accumulator rows: dims 8g + 4hh + (0..3)
    float v[4] = {o[4 * g] * inv, o[4 * g + 1] * inv, o[4 * g + 2] * inv, o[4 * g + 3] * inv};
    st16(op + 8 * g + 4 * hh, pack16<float>(v));
  }
}

}  // namespace

// 1: not served (the caller takes attention.hip's register-staged split kernel)
int spe_launch_attention_split(const AttnArgs& a, hipStream_t s) {
  if (!a.presplit || !a.vt_swz || a.Tk % 16 || a.ldk % 8 || a.ldq % 4 || a.ldo % 4) return 1;
  if ((long long)a.Tk * a.ldk * 2 >= (1LL << 31) || (long long)32 * a.Tk * 2 >= (1LL << 31)) return 1;
  const dim3 grid(a.B * a.H * ((a.Tq + 127) / 128)), block(NT);
  if (a.v_f16) hipLaunchKernelGGL(attn_split_kernel<true>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(attn_split_kernel<false>, grid, block, 0, s, a);
  return (int)hipGetLastError();
}
