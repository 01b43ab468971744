// Shared device helpers for the gfx950 (CDNA4) keypoint-set pose path.
// Storage type T is either __bf16 (throughput path, fp32 accumulate) or float (parity path,
// exact-f32 MFMA).  Every kernel is written once for both, so the fp32 parity tests exercise
// the same tiling and indexing as the bf16 bench path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

#define SPE_DEV __device__ __forceinline__

SPE_DEV float to_f32(float x) { return x; }
SPE_DEV float to_f32(bf16 x) { return (float)x; }
template <typename T> SPE_DEV T from_f32(float x);
template <> SPE_DEV float from_f32<float>(float x) { return x; }
template <> SPE_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

// 16-byte chunk holds CE elements of T.
template <typename T> struct Chunk { static constexpr int CE = 16 / sizeof(T); };

// load / store 16 bytes
SPE_DEV u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
SPE_DEV void st16(void* p, u32x4 v) { *reinterpret_cast<u32x4*>(p) = v; }
SPE_DEV u32x2 ld8(const void* p) { return *reinterpret_cast<const u32x2*>(p); }
SPE_DEV void st8(void* p, u32x2 v) { *reinterpret_cast<u32x2*>(p) = v; }

// unpack a 16-byte chunk to floats / pack floats to a chunk
template <typename T> SPE_DEV void unpack16(u32x4 v, float* f);
template <> SPE_DEV void unpack16<float>(u32x4 v, float* f) {
  f[0] = __uint_as_float(v.x); f[1] = __uint_as_float(v.y);
  f[2] = __uint_as_float(v.z); f[3] = __uint_as_float(v.w);
}
template <> SPE_DEV void unpack16<bf16>(u32x4 v, float* f) {
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <typename T> SPE_DEV u32x4 pack16(const float* f);
template <> SPE_DEV u32x4 pack16<float>(const float* f) {
  return u32x4{__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])};
}
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
// two floats -> two RNE bf16 in one v_cvt_pk_bf16_f32 (two scalar casts + shift/or cost 4 VALU)
SPE_DEV uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, bf16x2));
}
template <> SPE_DEV u32x4 pack16<bf16>(const float* f) {
  return u32x4{pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7])};
}

// fp16 storage (encoder attention operands in the fp16-attention mode, BASELINE config 5)
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <> SPE_DEV f16 from_f32<f16>(float x) { return (f16)x; }
SPE_DEV uint32_t pack_f16x2(float lo, float hi) {                 // RNE
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, f16x2));
}
template <> SPE_DEV void unpack16<f16>(u32x4 v, float* f) {
  const f16x8 h = __builtin_bit_cast(f16x8, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)h[i];
}
template <> SPE_DEV u32x4 pack16<f16>(const float* f) {
  return u32x4{pack_f16x2(f[0], f[1]), pack_f16x2(f[2], f[3]), pack_f16x2(f[4], f[5]), pack_f16x2(f[6], f[7])};
}
// 16-bit GEMM outputs: bf16 unless the launch asked for fp16 (GemmArgs::out_f16).  fp16 outputs
// saturate at +-65504 instead of overflowing to inf (an inf V or q/k entry would turn the
// attention output into NaN); NaN stays NaN.
SPE_DEV float sat_f16(float v) { return fabsf(v) > 65504.f ? copysignf(65504.f, v) : v; }
SPE_DEV uint32_t pack_out2(float lo, float hi, bool f16o) {
  return f16o ? pack_f16x2(sat_f16(lo), sat_f16(hi)) : pack_bf16x2(lo, hi);
}
SPE_DEV u32x4 pack_out8(const float* f, bool f16o) {
  if (!f16o) return pack16<bf16>(f);
  float s[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = sat_f16(f[i]);
  return pack16<f16>(s);
}
SPE_DEV void store_out1(void* base, size_t i, float v, bool f16o) {
  if (f16o) reinterpret_cast<f16*>(base)[i] = (f16)sat_f16(v);
  else reinterpret_cast<bf16*>(base)[i] = (bf16)v;
}

SPE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SPE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Published max |x| of a tensor (the fp32h3 activation scales): a float >= 0 kept as its bit
// pattern, raised with an unsigned atomic max.  Every producing wave publishes, so the atomics of
// a launch all hit one L2 line: 10^5 of them serialise there for ~1 ms.  The slot is read first
// (a relaxed agent-scope load; a stale value is never larger than the current one, so a skipped
// update is always covered) and the atomic goes out only when this wave's value is larger --
// a few times per launch instead of once per wave.
SPE_DEV void amax_update(float* slot, float v) {
  const unsigned cur = __hip_atomic_load((unsigned*)slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__float_as_uint(v) > cur) atomicMax((unsigned*)slot, __float_as_uint(v));
}

// max over the work-group of the threads' am (>= 0) raised into slot (times mul when mul > 0) with
// ONE atomic: every thread of the block calls it (blockDim.x a multiple of 64); red = LDS scratch of
// blockDim.x / 64 floats that no thread reads or writes any more (barriers on both sides).  The
// work-groups of a small launch end together, and per-wave atomics on the one slot serialize.
SPE_DEV void amax_publish_block(float am, float* slot, float mul, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = am;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) am = fmaxf(am, red[w]);
    if (am > 0.f) amax_update(slot, am * (mul > 0.f ? mul : 1.f));
  }
}

// Bijective XCD-aware remap of a 1-D grid: blocks that land on one XCD (b % 8 equal under
// round-robin dispatch) get a contiguous range of tile ids, so neighbouring tiles that share
// operand panels hit the same L2.  Speed only, never correctness.
SPE_DEV int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = bid & 7, idx = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// epilogue activation (ACT_* in spe_kernels.h); SiLU as torch's x / (1 + exp(-x)), GELU exact
SPE_DEV float apply_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return v / (1.f + expf(-v));
  if (act == 3) return 0.5f * v * (1.f + erff(v * 0.7071067811865476f));
  return v;
}

// LDS weight images of KB-byte rows read as 16x16x32 bf16 fragments (lane -> row 16j + (lane & 15),
// 16-byte chunk 4kf + (lane >> 4)): chunk c of row n sits at slot c ^ (n & wkey_mask(KB)).  With
// the mask min(KB/16, 16) - 1 the 16 lanes of every gfx950 ds_read_b128 lane group hit 16
// distinct 16-byte bank groups for any KB >= 128; the older 128-byte-group form (chunk & 7) ^
// (n & 7) left half of the banks unused for KB >= 256 (2-way conflicts: 28-45 % of the LDS
// cycles of the bottleneck-tail kernels).
SPE_DEV constexpr int wkey_mask(int KB) { return (KB / 16 < 16 ? KB / 16 : 16) - 1; }
SPE_DEV constexpr int wkey_addr(int n, int chunk, int KB) { return n * KB + ((chunk ^ (n & wkey_mask(KB))) << 4); }

// fp16 hi / lo planes of a tensor with a bounded range (GemmArgs::s_f16 -> AttnArgs::v_f16): the
// factor 2^(14 - e) applied before the split, with bound = amax * l1 + bmax in [2^(e-1), 2^e), keeps
// every scaled |x| below 2^14 (fp16 max 65504); 1 without a finite positive bound.  Producer and
// consumer evaluate this same expression on the same inputs, so they agree on the power of two.
SPE_DEV float vplane_scale(const float* amax, float l1, float bmax) {
  if (!amax) return 1.f;
  const float bound = __builtin_fmaf(*amax, l1, bmax);
  if (!(bound > 0.f) || !(bound <= 3.0e38f)) return 1.f;
  return __builtin_ldexpf(1.f, 14 - __builtin_amdgcn_frexp_expf(bound));
}
// four fp32 values -> fp16 hi = RNE(x) and lo = RNE(x - hi) (x - hi exact in fp32), two words each
SPE_DEV void split_f16x4(const float* v, u32x2& h, u32x2& l) {
  const f16x2 h0 = __builtin_convertvector(f32x2{v[0], v[1]}, f16x2), h1 = __builtin_convertvector(f32x2{v[2], v[3]}, f16x2);
  h = u32x2{__builtin_bit_cast(uint32_t, h0), __builtin_bit_cast(uint32_t, h1)};
  l = u32x2{pack_f16x2(v[0] - (float)h0[0], v[1] - (float)h0[1]), pack_f16x2(v[2] - (float)h1[0], v[3] - (float)h1[1])};
}
