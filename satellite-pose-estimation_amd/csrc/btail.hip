// Bottleneck tail + next conv1 in one streaming pass (ResNet-50 layer 1, REV/models/backbone.py
// :114-125, torchvision Bottleneck):
//
//     y = relu(A . W3^T + b3 (+ R))          conv3 1x1 + bn3 (+ identity) + relu   -> stored
//     z = relu(y . W1^T + b1)                the NEXT block's conv1 1x1 + bn1 + relu -> stored
//
// The separate launches read y back from HBM right after writing it (354 MB per 64-image layer-1
// boundary); here y goes to HBM once (it is the next block's residual) and feeds the second
// product from registers.  y is N1 = 256 channels, the conv3 input K1 = 64 (or 128: block 0's
// [conv2 output | max-pool output] concatenation, registry.cpp c3ds), the next conv1 N2 = 64
// (layer 1) or 128 (layer 2 block 0).
//
// * Persistent workgroup of 8 waves per CU; W3 and W1 live in LDS for the kernel's life
//   (XOR-swizzled 16-byte chunks, conflict-free fragment reads).  Each wave streams 16-row
//   tiles: A and R of the next tile are loaded before the current one is multiplied.
// * First product in the C^T form MFMA(W3, A): a lane owns row m = fr and channels
//   16 j + 4 fg + r of y -- the store layout (8-byte row pieces) and, packed to bf16, the
//   operand of the second product without any data movement: for K-chunk kc the lane's 8
//   elements are channels 32 kc + 4 fg + {0..3} and 32 kc + 16 + 4 fg + {0..3}.  W1 is stored
//   with its columns permuted the same way (btail_perm, registry.cpp), so MFMA(W1p, y) pairs
//   them correctly; z is exact up to the MFMA's internal summation order.
#include "spe_common.h"
#include "spe_kernels.h"

#include <algorithm>
#include <cstdlib>

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;
constexpr int N1 = 256, NT = 512, NW = 8;

template <int K1, int N2, bool HAS_R>
__global__ __launch_bounds__(NT, 1) void btail_kernel(BtailArgs a, int row_tiles) {
  constexpr int KB1 = K1 * 2, KF1 = K1 / 32;          // W3 row bytes, K fragments of the first product
  constexpr int KB2 = N1 * 2;                          // W1 row bytes (K2 = N1)
  constexpr int J1 = N1 / 16, J2 = N2 / 16;            // column fragments
  __shared__ __attribute__((aligned(1024))) char w3s[N1 * KB1];
  __shared__ __attribute__((aligned(1024))) char w1s[N2 * KB2];
  __shared__ __attribute__((aligned(16))) float sb3[N1], sb1[N2];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fg = lane >> 4, fr = lane & 15;
  // ---- weights -> LDS.  Row n, 16-byte chunk c at n*KB + (c ^ (n & wkey_mask(KB)))*16; one
  // direct-to-LDS wave instruction fills 1 KB linearly, the swizzle applied on the source.
  {
    constexpr int INS3 = N1 * KB1 / 1024, INS1 = N2 * KB2 / 1024;
    for (int q = wid; q < INS3 + INS1; q += NW) {
      const bool first = q < INS3;
      const int qq = first ? q : q - INS3, KB = first ? KB1 : KB2;
      const int o = qq * 1024 + lane * 16;
      const int n = o / KB, within = o - n * KB;
      const int chunk = (within >> 4) ^ (n & wkey_mask(KB));
      const char* src = first ? (const char*)a.w3 + (size_t)n * a.ld3 * 2 + chunk * 16
                              : (const char*)a.w1 + (size_t)n * a.ld1 * 2 + chunk * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_ptr_t)((first ? w3s : w1s) + qq * 1024), 16, 0, 0);
    }
    for (int i = tid; i < N1; i += NT) sb3[i] = a.b3[i];
    for (int i = tid; i < N2; i += NT) sb1[i] = a.b1[i];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  auto w_addr = [](int n, int chunk, int KB) { return wkey_addr(n, chunk, KB); };

  auto load_a = [&](int t, u32x4 (&x)[KF1]) {
    t = t < row_tiles ? t : row_tiles - 1;
    int m = t * 16 + fr;
    m = m < a.M ? m : a.M - 1;
    const char* p = (const char*)a.A + (size_t)m * a.lda * 2 + fg * 16;
#pragma unroll
    for (int kf = 0; kf < KF1; ++kf) x[kf] = ld16(p + kf * 64);
  };
  auto load_r = [&](int t, u32x2 (&r)[HAS_R ? J1 : 1]) {
    if constexpr (HAS_R) {
      t = t < row_tiles ? t : row_tiles - 1;
      int m = t * 16 + fr;
      m = m < a.M ? m : a.M - 1;
      const char* p = (const char*)a.R + ((size_t)m * a.ldr + 4 * fg) * 2;
#pragma unroll
      for (int j = 0; j < J1; ++j) r[j] = ld8(p + j * 32);
    }
  };

  const int G = gridDim.x;
  const int stride = G * NW;
  const int t0 = xcd_remap(blockIdx.x, G) * NW + wid;
  if (t0 >= row_tiles) return;
  auto tile = [&](int t, const u32x4 (&ab)[KF1], const u32x2 (&rb)[HAS_R ? J1 : 1]) {
    // (a compiler-only fence: the weight fragments are loop-invariant LDS reads, and hoisting
    // them out of the tile loop would pin 256 registers)
    asm volatile("" ::: "memory");
    f32x4 acc[J1];
#pragma unroll
    for (int j = 0; j < J1; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kf = 0; kf < KF1; ++kf) {
      const bf16x8 av = __builtin_bit_cast(bf16x8, ab[kf]);
#pragma unroll
      for (int j = 0; j < J1; ++j) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, ld16(w3s + w_addr(16 * j + fr, 4 * kf + fg, KB1)));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, av, acc[j], 0, 0, 0);
      }
    }
    // ---- y = relu(acc + b3 (+ R)): store, and pack as the second product's operand
    const int m = t * 16 + fr;
    const bool ok = m < a.M;
    char* yp = (char*)a.y + ((size_t)m * a.ldy + 4 * fg) * 2;
    u32x2 yw[J1];
#pragma unroll
    for (int j = 0; j < J1; ++j) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sb3 + 16 * j + 4 * fg);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc[j][e] + bv[e];
      if constexpr (HAS_R) {
        v[0] += __uint_as_float(rb[j].x << 16);
        v[1] += __uint_as_float(rb[j].x & 0xffff0000u);
        v[2] += __uint_as_float(rb[j].y << 16);
        v[3] += __uint_as_float(rb[j].y & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      yw[j] = u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])};
      if (ok) st8(yp + j * 32, yw[j]);
    }
    // ---- z = relu(y . W1^T + b1), K-chunk kc = column fragments 2kc, 2kc+1 of y
    f32x4 acc2[J2];
#pragma unroll
    for (int j = 0; j < J2; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < N1 / 32; ++kc) {
      const bf16x8 yv = __builtin_bit_cast(bf16x8, u32x4{yw[2 * kc].x, yw[2 * kc].y, yw[2 * kc + 1].x, yw[2 * kc + 1].y});
#pragma unroll
      for (int j = 0; j < J2; ++j) {
        const bf16x8 w = __builtin_bit_cast(bf16x8, ld16(w1s + w_addr(16 * j + fr, 4 * kc + fg, KB2)));
        acc2[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, yv, acc2[j], 0, 0, 0);
      }
    }
    asm volatile("" ::: "memory");
    char* zp = (char*)a.z + ((size_t)m * a.ldz + 4 * fg) * 2;
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const f32x4 bv = *reinterpret_cast<const f32x4*>(sb1 + 16 * j + 4 * fg);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(acc2[j][e] + bv[e], 0.f);
      if (ok) st8(zp + j * 32, u32x2{pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])});
    }
  };

  // two operand sets in rotation (unrolled by two: register arrays are never indexed at run
  // time): the next tile's A and R are in flight while the current tile is multiplied
  u32x4 a0[KF1], a1[KF1];
  u32x2 r0[HAS_R ? J1 : 1], r1[HAS_R ? J1 : 1];
  load_a(t0, a0);
  load_r(t0, r0);
  for (int t = t0;;) {
    load_a(t + stride, a1);
    load_r(t + stride, r1);
    tile(t, a0, r0);
    t += stride;
    if (t >= row_tiles) break;
    load_a(t + stride, a0);
    load_r(t + stride, r0);
    tile(t, a1, r1);
    t += stride;
    if (t >= row_tiles) break;
  }
}

template <int K1, int N2, bool HAS_R>
int launch(const BtailArgs& a, hipStream_t s) {
  const int row_tiles = (a.M + 15) / 16;
  const int G = spe_cu_count();
  hipLaunchKernelGGL((btail_kernel<K1, N2, HAS_R>), dim3(G), dim3(NT), 0, s, a, row_tiles);
  return (int)hipGetLastError();
}

}  // namespace

// K-order permutation of the second product's weights (header above): stored column
// 32 kc + 8 g + e holds channel 32 kc + (e < 4 ? 4 g + e : 16 + 4 g + e - 4).
int spe_btail_perm(int k) {
  const int kc = k >> 5, g = (k >> 3) & 3, e = k & 7;
  return 32 * kc + (e < 4 ? 4 * g + e : 16 + 4 * g + e - 4);
}

bool spe_btail_enabled() {
  static const int on = [] { const char* e = getenv("SPE_BTAIL"); return e ? atoi(e) : 1; }();
  return on != 0;
}

// 1 = not a problem for this kernel
int spe_launch_btail(const BtailArgs& a, hipStream_t s) {
  if (a.M <= 0) return 0;
  if (a.lda % 8 || a.ldy % 4 || a.ldz % 4 || (a.R && a.ldr % 4) || a.ld3 < a.k1 || a.ld1 < a.n1) return 1;
  if (a.n1 != N1) return 1;
  if (a.k1 == 64 && a.n2 == 64 && a.R) return launch<64, 64, true>(a, s);
  if (a.k1 == 64 && a.n2 == 128 && a.R) return launch<64, 128, true>(a, s);
  if (a.k1 == 128 && a.n2 == 64 && !a.R) return launch<128, 64, false>(a, s);
  return 1;
}
