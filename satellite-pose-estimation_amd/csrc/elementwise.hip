// HBM-bound helpers of the backbone / transformer, vectorised 16 B per lane.
//   pack_input   NCHW fp32 crop batch (REV/datasets/speed.py:25-41 output contract), or the 8-bit
//                crops it is normalised from -> NHWC with channels padded to 8 (stem operand)
//   maxpool3s2   torchvision ResNet stem max-pool (3x3, stride 2, pad 1)
//   upsample2x   nn.UpsamplingBilinear2d(scale_factor=2) == align_corners=True
//                (REV/models/backbone.py:127,141)
//   layernorm    nn.LayerNorm(256, eps=1e-5), one wave per row, two-pass variance
//                (REV/models/transformer.py:147-148,165,167,194-196,117-124)
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

// input sources of the pack kernels: three channel values of pixel hw of image b
struct SrcF32 {
  const float* p; int S;
  SPE_DEV void load(size_t b, size_t hw, float v[3]) const {
    const float* src = p + b * 3 * S * S + hw;
    v[0] = src[0]; v[1] = src[(size_t)S * S]; v[2] = src[2 * (size_t)S * S];
  }
};
// 8-bit crops [B][S][S][C]: to_tensor (u8 / 255) + Normalize ((x - mean) / std), fp32, IEEE division
// (ch = 1: one gray value feeds all three channels, as Image.convert('RGB') replicates it)
struct SrcU8 {
  const uint8_t* p; int S, C;
  SPE_DEV void load(size_t b, size_t hw, float v[3]) const {
    const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
    const uint8_t* src = p + (b * S * S + hw) * C;
#pragma unroll
    for (int c = 0; c < 3; ++c) v[c] = ((float)src[C == 1 ? 0 : c] / 255.f - mean[c]) / stdv[c];
  }
};

template <typename T, int CP = 8, typename Src = SrcF32>
__global__ void pack_input_kernel(Src img, T* __restrict__ out, int B, int S, float* amax) {
  const size_t npx = (size_t)B * S * S;
  float am = 0.f;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < npx; p += (size_t)gridDim.x * blockDim.x) {
    const size_t b = p / ((size_t)S * S), hw = p - b * S * S;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    img.load(b, hw, v);
    am = fmaxf(am, fmaxf(fabsf(v[0]), fmaxf(fabsf(v[1]), fabsf(v[2]))));
    if constexpr (sizeof(T) == 2) {
      st16(out + p * 8, pack16<T>(v));
    } else if constexpr (CP == 4) {
      st16(out + p * 4, pack16<T>(v));
    } else {
      st16(out + p * 8, pack16<T>(v));
      st16(out + p * 8 + 4, pack16<T>(v + 4));
    }
  }
  if (amax) {                                    // every lane reaches here (grid-stride loop)
    __shared__ float wm[4];                        // one slot update per workgroup (256 threads)
    am = wave_max(am);
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = am;
    __syncthreads();
    if (threadIdx.x == 0) {
      am = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
      if (am > 0.f) amax_update(amax, am);
    }
  }
}

// bf16 stem input for the pair-packed stem (forward.cpp): [B][S+6][S+6][4] with the conv's
// 3-pixel zero border materialised (channel 3 zero), so a 16-byte chunk is two horizontally
// adjacent pixels and every tap of the 7x7/s2 window is in range.  The border is rewritten on
// every call (the buffer is shared with later activations).
template <typename Src>
__global__ void pack_input_pad4_kernel(Src img, bf16* __restrict__ out, int B, int S) {
  const int P = S + 6;
  const size_t npx = (size_t)B * P * P;
  for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < npx; p += (size_t)gridDim.x * blockDim.x) {
    const size_t b = p / ((size_t)P * P);
    const int r = (int)(p - b * P * P), y = r / P - 3, x = r % P - 3;
    u32x2 v{0, 0};
    if (y >= 0 && y < S && x >= 0 && x < S) {
      float c[3];
      img.load(b, (size_t)y * S + x, c);
      v = u32x2{pack_bf16x2(c[0], c[1]), pack_bf16x2(c[2], 0.f)};
    }
    st8(out + p * 4, v);
  }
}

template <typename T>
__global__ void maxpool_kernel(const T* __restrict__ in, T* __restrict__ out, int B, int H, int W, int C, int Ho, int Wo,
                               int ldo) {
  constexpr int CE = Chunk<T>::CE;
  const int cch = C / CE;
  const size_t n = (size_t)B * Ho * Wo * cch;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cch);
    size_t r = i / cch;
    const int ow = (int)(r % Wo); r /= Wo;
    const int oh = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float mx[CE];
#pragma unroll
    for (int e = 0; e < CE; ++e) mx[e] = -INFINITY;
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = ow * 2 - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float f[CE];
        unpack16<T>(ld16(in + (((size_t)b * H + ih) * W + iw) * C + c * CE), f);
#pragma unroll
        for (int e = 0; e < CE; ++e) mx[e] = fmaxf(mx[e], f[e]);
      }
    }
    st16(out + (((size_t)b * Ho + oh) * Wo + ow) * ldo + c * CE, pack16<T>(mx));
  }
}

template <typename T>
__global__ void upsample_kernel(const T* __restrict__ in, T* __restrict__ out, int B, int H, int W, int C) {
  constexpr int CE = Chunk<T>::CE;
  const int Ho = 2 * H, Wo = 2 * W, cch = C / CE;
  const float sy = Ho > 1 ? (float)(H - 1) / (float)(Ho - 1) : 0.f;
  const float sx = Wo > 1 ? (float)(W - 1) / (float)(Wo - 1) : 0.f;
  const size_t n = (size_t)B * Ho * Wo * cch;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % cch);
    size_t r = i / cch;
    const int ox = (int)(r % Wo); r /= Wo;
    const int oy = (int)(r % Ho);
    const int b = (int)(r / Ho);
    // PyTorch upsample_bilinear2d, align_corners=True: src = dst * (in-1)/(out-1)
    const float fy = oy * sy, fx = ox * sx;
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = y0 + (y0 < H - 1), x1 = x0 + (x0 < W - 1);
    const float ly = fy - y0, lx = fx - x0;
    const float hy = 1.f - ly, hx = 1.f - lx;
    const T* base = in + (size_t)b * H * W * C + c * CE;
    float a[CE], bb[CE], cc[CE], d[CE], v[CE];
    unpack16<T>(ld16(base + ((size_t)y0 * W + x0) * C), a);
    unpack16<T>(ld16(base + ((size_t)y0 * W + x1) * C), bb);
    unpack16<T>(ld16(base + ((size_t)y1 * W + x0) * C), cc);
    unpack16<T>(ld16(base + ((size_t)y1 * W + x1) * C), d);
#pragma unroll
    for (int e = 0; e < CE; ++e) v[e] = hy * (hx * a[e] + lx * bb[e]) + ly * (hx * cc[e] + lx * d[e]);
    st16(out + (((size_t)b * Ho + oy) * Wo + ox) * C + c * CE, pack16<T>(v));
  }
}

// 3x3 / pad 1 conv over the align_corners bilinear x2 upsample of x, by linearity evaluated at
// the low resolution: Z[p][t*C + c] = (W_t . x[p])[c] for each tap t = (dy+1)*3 + (dx+1) (one
// GEMM with N = 9C), then
//   out[Y][X][c] = sum_t [U = Y+dy, V = X+dx inside the 2h x 2w grid] bilerp(Z[.][t*C + c], U, V)
// with bilerp the upsample kernel's weights above.  (REV/models/backbone.py:141
// s16_latern(up16sto8s(xs16)): 4x fewer MFMA flops and no 2h x 2w x Cin intermediate.)
// A thread owns four channels of one output row Y and walks a segment of UC_SEG output
// columns.  Per tap (dy, dx) it keeps the two corner columns x0, x1 in registers, already
// interpolated along y (fp32, hy * Z[y0] + ly * Z[y1]); stepping X -> X+1 moves every tap's source
// column V = X+dx-1 by one output pixel, i.e. by sx < 1/2 low-resolution columns, so x0 advances
// by 0 or 1 -- uniformly over the workgroup (it depends on V only): an advance shifts x1 into x0
// and brings in the new x1, whose loads are issued before the current column is computed.  About
// 9 instead of 36 reads per output (each Z element was fetched 16 times through L2).
#ifndef SPE_UC_SEG
#define SPE_UC_SEG 8
#endif
constexpr int UC_SEG = SPE_UC_SEG;
template <typename T> struct Q4;                 // four channels of T in registers
template <> struct Q4<bf16> {
  typedef u32x2 V;
  static SPE_DEV V ld(const bf16* p) { return ld8(p); }
  static SPE_DEV void unpack(V v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  }
  static SPE_DEV void st(bf16* p, const float* f) { st8(p, u32x2{pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3])}); }
};
template <> struct Q4<float> {
  typedef u32x4 V;
  static SPE_DEV V ld(const float* p) { return ld16(p); }
  static SPE_DEV void unpack(V v, float* f) { unpack16<float>(v, f); }
  static SPE_DEV void st(float* p, const float* f) { st16(p, pack16<float>(f)); }
};
template <typename T>
__global__ __launch_bounds__(256) void upconv_combine_kernel(const T* __restrict__ z, T* __restrict__ out, int ldo, int B, int H,
                                                             int W, int C) {
  typedef Q4<T> Q;
  typedef typename Q::V V;
  const int Ho = 2 * H, Wo = 2 * W, cch = C / 4;
  const int ldz = 9 * C;
  const float sy = (float)(H - 1) / (float)(Ho - 1);
  const float sx = (float)(W - 1) / (float)(Wo - 1);
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= B * Ho * cch) return;
  const int c = j % cch, r = j / cch, Y = r % Ho, b = r / Ho;
  const int X0 = blockIdx.y * UC_SEG, X1 = min(X0 + UC_SEG, Wo);
  const T* zb = z + (size_t)b * H * W * ldz + c * 4;
  // per dy: the two source rows (a row outside the 2H grid gets zero weights)
  int zr[3][2];                                   // element offsets from zb (32-bit: one image's Z)
  float wy[3][2];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int U = Y + dy - 1;
    const bool in = U >= 0 && U < Ho;
    const float fy = (in ? U : 0) * sy;
    const int y0 = (int)fy, y1 = y0 + (y0 < H - 1);
    const float ly = fy - y0;
    wy[dy][0] = in ? 1.f - ly : 0.f;
    wy[dy][1] = in ? ly : 0.f;
    zr[dy][0] = y0 * W * ldz + dy * 3 * C;
    zr[dy][1] = y1 * W * ldz + dy * 3 * C;
  }
  auto col0 = [&](int V) { return min((int)((V < 0 ? 0 : V) * sx), W - 1); };
  auto ymix = [&](int dy, V top, V bot, f32x4& o) {
    float t[4], u[4];
    Q::unpack(top, t);
    Q::unpack(bot, u);
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = wy[dy][0] * t[e] + wy[dy][1] * u[e];
  };
  f32x4 c0[3][3], c1[3][3];                       // [dy][dx]: y-interpolated corners x0, x1
  int xs[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int x0 = col0(X0 + dx - 1), x1 = x0 + (x0 < W - 1);
    xs[dx] = x0;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
      const T* p = zb + zr[dy][0] + dx * C;
      const T* q = zb + zr[dy][1] + dx * C;
      ymix(dy, Q::ld(p + x0 * ldz), Q::ld(q + x0 * ldz), c0[dy][dx]);
      ymix(dy, Q::ld(p + x1 * ldz), Q::ld(q + x1 * ldz), c1[dy][dx]);
    }
  }
  for (int X = X0; X < X1; ++X) {
    // next column's new corners in flight while this one is combined
    const bool more = X + 1 < X1;
    bool adv[3];
    V nt[3][3][2];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int x0 = col0(X + dx);
      adv[dx] = more && x0 != xs[dx];               // uniform
      if (adv[dx]) {
        xs[dx] = x0;
        const int x1 = x0 + (x0 < W - 1);
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int h = 0; h < 2; ++h) nt[dy][dx][h] = Q::ld(zb + (zr[dy][h] + dx * C + x1 * ldz));
      }
    }
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int V = X + dx - 1;
      if (V < 0 || V >= Wo) continue;
      const float fx = V * sx;
      const float lx = fx - min((int)fx, W - 1), hx = 1.f - lx;
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += hx * c0[dy][dx][e] + lx * c1[dy][dx][e];
    }
    Q::st(out + (((size_t)b * Ho + Y) * Wo + X) * ldo + c * 4, acc);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
      if (adv[dx]) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          c0[dy][dx] = c1[dy][dx];
          ymix(dy, nt[dy][dx][0], nt[dy][dx][1], c1[dy][dx]);
        }
      }
  }
}

// D = 256: each lane owns 4 consecutive features.
template <typename T>
__global__ void layernorm_kernel(const T* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
                                 T* __restrict__ out, float* __restrict__ out_f32, int M, int D) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  float v[4];
  if constexpr (sizeof(T) == 2) {
    u32x2 u = ld8(xr + 4 * lane);
    v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    unpack16<float>(ld16(xr + 4 * lane), v);
  }
  const float mean = wave_sum(v[0] + v[1] + v[2] + v[3]) * (1.f / D);
  float d0 = v[0] - mean, d1 = v[1] - mean, d2 = v[2] - mean, d3 = v[3] - mean;
  const float var = wave_sum(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3) * (1.f / D);
  const float rs = rsqrtf(var + 1e-5f);
  const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + 4 * lane);
  const f32x4 be = *reinterpret_cast<const f32x4*>(beta + 4 * lane);
  float y[4] = {d0 * rs * g[0] + be[0], d1 * rs * g[1] + be[1], d2 * rs * g[2] + be[2], d3 * rs * g[3] + be[3]};
  if (out) {
    T* o = out + (size_t)row * D + 4 * lane;
    if constexpr (sizeof(T) == 2) st8(o, u32x2{pack_bf16x2(y[0], y[1]), pack_bf16x2(y[2], y[3])});
    else st16(o, pack16<float>(y));
  }
  if (out_f32) st16(out_f32 + (size_t)row * D + 4 * lane, pack16<float>(y));
}

inline int grid_for(size_t n, int block) {
  size_t g = (n + block - 1) / block;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

int spe_launch_pack_input(const ImageSrc& img, void* out, int B, int S, int dtype, hipStream_t s, float* amax, int cpad) {
  const size_t n = (size_t)B * S * S;
  if (!img.f32 && !(img.u8 && (img.ch == 1 || img.ch == 3))) return -5;
  const SrcF32 sf{img.f32, S};
  const SrcU8 su{img.u8, S, img.ch};
  if (dtype == SPE_DTYPE_BF16) {
    if (img.f32) hipLaunchKernelGGL((pack_input_kernel<bf16, 8, SrcF32>), grid_for(n, 256), 256, 0, s, sf, (bf16*)out, B, S, (float*)nullptr);
    else hipLaunchKernelGGL((pack_input_kernel<bf16, 8, SrcU8>), grid_for(n, 256), 256, 0, s, su, (bf16*)out, B, S, (float*)nullptr);
  } else {   // (fp32: at most 4096 workgroups, each publishing its max |x| once)
    const int grid = std::min(grid_for(n, 256), 4096);
    if (img.f32) {
      if (cpad == 4) hipLaunchKernelGGL((pack_input_kernel<float, 4, SrcF32>), grid, 256, 0, s, sf, (float*)out, B, S, amax);
      else hipLaunchKernelGGL((pack_input_kernel<float, 8, SrcF32>), grid, 256, 0, s, sf, (float*)out, B, S, amax);
    } else {
      if (cpad == 4) hipLaunchKernelGGL((pack_input_kernel<float, 4, SrcU8>), grid, 256, 0, s, su, (float*)out, B, S, amax);
      else hipLaunchKernelGGL((pack_input_kernel<float, 8, SrcU8>), grid, 256, 0, s, su, (float*)out, B, S, amax);
    }
  }
  return (int)hipGetLastError();
}

int spe_launch_pack_input_pad4(const ImageSrc& img, void* out, int B, int S, hipStream_t s) {
  const size_t n = (size_t)B * (S + 6) * (S + 6);
  if (img.f32) hipLaunchKernelGGL(pack_input_pad4_kernel<SrcF32>, grid_for(n, 256), 256, 0, s, SrcF32{img.f32, S}, (bf16*)out, B, S);
  else if (img.u8 && (img.ch == 1 || img.ch == 3))
    hipLaunchKernelGGL(pack_input_pad4_kernel<SrcU8>, grid_for(n, 256), 256, 0, s, SrcU8{img.u8, S, img.ch}, (bf16*)out, B, S);
  else return -5;
  return (int)hipGetLastError();
}

int spe_launch_maxpool3s2(const void* in, void* out, int B, int H, int W, int C, int Ho, int Wo, int dtype, hipStream_t s,
                          int ldo) {
  const int ce = dtype == SPE_DTYPE_BF16 ? 8 : 4;
  if (ldo <= 0) ldo = C;
  if (C % ce || ldo % ce || ldo < C) return -5;
  const size_t n = (size_t)B * Ho * Wo * (C / ce);
  if (dtype == SPE_DTYPE_BF16)
    hipLaunchKernelGGL(maxpool_kernel<bf16>, grid_for(n, 256), 256, 0, s, (const bf16*)in, (bf16*)out, B, H, W, C, Ho, Wo, ldo);
  else
    hipLaunchKernelGGL(maxpool_kernel<float>, grid_for(n, 256), 256, 0, s, (const float*)in, (float*)out, B, H, W, C, Ho, Wo, ldo);
  return (int)hipGetLastError();
}

int spe_launch_upsample2x(const void* in, void* out, int B, int H, int W, int C, int dtype, hipStream_t s) {
  const int ce = dtype == SPE_DTYPE_BF16 ? 8 : 4;
  if (C % ce) return -5;
  const size_t n = (size_t)B * 4 * H * W * (C / ce);
  if (dtype == SPE_DTYPE_BF16)
    hipLaunchKernelGGL(upsample_kernel<bf16>, grid_for(n, 256), 256, 0, s, (const bf16*)in, (bf16*)out, B, H, W, C);
  else
    hipLaunchKernelGGL(upsample_kernel<float>, grid_for(n, 256), 256, 0, s, (const float*)in, (float*)out, B, H, W, C);
  return (int)hipGetLastError();
}

int spe_launch_upconv_combine(const void* z, void* out, int ldo, int B, int H, int W, int C, int dtype, hipStream_t s) {
  if (C % 4 || ldo % 4 || ldo < C) return -5;
  if (H < 1 || W < 1 || (size_t)B * 2 * H * (C / 4) >= (1u << 31) || (size_t)H * W * 9 * C >= (1u << 31)) return -5;
  const int rows = B * 2 * H * (C / 4);
  dim3 grid((rows + 255) / 256, (2 * W + UC_SEG - 1) / UC_SEG);
  if (dtype == SPE_DTYPE_BF16)
    hipLaunchKernelGGL(upconv_combine_kernel<bf16>, grid, 256, 0, s, (const bf16*)z, (bf16*)out, ldo, B, H, W, C);
  else
    hipLaunchKernelGGL(upconv_combine_kernel<float>, grid, 256, 0, s, (const float*)z, (float*)out, ldo, B, H, W, C);
  return (int)hipGetLastError();
}

int spe_launch_layernorm(const void* x, const float* gamma, const float* beta, void* out, float* out_f32, int M, int D,
                         int dtype, hipStream_t s) {
  if (D != 256) return -6;
  const int rows_per_block = 4;
  dim3 grid((M + rows_per_block - 1) / rows_per_block), block(64 * rows_per_block);
  if (dtype == SPE_DTYPE_BF16)
    hipLaunchKernelGGL(layernorm_kernel<bf16>, grid, block, 0, s, (const bf16*)x, gamma, beta, (bf16*)out, out_f32, M, D);
  else
    hipLaunchKernelGGL(layernorm_kernel<float>, grid, block, 0, s, (const float*)x, gamma, beta, (float*)out, out_f32, M, D);
  return (int)hipGetLastError();
}
