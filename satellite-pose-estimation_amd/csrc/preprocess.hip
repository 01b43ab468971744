// On-device validation input pipeline for gfx950: the part of
// SpeedTrain.__getitem__(train=False) between the decoded frame and the model input
// (REV/datasets/speed.py:209-233):
//
//   generate_clip_bbox_val (:246-258)    1.2 x max-side square about the box centre, clipped
//                                        to the frame, fp64
//   img.crop(bbox_clip)                  Pillow: integer box by Python round (half to even)
//   A.Resize(S, S, cv2.INTER_CUBIC)      make_transforms(train=False) (:295-299): OpenCV 4.4's
//                                        generic 8-bit cubic resize -- float coefficients
//                                        (A = -0.75) rounded to short at scale 2048, replicated
//                                        border, int horizontal and vertical sums,
//                                        (v + 2^21) >> 22 saturated to u8
//   F.to_tensor + Normalize (:25-41)     u8 / 255, (x - mean) / std, fp32, CHW
//
// One thread per output pixel: its 4 x 4 source taps are L1/L2-resident neighbours, the
// coefficient arithmetic is a few dozen VALU ops (recomputed per pixel, no scratch), and a
// grayscale frame (SPEED ships 8-bit grayscale; Image.convert('RGB') replicates it) is
// resampled once and normalised into the three channels.  Arithmetic follows the restatement
// in oracle/preprocess_ref.py operation for operation (this file is built with
// -ffp-contract=off; divisions are IEEE), so the u8 crops match it bit for bit.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

struct Box { int x0, y0, w, h; float clip[4]; };

SPE_DEV Box crop_box(const double* bb, int W, int H) {
  const double x1 = bb[0], y1 = bb[1], x2 = bb[2], y2 = bb[3];
  const double scale = fmax(x2 - x1, y2 - y1) * 1.2;
  const double xc = (x1 + x2) / 2, yc = (y1 + y2) / 2, hs = scale / 2;
  double c[4] = {xc - hs, yc - hs, xc + hs, yc + hs};
  c[0] = fmin(fmax(c[0], 0.0), (double)W);
  c[2] = fmin(fmax(c[2], 0.0), (double)W);
  c[1] = fmin(fmax(c[1], 0.0), (double)H);
  c[3] = fmin(fmax(c[3], 0.0), (double)H);
  Box b;
  const int ix0 = (int)rint(c[0]), iy0 = (int)rint(c[1]), ix1 = (int)rint(c[2]), iy1 = (int)rint(c[3]);
  b.x0 = ix0; b.y0 = iy0; b.w = ix1 - ix0; b.h = iy1 - iy0;
  for (int k = 0; k < 4; ++k) b.clip[k] = (float)c[k];
  return b;
}

// interpolateCubic (OpenCV), float, in its operation order; coefficients at scale 2048
SPE_DEV void cubic_taps(int dst_i, int dst, int src, int& first, int coef[4]) {
  const double scale = 1.0 / ((double)dst / (double)src);
  float fx = (float)(((double)dst_i + 0.5) * scale - 0.5);
  const int sx = (int)floorf(fx);
  fx = fx - (float)sx;
  const float A = -0.75f;
  const float t = fx + 1.f;
  const float c0 = ((A * t - 5.f * A) * t + 8.f * A) * t - 4.f * A;
  const float c1 = ((A + 2.f) * fx - (A + 3.f)) * fx * fx + 1.f;
  const float u = 1.f - fx;
  const float c2 = ((A + 2.f) * u - (A + 3.f)) * u * u + 1.f;
  const float c3 = 1.f - c0 - c1 - c2;
  coef[0] = (int)rintf(c0 * 2048.f);
  coef[1] = (int)rintf(c1 * 2048.f);
  coef[2] = (int)rintf(c2 * 2048.f);
  coef[3] = (int)rintf(c3 * 2048.f);
  first = sx - 1;
}

template <int C>
__global__ __launch_bounds__(256) void preprocess_kernel(const uint8_t* __restrict__ frames, int H, int W,
                                                         const double* __restrict__ bbox, int S,
                                                         float* __restrict__ images, float* __restrict__ clip_out,
                                                         int32_t* __restrict__ status) {
  const int b = blockIdx.z, oy = blockIdx.y, ox = blockIdx.x * 256 + threadIdx.x;
  const Box bx = crop_box(bbox + 4 * b, W, H);
  if (oy == 0 && blockIdx.x == 0 && threadIdx.x < 4) {
    clip_out[4 * b + threadIdx.x] = bx.clip[threadIdx.x];
    if (threadIdx.x == 0 && status) status[b] = (bx.w <= 0 || bx.h <= 0) ? 1 : 0;
  }
  if (ox >= S) return;
  const size_t plane = (size_t)S * S;
  float* out = images + (size_t)b * 3 * plane + (size_t)oy * S + ox;
  if (bx.w <= 0 || bx.h <= 0) {                    // empty crop (the reference would raise)
    out[0] = 0.f; out[plane] = 0.f; out[2 * plane] = 0.f;
    return;
  }
  int xs, ys, cx[4], cy[4];
  cubic_taps(ox, S, bx.w, xs, cx);
  cubic_taps(oy, S, bx.h, ys, cy);
  int col[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) col[k] = bx.x0 + min(max(xs + k, 0), bx.w - 1);
  const uint8_t* fr = frames + (size_t)b * H * W * C;
  int v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = bx.y0 + min(max(ys + j, 0), bx.h - 1);
    const uint8_t* rp = fr + (size_t)row * W * C;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int hsum = 0;                                // HResizeCubic: int sum of u8 x short
#pragma unroll
      for (int k = 0; k < 4; ++k) hsum += (int)rp[col[k] * C + c] * cx[k];
      v[c] += hsum * cy[j];                        // VResizeCubic
    }
  }
  const float mean[3] = {0.485f, 0.456f, 0.406f}, stdv[3] = {0.229f, 0.224f, 0.225f};
#pragma unroll
  for (int ch = 0; ch < 3; ++ch) {
    const int c = C == 1 ? 0 : ch;
    const int u8 = min(max((v[c] + (1 << 21)) >> 22, 0), 255);   // FixedPtCast<int, uchar, 22>
    out[ch * plane] = ((float)u8 / 255.f - mean[ch]) / stdv[ch];
  }
}

}  // namespace

int spe_launch_preprocess(const uint8_t* frames, int B, int H, int W, int C, const double* bbox, int S,
                          float* images, float* clip_bbox, int32_t* status, hipStream_t s) {
  if (B <= 0) return 0;
  if (!frames || !bbox || !images || !clip_bbox || H <= 0 || W <= 0 || S <= 0 || (C != 1 && C != 3)) return -5;
  const dim3 grid((S + 255) / 256, S, B);
  if (C == 1)
    hipLaunchKernelGGL(preprocess_kernel<1>, grid, dim3(256), 0, s, frames, H, W, bbox, S, images, clip_bbox, status);
  else
    hipLaunchKernelGGL(preprocess_kernel<3>, grid, dim3(256), 0, s, frames, H, W, bbox, S, images, clip_bbox, status);
  return (int)hipGetLastError();
}
