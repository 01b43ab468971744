// Keypoint / class / sigma heads fused with PostProcess, fp32.
//   cls_embed   Linear(256 -> 12)                         REV/models/detr_speed.py:50,83
//   point_embed MLP(256,256,2,3) + sigmoid                REV/models/detr_speed.py:16-29,52,84
//   sigma head  MLP(256,256,1,3) repeated to 2, exp       UNC/src/zoo/rtdetr/rtdetr_decoder.py:295-297,367,
//                                                         UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:53
//   PostProcess softmax(12) + crop->image px rescale      REV/models/detr_speed.py:266-293
// Only the last decoder layer feeds PostProcess; the aux layers only feed the training
// criterion (REV/models/detr_speed.py:89-100) and are not evaluated on the inference path.
// One workgroup (256 threads) per query row; weights are stored transposed [in][out] so the
// per-output-column dot products read coalesced rows.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int NT = 256;

__device__ void dense256(const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ b,
                         float* __restrict__ y, int D, bool relu) {
  for (int j = threadIdx.x; j < D; j += NT) {
    float acc = b[j];
    for (int k = 0; k < D; ++k) acc = fmaf(x[k], wt[(size_t)k * D + j], acc);
    y[j] = relu ? fmaxf(acc, 0.f) : acc;
  }
}

// y[o] = b[o] + sum_k x[k] wt[k*nout + o] for small nout, block reduction
__device__ void dense_small(const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ b,
                            float* __restrict__ y, int D, int nout, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int o = 0; o < nout; ++o) {
    float p = 0.f;
    for (int k = threadIdx.x; k < D; k += NT) p = fmaf(x[k], wt[(size_t)k * nout + o], p);
    p = wave_sum(p);
    if (lane == 0) red[wid * 16 + o] = p;
  }
  __syncthreads();
  if (threadIdx.x < nout) {
    float s = b[threadIdx.x];
    for (int w = 0; w < NT / 64; ++w) s += red[w * 16 + threadIdx.x];
    y[threadIdx.x] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(NT) void heads_kernel(HeadArgs a) {
  __shared__ float x[256], h1[256], h2[256], out[16], red[64];
  const int row = blockIdx.x;
  const int D = a.D;
  for (int k = threadIdx.x; k < D; k += NT) x[k] = a.hs[(size_t)row * D + k];
  __syncthreads();

  // classification logits + softmax
  dense_small(x, a.cls_wt, a.cls_b, out, D, 12, red);
  if (threadIdx.x == 0) {
    float mx = -INFINITY;
    for (int c = 0; c < 12; ++c) mx = fmaxf(mx, out[c]);
    float e[12], s = 0.f;
    for (int c = 0; c < 12; ++c) { e[c] = expf(out[c] - mx); s += e[c]; }
    for (int c = 0; c < 12; ++c) {
      a.logits[(size_t)row * 12 + c] = out[c];
      if (a.probs) a.probs[(size_t)row * 12 + c] = e[c] / s;
    }
  }
  __syncthreads();

  // point head
  dense256(x, a.pt_w0t, a.pt_b0, h1, D, true);
  __syncthreads();
  dense256(h1, a.pt_w1t, a.pt_b1, h2, D, true);
  __syncthreads();
  dense_small(h2, a.pt_w2t, a.pt_b2, out, D, 2, red);
  if (threadIdx.x == 0) {
    const float px = 1.f / (1.f + expf(-out[0]));
    const float py = 1.f / (1.f + expf(-out[1]));
    a.points[(size_t)row * 2 + 0] = px;
    a.points[(size_t)row * 2 + 1] = py;
    if (a.points_px && a.clip_bbox) {
      const float* bb = a.clip_bbox + (size_t)(row / a.Q) * 4;
      const float w = bb[2] - bb[0], hgt = bb[3] - bb[1];
      a.points_px[(size_t)row * 2 + 0] = px * w + bb[0];
      a.points_px[(size_t)row * 2 + 1] = py * hgt + bb[1];
    }
  }
  __syncthreads();

  if (a.sg_w0t) {
    dense256(x, a.sg_w0t, a.sg_b0, h1, D, true);
    __syncthreads();
    dense256(h1, a.sg_w1t, a.sg_b1, h2, D, true);
    __syncthreads();
    dense_small(h2, a.sg_w2t, a.sg_b2, out, D, 1, red);
    if (threadIdx.x == 0) {
      const float ls = out[0];
      if (a.log_sigmas) { a.log_sigmas[(size_t)row * 2] = ls; a.log_sigmas[(size_t)row * 2 + 1] = ls; }
      if (a.sigmas) { const float e = expf(ls); a.sigmas[(size_t)row * 2] = e; a.sigmas[(size_t)row * 2 + 1] = e; }
    }
  }
}

__global__ void postprocess_kernel(const float* __restrict__ logits, const float* __restrict__ points,
                                   const float* __restrict__ clip_bbox, int B, int Q, float* __restrict__ probs,
                                   float* __restrict__ points_px) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= B * Q) return;
  const float* lg = logits + (size_t)row * 12;
  float mx = -INFINITY;
  for (int c = 0; c < 12; ++c) mx = fmaxf(mx, lg[c]);
  float e[12], s = 0.f;
  for (int c = 0; c < 12; ++c) { e[c] = expf(lg[c] - mx); s += e[c]; }
  for (int c = 0; c < 12; ++c) probs[(size_t)row * 12 + c] = e[c] / s;
  const float* bb = clip_bbox + (size_t)(row / Q) * 4;
  points_px[(size_t)row * 2] = points[(size_t)row * 2] * (bb[2] - bb[0]) + bb[0];
  points_px[(size_t)row * 2 + 1] = points[(size_t)row * 2 + 1] * (bb[3] - bb[1]) + bb[1];
}

}  // namespace

int spe_launch_heads(const HeadArgs& a, hipStream_t s) {
  if (a.D != 256) return -6;
  if (a.B * a.Q == 0) return 0;
  hipLaunchKernelGGL(heads_kernel, dim3(a.B * a.Q), dim3(NT), 0, s, a);
  return (int)hipGetLastError();
}

int spe_launch_postprocess(const float* logits, const float* points, const float* clip_bbox, int B, int Q,
                           float* probs, float* points_px, hipStream_t s) {
  const int n = B * Q;
  if (n == 0) return 0;
  hipLaunchKernelGGL(postprocess_kernel, dim3((n + 127) / 128), dim3(128), 0, s, logits, points, clip_bbox, B, Q, probs,
                     points_px);
  return (int)hipGetLastError();
}
