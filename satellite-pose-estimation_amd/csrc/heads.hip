// Keypoint / class / sigma heads fused with PostProcess, fp32.
//   cls_embed   Linear(256 -> 12)                         REV/models/detr_speed.py:50,83
//   point_embed MLP(256,256,2,3) + sigmoid                REV/models/detr_speed.py:16-29,52,84
//   sigma head  MLP(256,256,1,3) repeated to 2, exp       UNC/src/zoo/rtdetr/rtdetr_decoder.py:295-297,367,
//                                                         UNC/src/zoo/rtdetr/rtdetr_postprocessor.py:53
//   PostProcess softmax(12) + crop->image px rescale      REV/models/detr_speed.py:266-293
// Only the last decoder layer feeds PostProcess; the aux layers only feed the training
// criterion (REV/models/detr_speed.py:89-100) and are not evaluated on the inference path.
// One workgroup (256 threads) per HR = 4 query rows: each weight element read from L2 serves the
// four rows (one workgroup per row moved the 1 MB of MLP weights 704 times per batch of 64 and
// took ~68 us); weights are stored transposed [in][out] so the per-output-column dot products
// read coalesced rows.  Sums keep the one-row kernel's order exactly: the 256-wide layers as a
// k-ordered fmaf chain from the bias, the narrow outputs as bias + the four 64-lane wave sums in
// wave order.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int NT = 256, HR = 4;

// y[j][r] = act(b[j] + sum_k x[k][r] wt[k][j]) for the HR rows, thread j = output column
SPE_DEV void dense_rows(const float (*__restrict__ x)[HR], const float* __restrict__ wt, const float* __restrict__ b,
                        float (*__restrict__ y)[HR], bool relu) {
  const int j = threadIdx.x;
  float acc[HR];
#pragma unroll
  for (int r = 0; r < HR; ++r) acc[r] = b[j];
#pragma unroll 16
  for (int k = 0; k < NT; ++k) {
    const float w = wt[(size_t)k * NT + j];
    const f32x4 xv = *reinterpret_cast<const f32x4*>(x[k]);     // (one address for all lanes)
#pragma unroll
    for (int r = 0; r < HR; ++r) acc[r] = fmaf(xv[r], w, acc[r]);
  }
#pragma unroll
  for (int r = 0; r < HR; ++r) y[j][r] = relu ? fmaxf(acc[r], 0.f) : acc[r];
}

// narrow output for row r = this wave's: out[o] = b[o] + sum_w (wave sum over k in [64w, 64w+64))
SPE_DEV float dense_narrow(const float (*__restrict__ x)[HR], const float* __restrict__ wt, const float* __restrict__ b,
                           int nout, int o) {
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;
  float s = b[o];
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const int k = 64 * w + lane;
    s += wave_sum(fmaf(x[k][r], wt[(size_t)k * nout + o], 0.f));   // (no contraction into the sum)
  }
  return s;
}

__global__ __launch_bounds__(NT) void heads_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float x[NT][HR], h1[NT][HR], h2[NT][HR];
  const int rows = a.B * a.Q, row0 = blockIdx.x * HR;
  const int lane = threadIdx.x & 63, r = threadIdx.x >> 6;     // wave r finishes row row0 + r
  const int row = row0 + r;
#pragma unroll
  for (int i = 0; i < HR; ++i) x[threadIdx.x][i] = row0 + i < rows ? a.hs[(size_t)(row0 + i) * NT + threadIdx.x] : 0.f;
  __syncthreads();

  // classification logits + softmax (row r on wave r)
  {
    float lg[12];
#pragma unroll
    for (int c = 0; c < 12; ++c) lg[c] = dense_narrow(x, a.cls_wt, a.cls_b, 12, c);
    if (lane == 0 && row < rows) {
      float mx = -INFINITY;
      for (int c = 0; c < 12; ++c) mx = fmaxf(mx, lg[c]);
      float e[12], s = 0.f;
      for (int c = 0; c < 12; ++c) { e[c] = expf(lg[c] - mx); s += e[c]; }
      for (int c = 0; c < 12; ++c) {
        a.logits[(size_t)row * 12 + c] = lg[c];
        if (a.probs) a.probs[(size_t)row * 12 + c] = e[c] / s;
      }
    }
  }

  // point head
  dense_rows(x, a.pt_w0t, a.pt_b0, h1, true);
  __syncthreads();
  dense_rows(h1, a.pt_w1t, a.pt_b1, h2, true);
  __syncthreads();
  {
    const float o0 = dense_narrow(h2, a.pt_w2t, a.pt_b2, 2, 0), o1 = dense_narrow(h2, a.pt_w2t, a.pt_b2, 2, 1);
    if (lane == 0 && row < rows) {
      const float px = 1.f / (1.f + expf(-o0));
      const float py = 1.f / (1.f + expf(-o1));
      a.points[(size_t)row * 2 + 0] = px;
      a.points[(size_t)row * 2 + 1] = py;
      if (a.points_px && a.clip_bbox) {
        const float* bb = a.clip_bbox + (size_t)(row / a.Q) * 4;
        const float w = bb[2] - bb[0], hgt = bb[3] - bb[1];
        a.points_px[(size_t)row * 2 + 0] = px * w + bb[0];
        a.points_px[(size_t)row * 2 + 1] = py * hgt + bb[1];
      }
    }
  }

  if (a.sg_w0t) {
    __syncthreads();                              // (h1 / h2 are re-used)
    dense_rows(x, a.sg_w0t, a.sg_b0, h1, true);
    __syncthreads();
    dense_rows(h1, a.sg_w1t, a.sg_b1, h2, true);
    __syncthreads();
    const float ls = dense_narrow(h2, a.sg_w2t, a.sg_b2, 1, 0);
    if (lane == 0 && row < rows) {
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
  hipLaunchKernelGGL(heads_kernel, dim3((a.B * a.Q + HR - 1) / HR), dim3(NT), 0, s, a);
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
