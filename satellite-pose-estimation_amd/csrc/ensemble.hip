// Multi-checkpoint ensemble front end on the device: Multi_Mean_PoseSolver's
// keypoint fusion (REV/utils/speed_eval.py:42-100) for a whole batch, feeding the same batched
// P3P-RANSAC + LM solve as the single-model path (spe_pnp_batch).
//
// Per image: for every model, label = argmax of its PostProcess probabilities (background
// dropped); points are pooled per label in model-then-query order, labels in first-seen order;
// each label's fused point is the float32 mean of its points, or -- with 3 or more points --
// the float32 mean of those closer than 3 std (population, fp64) of the fp64 distances to that
// mean (mean_and_filter, :54-71).  numpy's reduction orders are followed exactly (row-by-row
// float32 axis-0 sums, pairwise fp64 sums for the 1-D std), so results equal the restatement in
// oracle/ensemble_ref.py bit for bit (this file is built with -ffp-contract=off).  Output rows
// are laid out for spe_pnp_batch's selection: row i = i-th first-seen label with a one-hot
// probability row, the remaining rows background.  One thread per image (M * Q <= a few hundred
// points): the fusion is a tiny prologue to the fp64 solver.
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int KMAX = 16;     // labels (num_classes - 1)

// numpy pairwise summation of n fp64 values produced by f(i) (n < 128)
template <typename F>
SPE_DEV double pairwise_sum(int n, F f) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += f(i);
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = f(j);
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += f(i + j);
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += f(i);
  return res;
}

__global__ __launch_bounds__(64) void ensemble_fuse_kernel(EnsembleArgs a) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= a.B) return;
  const int M = a.M, Q = a.Q, C = a.C, K = C - 1;
  // first-seen label order and each query's label
  int order[KMAX], nl = 0;
  bool seen[KMAX];
  for (int k = 0; k < K; ++k) seen[k] = false;
  auto label_of = [&](int m, int q) {
    const float* p = a.probs + (((size_t)m * a.B + b) * Q + q) * C;
    int am = 0;
    float mx = p[0];
    for (int c = 1; c < C; ++c)
      if (p[c] > mx) { mx = p[c]; am = c; }
    return am;
  };
  for (int m = 0; m < M; ++m)
    for (int q = 0; q < Q; ++q) {
      const int l = label_of(m, q);
      if (l != K && !seen[l]) { seen[l] = true; order[nl++] = l; }
    }
  float* outp = a.fused_points + (size_t)b * K * 2;
  float* outr = a.fused_probs + (size_t)b * K * C;
  for (int i = 0; i < K; ++i)
    for (int c = 0; c < C; ++c) outr[i * C + c] = c == K ? 1.f : 0.f;
  for (int i = 0; i < nl; ++i) {
    const int l = order[i];
    // pass 1: float32 row-by-row mean of the label's points
    float sx = 0.f, sy = 0.f;
    int n = 0;
    for (int m = 0; m < M; ++m)
      for (int q = 0; q < Q; ++q)
        if (label_of(m, q) == l) {
          const float* pt = a.points + (((size_t)m * a.B + b) * Q + q) * 2;
          sx = sx + pt[0];
          sy = sy + pt[1];
          ++n;
        }
    float fx = sx / (float)n, fy = sy / (float)n;
    if (n >= 3) {
      // fp64 distances to the mean, in pooling order (<= M * Q of them)
      double d[256];
      int nd = 0;
      for (int m = 0; m < M; ++m)
        for (int q = 0; q < Q; ++q)
          if (label_of(m, q) == l && nd < 256) {
            const float* pt = a.points + (((size_t)m * a.B + b) * Q + q) * 2;
            const double dx = (double)pt[0] - (double)fx, dy = (double)pt[1] - (double)fy;
            d[nd++] = sqrt(dx * dx + dy * dy);
          }
      const double mu = pairwise_sum(nd, [&](int j) { return d[j]; }) / nd;
      const double sd = sqrt(pairwise_sum(nd, [&](int j) { return (d[j] - mu) * (d[j] - mu); }) / nd);
      float kx = 0.f, ky = 0.f;
      int nk = 0, j = 0;
      for (int m = 0; m < M; ++m)
        for (int q = 0; q < Q; ++q)
          if (label_of(m, q) == l) {
            if (d[j] < sd * 3) {
              const float* pt = a.points + (((size_t)m * a.B + b) * Q + q) * 2;
              kx = kx + pt[0];
              ky = ky + pt[1];
              ++nk;
            }
            ++j;
          }
      // np.mean of an empty selection (every distance >= 3 std, e.g. coinciding points with
      // std 0) is NaN, like the reference: 0 / 0 here
      fx = kx / (float)nk;
      fy = ky / (float)nk;
    }
    outp[2 * i] = fx;
    outp[2 * i + 1] = fy;
    outr[i * C + K] = 0.f;
    outr[i * C + l] = 1.f;
  }
  for (int i = nl; i < K; ++i) { outp[2 * i] = 0.f; outp[2 * i + 1] = 0.f; }
}

}  // namespace

int spe_launch_ensemble_fuse(const EnsembleArgs& a, hipStream_t s) {
  if (a.B <= 0) return 0;
  if (a.M < 1 || a.Q < 1 || a.C < 2 || a.C - 1 > KMAX || (size_t)a.M * a.Q > 256) return -5;
  hipLaunchKernelGGL(ensemble_fuse_kernel, dim3((a.B + 63) / 64), dim3(64), 0, s, a);
  return (int)hipGetLastError();
}
