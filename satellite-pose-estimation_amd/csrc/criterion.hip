// Set criterion of evaluate() on the device: HungarianMatcher + SetCriterion
// losses for the last decoder layer and every aux layer (REV/engine.py:99-112,
// REV/models/detr_speed.py:103-261, REV/models/matcher.py:35-88).
//
//   cost[q][t] = cost_pts * (|px - tx| + |py - ty|) - cost_class * softmax(logits_q)[label_t]
//                (fp32, torch's order), assignment minimising the fp64 sum (scipy's
//                linear_sum_assignment: rectangular shortest augmenting path, rows <= columns,
//                the matrix transposed otherwise; restated in oracle/criterion_ref.lsap)
//   loss_ce            weighted cross entropy over all queries (unmatched -> no-object, weight
//                      eos_coef), class_error = 100 - top-1 accuracy of the matched queries,
//   cardinality_error  mean |#queries not predicting no-object - #targets|,
//   loss_points        smooth L1 (beta 1/200) over matched pairs / num_points.
//
// One wave per (layer, image): lanes build the cost matrix and the per-query terms, lane 0 runs
// the O(n^3) assignment in LDS (n <= 64; the criterion only feeds logging), and the per-image
// partial sums are reduced per layer in image order by a second launch (deterministic).
#include "spe_common.h"
#include "spe_kernels.h"

namespace {

constexpr int QMAX = 64, TMAX = 32, CMAX = 32;
constexpr double INF = 1.0e300;

// scipy's augmenting-path LSAP on an [nr][nc] row-major fp64 matrix in LDS (nr <= nc);
// col4row[r] = assigned column.  Sequential (one lane), in oracle/criterion_ref.lsap's order.
SPE_DEV void lsap_lane(const double* c, int nr, int nc, int* col4row, int* row4col, double* u, double* v,
                       double* spc, int* path, bool* sr, bool* sc, int* remaining) {
  for (int i = 0; i < nr; ++i) { u[i] = 0.0; col4row[i] = -1; }
  for (int j = 0; j < nc; ++j) { v[j] = 0.0; row4col[j] = -1; }
  for (int cur = 0; cur < nr; ++cur) {
    for (int j = 0; j < nc; ++j) { spc[j] = INF; path[j] = -1; sc[j] = false; remaining[j] = nc - 1 - j; }
    for (int i = 0; i < nr; ++i) sr[i] = false;
    int nrem = nc, i = cur, sink = -1;
    double min_val = 0.0;
    while (sink == -1) {
      sr[i] = true;
      int index = -1;
      double lowest = INF;
      for (int it = 0; it < nrem; ++it) {
        const int j = remaining[it];
        const double r = min_val + c[i * nc + j] - u[i] - v[j];
        if (r < spc[j]) { path[j] = i; spc[j] = r; }
        if (spc[j] < lowest || (spc[j] == lowest && row4col[j] == -1)) { lowest = spc[j]; index = it; }
      }
      min_val = lowest;
      if (index < 0 || !(min_val < INF)) return;     // infeasible (non-finite costs): leave -1s
      const int j = remaining[index];
      if (row4col[j] == -1) sink = j;
      else i = row4col[j];
      sc[j] = true;
      remaining[index] = remaining[--nrem];
    }
    u[cur] += min_val;
    for (int r = 0; r < nr; ++r)
      if (sr[r] && r != cur) u[r] += min_val - spc[col4row[r]];
    for (int j = 0; j < nc; ++j)
      if (sc[j]) v[j] -= min_val - spc[j];
    int j = sink;
    while (true) {
      const int r = path[j];
      row4col[j] = r;
      const int t = col4row[r];
      col4row[r] = j;
      j = t;
      if (r == cur) break;
    }
  }
}

__global__ __launch_bounds__(64) void criterion_match_kernel(CritArgs a) {
  const int lb = blockIdx.x, l = lb / a.B, b = lb - l * a.B, q = threadIdx.x;
  const int Q = a.Q, T = a.T, C = a.C;
  __shared__ double cost[QMAX * TMAX];
  __shared__ float prob[QMAX][CMAX];
  __shared__ int tclass[QMAX], amax[QMAX];
  __shared__ int col4row[QMAX], row4col[QMAX], path[QMAX], remaining[QMAX];
  __shared__ double u[QMAX], v[QMAX], spc[QMAX];
  __shared__ bool sr[QMAX], sc[QMAX];
  __shared__ int mq[TMAX];
  const float* lg = a.logits + ((size_t)l * a.B + b) * Q * C;
  const float* pt = a.points + ((size_t)l * a.B + b) * Q * 2;
  const int* tl = a.tgt_labels + (size_t)b * T;
  const float* tp = a.tgt_points + (size_t)b * T * 2;
  float lse = 0.f, mx = 0.f;
  if (q < Q) {
    // softmax (fp32: max, exp(x - max), sum, divide) and the log-sum-exp for the cross entropy
    mx = lg[q * C];
    int am = 0;
    for (int k = 1; k < C; ++k)
      if (lg[q * C + k] > mx) { mx = lg[q * C + k]; am = k; }
    float s = 0.f;
    for (int k = 0; k < C; ++k) s += expf(lg[q * C + k] - mx);
    for (int k = 0; k < C; ++k) prob[q][k] = expf(lg[q * C + k] - mx) / s;
    lse = logf(s);
    amax[q] = am;
    tclass[q] = C - 1;                       // no-object unless matched
    const float px = pt[2 * q], py = pt[2 * q + 1];
    // cost in the matcher's orientation [Q][T], or transposed [T][Q] when Q > T (scipy)
    for (int t = 0; t < T; ++t) {
      const float cp = fabsf(px - tp[2 * t]) + fabsf(py - tp[2 * t + 1]);
      const float cc = -prob[q][tl[t]];
      const float cst = a.cost_pts * cp + a.cost_class * cc;
      if (Q > T) cost[t * Q + q] = (double)cst;
      else cost[q * T + t] = (double)cst;
    }
  }
  __syncthreads();
  if (q == 0) {
    const bool tr = Q > T;
    lsap_lane(cost, tr ? T : Q, tr ? Q : T, col4row, row4col, u, v, spc, path, sr, sc, remaining);
    for (int t = 0; t < T; ++t) mq[t] = -1;
    if (tr) {
      for (int t = 0; t < T; ++t) mq[t] = col4row[t];
    } else {
      for (int qq = 0; qq < Q; ++qq)
        if (col4row[qq] >= 0) mq[col4row[qq]] = qq;
    }
    for (int t = 0; t < T; ++t)
      if (mq[t] >= 0) tclass[mq[t]] = tl[t];
  }
  __syncthreads();
  if (q < T) a.match[((size_t)l * a.B + b) * T + q] = mq[q];
  // per-query terms (fp64): weighted NLL, weight
  double w = 0.0, wnll = 0.0, card = 0.0;
  if (q < Q) {
    const int tc = tclass[q];
    w = tc == C - 1 ? (double)a.eos_coef : 1.0;
    wnll = w * -((double)lg[q * C + tc] - (double)mx - (double)lse);
    card = amax[q] != C - 1 ? 1.0 : 0.0;
  }
  // per-target terms: top-1 hit of the matched query, smooth L1 of its point
  double hit = 0.0, sl1 = 0.0;
  if (q < T && mq[q] >= 0) {
    const int qq = mq[q];
    hit = amax[qq] == tl[q] ? 1.0 : 0.0;
    const double beta = 1.0 / 200.0;
    for (int d = 0; d < 2; ++d) {
      const double df = fabs((double)pt[2 * qq + d] - (double)tp[2 * q + d]);
      sl1 += df < beta ? 0.5 * df * df / beta : df - 0.5 * beta;
    }
  }
  // wave reductions in lane order (xor tree: deterministic)
  double vals[5] = {w, wnll, card, hit, sl1};
  for (int k = 0; k < 5; ++k) {
    double x = vals[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    vals[k] = x;
  }
  if (q == 0) {
    double* p = a.partial + ((size_t)l * a.B + b) * 5;
    p[0] = vals[0];
    p[1] = vals[1];
    p[2] = fabs(vals[2] - (double)T);
    p[3] = vals[3];
    p[4] = vals[4];
  }
}

__global__ __launch_bounds__(64) void criterion_reduce_kernel(CritArgs a) {
  const int l = blockIdx.x;
  if (threadIdx.x != 0) return;
  double s[5] = {0, 0, 0, 0, 0};
  for (int b = 0; b < a.B; ++b)
    for (int k = 0; k < 5; ++k) s[k] += a.partial[((size_t)l * a.B + b) * 5 + k];
  double* o = a.losses + (size_t)l * 4;
  o[0] = s[1] / s[0];                                    // loss_ce
  o[1] = 100.0 - 100.0 * s[3] / ((double)a.B * a.T);     // class_error
  o[2] = s[2] / a.B;                                     // cardinality_error
  o[3] = s[4] / a.num_points;                            // loss_points
}

}  // namespace

int spe_launch_criterion(const CritArgs& a, hipStream_t s) {
  if (a.L <= 0 || a.B <= 0) return 0;
  if (a.Q < 1 || a.Q > QMAX || a.T < 1 || a.T > TMAX || a.T > a.Q || a.C < 2 || a.C > CMAX || !a.partial) return -5;
  hipLaunchKernelGGL(criterion_match_kernel, dim3(a.L * a.B), dim3(64), 0, s, a);
  hipLaunchKernelGGL(criterion_reduce_kernel, dim3(a.L), dim3(64), 0, s, a);
  return (int)hipGetLastError();
}
