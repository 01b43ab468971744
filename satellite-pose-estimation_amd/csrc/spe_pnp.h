// Pose-solver launcher interface (internal; public entry points are in include/spe.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/spe.h"

// One EPnP-RANSAC hypothesis (pnp_hyp_kernel -> pnp_kernel)
struct HypRec {
  double rt[6];            // rvec, tvec
  uint32_t mask;           // float32 inlier set over the correspondences
  int good, ok, pad;
};

struct PnpArgs {
  const float* points;     // [B][Q][2] image px (PostProcess output)
  const float* probs;      // [B][Q][C] softmax probabilities
  const float* sigmas;     // [B][Q][2] or null
  int B, Q, C;
  const double* K;         // 3x3 row-major (device)
  const double* world;     // [C-1][3] landmarks (device)
  int mode;                // SPE_PNP_*
  float repro;             // RANSAC / inlier reprojection threshold (px)
  const float* repro_img;  // [B] per-image threshold replacing repro (EPnPCeresSolver's area rule) or null
  int ransac_iters;        // cv2 default 100
  double confidence;       // cv2 default 0.99
  float* quat;             // [B][4] (float32 values, mathutils)
  double* tvec;            // [B][3]
  double* rvec;            // [B][3] or null
  int32_t* status;         // [B] or null
  int32_t* n_corr;         // [B] or null
  int32_t* corr_label;     // [B][16] or null
  uint32_t* inlier_mask;   // [B] or null (bit i = correspondence i)
  HypRec* hyp;             // [B][hyp_stride] scratch for the EPnP-RANSAC hypotheses (sigma mode) or null
  int hyp_stride;
};
int spe_launch_pnp(const PnpArgs& a, hipStream_t s);

struct SelfAssessArgs {
  const float* probs;         // [B][Q][C]
  const float* sigmas;        // [B][Q][2]
  const int32_t* status;      // [B]     (pnp_kernel outputs)
  const int32_t* corr_label;  // [B][16]
  const uint32_t* inlier_mask;// [B]
  int B, Q, C;
  float score_th, sigma_th;
  int min_inliers;
  float* mean_sigma;          // [B]
  int32_t* n_confident;       // [B]
  uint8_t* reliable;          // [B]
};
int spe_launch_self_assess(const SelfAssessArgs& a, hipStream_t s);
int spe_launch_score(const float* quat, const double* tvec, const double* q_gt, const double* t_gt, int B,
                     double* s_t, double* s_q, hipStream_t s);
