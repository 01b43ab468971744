/* spe.h — C ABI of the MI355X-native keypoint-set pose path (libspe.so).
 *
 * The reference (wwhitecyan/satellite-pose-estimation, REV/ = "Revisiting Monocular Satellite
 * Pose Estimation With Transformer") has no FFI layer: its seams are Python call signatures.
 * Each entry point below replaces one of them; the Python host package (spe/) binds them with
 * ctypes and keeps the reference's call surface.
 *
 * Conventions: plain pointers and sizes only; device pointers are caller-owned HIP device memory;
 * `stream` is a hipStream_t (NULL = default stream); no entry point allocates or synchronises
 * on the hot path (spe_forward / spe_pnp_batch / spe_speed_score are graph-capturable);
 * return 0 on success, a negative SPE_E_* code on argument errors, or a positive hipError_t.
 */
#ifndef SPE_H_
#define SPE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPE_ABI_VERSION 9

enum {
  SPE_E_ARG = -1,        /* bad argument / size */
  SPE_E_STATE = -2,      /* model not finalized / already finalized */
  SPE_E_MISSING = -3,    /* a required parameter key was never set */
  SPE_E_KEY = -4,        /* unknown parameter key or wrong element count */
  SPE_E_WORKSPACE = -5,  /* workspace too small */
  SPE_E_LAUNCH = -6      /* kernel launch rejected its shapes */
};

/* BF16_: bf16 storage, bf16 MFMA with fp32 accumulation (throughput mode); F32_: fp32 storage,
 * exact-f32 MFMA (parity mode); F16_: fp16 attention operands (attn_dtype only); F32X3_: fp32
 * storage, split-bf16 MFMA (x = hi + lo, products hi.hi + hi.lo + lo.hi, fp32 accumulation):
 * the fast parity mode on the reference goldens; F32X6_: the accuracy-contract mode (<= 1e-4 of the exact-f32
 * mode on the bench's amplifying weights too): fp32 storage, every GEMM / convolution with
 * near-fp32 precision (x = hi + mid + lo in bf16, the six products of relative order >= 2^-16), the
 * encoder attention contractions as F32X3_, the decoder attention (whose 64x-sharpened cross-attention
 * amplifies operand error most) in exact f32; F32H3_ (round 5): F32X6_ with the backbone / encoder GEMMs and
 * convolutions as three fp16 MFMAs on a two-way fp16 split (x.s = hi + lo, fp16 RNE each, s a power of two:
 * per output channel for the weights, per tensor for the activations from the producer's max |x|),
 * products hi.hi + hi.lo + lo.hi -- F32X6_'s accuracy (2^-22-level operands) at half its MFMAs */
enum { SPE_DTYPE_BF16_ = 0, SPE_DTYPE_F32_ = 1, SPE_DTYPE_F16_ = 2, SPE_DTYPE_F32X3_ = 4, SPE_DTYPE_F32X6_ = 5,
       SPE_DTYPE_F32H3_ = 6 };

/* Solver modes.
 *  SPE_PNP_EPNP              cv2.solvePnPGeneric(EPNP) on all selected points
 *                            (UNC/utils/speed_eval_ceres.py:153-169) — BASELINE config 2
 *  SPE_PNP_RANSAC_P3P_LM     cv2.solvePnPRansac(P3P) + solvePnPGeneric(ITERATIVE) on inliers
 *                            (REV/utils/speed_eval.py:209-230) — BASELINE config 3
 *  SPE_PNP_EPNP_RANSAC_SIGMA cv2.solvePnPRansac(EPNP) + sigma-weighted Huber LM
 *                            (UNC/utils/speed_eval.py:332-420) — BASELINE config 4
 *  SPE_PNP_EPNP_LM           EPnP + solvePnPGeneric(ITERATIVE) on all points
 *  SPE_PNP_EPNP_CERES        UNC EPnPCeresSolver (UNC/utils/speed_eval_ceres.py:43-243): EPnP on all points,
 *                            inliers = reprojection error < the image's threshold (get_repro_th, :53-58),
 *                            sigma-weighted Huber(0.001) LM on the inliers (weights normalised over them),
 *                            the EPnP pose kept when the refined error sum over all points is larger
 *                            (:142-146); exactly one inlier raises IndexError there -> status NO_FG;
 *                            no inlier -> status OK with the EPnP pose (the reference's own control flow
 *                            builds an empty Ceres problem, tests/golden/solver_front_ref.npz), PARITY
 *                            UNPINNED in one point: whether OpenCV 4.4's undistortPoints accepts the
 *                            empty point set (a cv2.error there would make SpeedEval log a zero pose)
 * SPE_PNP_EPNP's inlier_mask is epnp_init's set, reprojection error < repro (:163-166). */
enum { SPE_PNP_EPNP = 0, SPE_PNP_RANSAC_P3P_LM = 1, SPE_PNP_EPNP_RANSAC_SIGMA = 2, SPE_PNP_EPNP_LM = 3,
       SPE_PNP_EPNP_CERES = 4 };

/* Per-image solver status (reference exception mapping, REV/datasets/speed.py:355-363).
 *  OK              pose solved
 *  NO_FG           no foreground label -> IndexError in the reference -> zero pose
 *  CV_ERROR        fewer than 4 correspondences -> cv2.error (CV_Assert npoints >= 4) -> zero pose
 *  RANSAC_FALLBACK no consensus: the reference keeps the rvec/tvec of the last RANSAC hypothesis
 *                  (OpenCV's callback shares them) and skips refinement; same here
 *  UNPINNED        behaviour OpenCV leaves uninitialised (e.g. P3P failure on exactly 4 points);
 *                  defined here as a zero pose */
enum { SPE_PNP_OK = 0, SPE_PNP_NO_FG = 1, SPE_PNP_CV_ERROR = 2, SPE_PNP_RANSAC_FALLBACK = 3, SPE_PNP_UNPINNED = 4 };

typedef struct spe_model spe_model;

/* Mirrors the argparse fields build_model(args) reads (REV/main.py:90-187). */
typedef struct {
  int input_size;       /* --input_size (416) */
  int num_queries;      /* --num_queries (11) */
  int enc_layers;       /* --enc_layers (6) */
  int dec_layers;       /* --dec_layers (6) */
  int hidden_dim;       /* --hidden_dim (256; only 256 supported) */
  int nheads;           /* --nheads (8; head_dim must be 32) */
  int dim_feedforward;  /* --dim_feedforward (2048) */
  int sigma_head;       /* 1: UNC-style sigma head (sigma_embed.layers.*) */
  int dtype;            /* SPE_DTYPE_BF16_ (bf16 storage, fp32 accumulate), SPE_DTYPE_F32_, _F32X3_, _F32X6_ or _F32H3_ */
  int attn_dtype;       /* encoder self-attention operands (q, k, V^T): 0 = as dtype; SPE_DTYPE_F16_ =
                         * fp16 (bf16 models only; BASELINE config 5's "fp16 MFMA attention") */
} spe_model_config;

typedef struct {
  float* logits;          /* [B,Q,12] pred_logits (required) */
  float* points;          /* [B,Q,2]  pred_points, sigmoid, crop-normalised (required) */
  const float* clip_bbox; /* [B,4] x1,y1,x2,y2 (nullable) -> fused PostProcess */
  float* probs;           /* [B,Q,12] softmax(pred_logits) (nullable, needs clip_bbox) */
  float* points_px;       /* [B,Q,2]  image-pixel points (nullable, needs clip_bbox) */
  float* log_sigmas;      /* [B,Q,2]  sigma head raw output (nullable) */
  float* sigmas;          /* [B,Q,2]  exp(log_sigmas) (nullable) */
  float* hs;              /* [B,Q,256] last decoder layer after decoder_norm (nullable) */
  float* aux_logits;      /* [dec_layers-1,B,Q,12] aux outputs (nullable; aux_loss=True, */
  float* aux_points;      /* [dec_layers-1,B,Q,2]   REV/models/detr_speed.py:88-99)       */
} spe_forward_outputs;

/* UNC RT-DETR keypoint model with the sigma head: RTDETR(PResNet-vd, HybridEncoder,
 * RTDETRTransformer) (UNC/src/zoo/rtdetr/rtdetr.py:20-38, UNC/nn/backbone/presnet.py:156-265,
 * UNC/src/zoo/rtdetr/hybrid_encoder.py:196-401, UNC/src/zoo/rtdetr/rtdetr_decoder.py:372-710) as
 * the speed configs build it (UNC/configs/rtdetr_speed/rtdetr_r{18,50}vd_6x_speed_kl_*.yml). */
typedef struct {
  int depth;            /* PResNet depth, variant d: 18 (BasicBlock) or 50 (BottleNeck) */
  int input_size;       /* eval_spatial_size (256); multiple of 32 */
  int num_queries;      /* RTDETRTransformer.num_queries (30), <= 64 */
  int dec_layers;       /* num_decoder_layers (3) */
  int enc_ff;           /* HybridEncoder.dim_feedforward (1024, GELU) */
  int dec_ff;           /* RTDETRTransformer.dim_feedforward (1024, ReLU) */
  int csp_hidden;       /* CSPRepLayer hidden channels = 256 * expansion (128 for expansion 0.5) */
  int num_classes;      /* 11 (+1 no-object logit) */
  int dtype;            /* SPE_DTYPE_BF16_ or SPE_DTYPE_F32_ */
} spe_rtdetr_config;

typedef struct {
  float* logits;          /* [B,Q,C+1] pred_logits of the last decoder layer (required) */
  float* points;          /* [B,Q,2]   pred_pts, refined reference points, crop-normalised (required) */
  float* log_sigmas;      /* [B,Q,2]   pred_sigmas (raw sigma head, repeated to 2) (nullable) */
  const float* clip_bbox; /* [B,4] (nullable) -> fused RTDETRPostProcessor: */
  float* probs;           /*   [B,Q,C+1] softmax (rtdetr_postprocessor.py:44-76) */
  float* points_px;       /*   [B,Q,2] image pixels */
  float* sigmas;          /*   [B,Q,2] exp(pred_sigmas) */
  float* aux_logits;      /* [L-1,B,Q,C+1] earlier decoder layers (nullable; aux_outputs) */
  float* aux_points;      /* [L-1,B,Q,2] */
  float* aux_log_sigmas;  /* [L-1,B,Q,2] */
  float* enc_logits;      /* [B,Q,C+1] encoder top-k logits (nullable; last aux_outputs entry) */
  float* enc_points;      /* [B,Q,2]   sigmoid(enc_bbox_head + anchors) of the selected tokens */
  int32_t* topk;          /* [B,Q] selected encoder tokens, descending score (nullable) */
  float* hs;              /* [B,Q,256] last decoder layer output, the heads' input (nullable) */
} spe_rtdetr_outputs;

/* Create an RT-DETR model handle.  The lifecycle entry points of spe_model (set_param with the
 * reference's state_dict keys, num_params / param_name, finalize, workspace_bytes, destroy,
 * profile_*) apply to it unchanged; BatchNorm2d num_batches_tracked buffers are not parameters. */
int spe_rtdetr_create(const spe_rtdetr_config* cfg, spe_model** out);
/* RTDETR.forward in eval (+ RTDETRPostProcessor when clip_bbox is given).  images: device
 * [B,3,S,S] fp32, ImageNet-normalised (UNC/src/data/speed/speed_dataset.py:40-66). */
int spe_rtdetr_forward(spe_model* m, void* stream, const float* images, int batch, void* workspace,
                       int64_t workspace_bytes, const spe_rtdetr_outputs* out);

int spe_abi_version(void);
const char* spe_last_error(void);

/* Model lifecycle.  Replaces build_model(args) (REV/models/__init__.py:5-6) + load_state_dict
 * (REV/main.py:264-274): parameters are handed over by their reference state_dict key
 * (412 keys, e.g. "backbone.0.body.layer1.0.conv1.weight"), fp32, host memory. */
int spe_model_create(const spe_model_config* cfg, spe_model** out);
void spe_model_destroy(spe_model* m);
int spe_model_set_param(spe_model* m, const char* key, const float* host_data, int64_t numel);
int spe_model_num_params(const spe_model* m);                 /* number of required keys */
const char* spe_model_param_name(const spe_model* m, int i);  /* i-th required key */
int spe_model_finalize(spe_model* m);  /* fold FrozenBN, pack NHWC/[N][K] weights, upload (current device) */
int64_t spe_model_workspace_bytes(const spe_model* m, int batch);

/* DETR.forward + PostProcess (REV/models/detr_speed.py:59-92,266-293).
 * images: device [B,3,S,S] fp32, ImageNet-normalised (REV/datasets/speed.py:25-41). */
int spe_forward(spe_model* m, void* stream, const float* images, int batch, void* workspace, int64_t workspace_bytes,
                const spe_forward_outputs* out);
/* The same pass split in two stages that may run on different streams: ENCODE = backbone +
 * neck + input_proj + encoder (images -> memory, kept in `workspace`), DECODE = decoder + heads +
 * PostProcess (memory in `workspace` -> out).  spe_forward == both stages in order.  A caller
 * that overlaps batch i's DECODE with batch i+1's ENCODE gives each in-flight batch its own
 * workspace. */
/* ENCODE itself splits in two: BACKBONE = backbone + neck + input_proj (images -> src in the
 * workspace) and TRANSFORMER = the encoder layers (src -> memory); ENCODE == BACKBONE followed by
 * TRANSFORMER.  A caller may run batch i's TRANSFORMER beside batch i+1's BACKBONE (the HBM-bound
 * convolutions beside the VALU-bound attention), each batch with its own workspace. */
enum { SPE_STAGE_ENCODE = 1, SPE_STAGE_DECODE = 2, SPE_STAGE_BACKBONE = 4, SPE_STAGE_TRANSFORMER = 8 };
int spe_forward_stages(spe_model* m, void* stream, const float* images, int batch, void* workspace,
                       int64_t workspace_bytes, const spe_forward_outputs* out, int stages);
/* The same stages fed with the 8-bit crops the validation transform produces before to_tensor +
 * Normalize (REV/datasets/speed.py:25-41, 209-233): crops = device [B][S][S][channels] u8 (channels 1:
 * grayscale, which Image.convert('RGB') replicates into three channels -- the SPEED frames -- or 3
 * RGB), normalised (u8 / 255 - mean) / std in fp32 inside the stem's input pack: bit-identical to
 * spe_forward_stages on the fp32 batch normalised that way, at a quarter (RGB) or a twelfth (gray) of
 * its bytes -- the form a host-side loader hands over PCIe (REV/engine.py:92 samples.to(device)).
 * (ABI 8 addition) */
int spe_forward_stages_u8(spe_model* m, void* stream, const uint8_t* crops, int channels, int batch, void* workspace,
                          int64_t workspace_bytes, const spe_forward_outputs* out, int stages);

/* Validation input pipeline on the device (SpeedTrain.__getitem__ with train=False,
 * REV/datasets/speed.py:209-233): generate_clip_bbox_val (:246-258), Pillow crop,
 * A.Resize(S, S, cv2.INTER_CUBIC) (make_transforms(train=False), :295-299), F.to_tensor and
 * Normalize (:25-41).  frames: device uint8 [B,H,W] (channels = 1: grayscale, replicated to RGB
 * like Image.convert('RGB')) or [B,H,W,3]; bbox_xxyy: device fp64 [B,4] detector boxes;
 * images: fp32 [B,3,S,S] (spe_forward's input); clip_bbox: fp32 [B,4] (PostProcess's box);
 * status (nullable): [B] 0 ok, 1 empty crop (the reference raises; zeros written). */
int spe_preprocess(void* stream, const uint8_t* frames, int batch, int height, int width, int channels,
                   const double* bbox_xxyy, int size, float* images, float* clip_bbox, int32_t* status);

/* Baseline-JPEG decode of grayscale frames on the device: the decode half of
 * `Image.open(img_path).convert('RGB')` in SpeedTrain.__getitem__ (REV/datasets/speed.py:209-210;
 * Pillow / libjpeg-turbo, islow IDCT), which the reference runs in DataLoader worker processes
 * (REV/main.py:252-254).  data: device bytes holding the batch's JPEG files; offsets / sizes:
 * device int64 [B] (file b = data[offsets[b] .. offsets[b] + sizes[b])); every file must be a
 * height x width 8-bit single-component sequential Huffman JPEG (SOF0/SOF1, restart intervals
 * allowed) of at most max_bytes_per_image bytes.  frames: device uint8 [B,height,width], the
 * 1-channel input spe_preprocess takes.  status (nullable): [B] 0 ok, 1 unsupported coding
 * (progressive, arithmetic, 12-bit, colour), 2 corrupt stream, 3 frame size != height x width,
 * 4 stream exceeds the workspace plan; a non-zero image gets a zero frame.  workspace: device
 * bytes, spe_jpeg_workspace_bytes(batch, height, width, max_bytes_per_image) of them. */
int64_t spe_jpeg_workspace_bytes(int batch, int height, int width, int64_t max_bytes_per_image);
int spe_jpeg_decode(void* stream, const uint8_t* data, const int64_t* offsets, const int64_t* sizes, int batch,
                    int height, int width, int64_t max_bytes_per_image, uint8_t* frames, int32_t* status,
                    void* workspace, int64_t workspace_bytes);

/* SetCriterion.forward with its HungarianMatcher (REV/models/detr_speed.py:214-261,
 * REV/models/matcher.py:60-88) for `layers` decoder layers (aux first, last layer last), the
 * logging half of evaluate() (REV/engine.py:99-112).  Device pointers: logits [L,B,Q,C] (C = 12),
 * points [L,B,Q,2], tgt_labels int32 [B,T], tgt_points [B,T,2] (crop-normalised), match int32
 * [L,B,T] (query matched to each target), losses fp64 [L,4] = loss_ce, class_error,
 * cardinality_error, loss_points.  num_points: targets per rank averaged over ranks, >= 1
 * (REV/models/detr_speed.py:235-244).  Q <= 64, T <= min(Q, 32). */
int spe_criterion(void* stream, const float* logits, const float* points, const int32_t* tgt_labels,
                  const float* tgt_points, int layers, int batch, int num_queries, int num_classes, int num_targets,
                  float cost_class, float cost_pts, float eos_coef, double num_points, int32_t* match, double* losses);

/* Multi-checkpoint ensemble front end (Multi_Mean_PoseSolver, REV/utils/speed_eval.py:42-100;
 * REV/gen_submission_multi.py:145-186): fuses M models' PostProcess outputs per image -- labels
 * in first-seen order, per label the mean of its points after the 3-sigma filter -- into
 * fused_points [B,C-1,2] + one-hot fused_probs [B,C-1,C], the input spe_pnp_batch then solves
 * (RANSAC_P3P_LM, like the reference).  points [M,B,Q,2] px, probs [M,B,Q,C]; M * Q <= 256. */
int spe_ensemble_fuse(void* stream, const float* points_px, const float* probs, int models, int batch,
                      int num_queries, int num_classes, float* fused_points, float* fused_probs);

/* PostProcess alone (REV/models/detr_speed.py:266-293). */
int spe_postprocess(void* stream, const float* logits, const float* points, const float* clip_bbox, int batch,
                    int num_queries, float* probs, float* points_px);

/* Batched solver (SimplePoseSolver.__call__ per image, REV/utils/speed_eval.py:164-242;
 * SimplePoseSolverSigma, UNC/utils/speed_eval.py:332-420).  All pointers are device memory.
 * K: 3x3 row-major fp64; world: [C-1][3] fp64 landmarks (REV/all_result.json).
 * quat: [B,4] (float32 values, Blender order w,x,y,z); tvec/rvec: [B,3] fp64;
 * corr_label: [B,16] label of each correspondence in first-seen order (-1 padded);
 * inlier_mask: [B] bit i = correspondence i is an inlier.  repro_per_image: [B] fp32 thresholds that
 * replace `repro` image by image (EPnPCeresSolver.get_repro_th of each image's box area).  Nullable:
 * sigmas, rvec, status, n_corr, corr_label, inlier_mask, repro_per_image. */
int spe_pnp_batch(void* stream, const float* points_px, const float* probs, const float* sigmas, int batch,
                  int num_queries, int num_classes, const double* K, const double* world, int mode, float repro,
                  int ransac_iters, double confidence, float* quat, double* tvec, double* rvec, int32_t* status,
                  int32_t* n_corr, int32_t* corr_label, uint32_t* inlier_mask, const float* repro_per_image);

/* Self-assessment filter over the sigma solver's output (BASELINE config 4).  No reference code
 * exists: the UNC README (ROOT/README.md:15-20) names the mechanism and the commented gate
 * `s_ > 0.5 and sig.mean() < 5` (UNC/utils/speed_eval_ceres.py:110-114) is its only trace, so
 * the rule is defined here (parity unpinned): over the RANSAC inliers of each image,
 * mean_sigma = mean sigma (both axes); n_confident = #inliers with score > score_th and mean
 * sigma < sigma_th; reliable = pose solved (status 0 or 3) and n_confident >= min_inliers and
 * mean_sigma < sigma_th.  Inputs are spe_forward's probs/sigmas and spe_pnp_batch's status /
 * corr_label / inlier_mask; all device pointers. */
int spe_self_assess(void* stream, const float* probs, const float* sigmas, const int32_t* status,
                    const int32_t* corr_label, const uint32_t* inlier_mask, int batch, int num_queries,
                    int num_classes, float score_th, float sigma_th, int min_inliers, float* mean_sigma,
                    int32_t* n_confident, uint8_t* reliable);

/* speed_score per image (REV/utils/speed_eval.py:245-262), device pointers. */
int spe_speed_score(void* stream, const float* quat, const double* tvec, const double* q_gt, const double* t_gt,
                    int batch, double* s_t, double* s_q);

/* Per-launch profiling of spe_forward with HIP events on the launch stream (no reference
 * counterpart; used by bench.py for the roofline).  begin: every later launch whose kind starts
 * with `kind_prefix` ("" = all; kinds: conv.*, gemm.*, attn.enc, attn.dec_*, ln.*, eltwise.*,
 * heads) is bracketed by events.  end: stops recording, waits for the events, returns the
 * record count.  get: record i -> kind, elapsed ms, algorithmic flops and bytes. */
int spe_model_profile_begin(spe_model* m, const char* kind_prefix);
int spe_model_profile_end(spe_model* m);
int spe_model_profile_get(const spe_model* m, int i, char* kind, int kind_len, double* ms, double* flops,
                          double* bytes);

/* Kernel test hooks: launch one kernel family on caller buffers (tests/test_gpu_kernels.py).
 * gemm: C[M,N] = act(A . W^T + bias + R) with act = act_code & 255 (0 none, 1 ReLU, 2 SiLU, 3
 * exact GELU); bit 8 of act_code adds R after the activation instead; mode 0 linear (A[m*lda+k]), 1 linear + P[(m%prow)
 * *ldp+k] added to A, 2 implicit-GEMM conv over NHWC A [*,H,W,Cin]; W is [N][ldb] (ldb % 64 == 0);
 * vt_T > 0 stores head-transposed C[((n/256)*vt_B + m/vt_T)*256 + n%256][m%vt_T]; r_period > 0
 * reads the residual row-periodically, R[(m % r_period)*ldr + n].  bf16 problems that fill the chip
 * with 256-row tiles run the direct-to-LDS kernel (gemm2.hip), the rest the 128x128 kernel.
 * attention: per (b,h) softmax(scale Q K^T) V with Q/K rows b*T+i at column h*32, V^T [B][H][32][Tk].
 * Bit 9 of the gemm act_code and bit 8 of the attention dtype select the swizzled V^T layout the
 * encoder uses with 16-bit operands (token t of every 16-token group stored at position t with
 * bits 2 and 3 swapped; Tk % 16 == 0): the v projection writes it, the LDS-DMA attention reads it. */
int spe_debug_gemm(void* stream, int dtype, int mode, const void* A, int lda, const void* P, int ldp, int prow, int H,
                   int W, int Cin, int KH, int KW, int stride, int pad, const void* Bw, int ldb, int M, int N, int K,
                   const float* bias, const void* R, int ldr, int act_code, void* C, int ldc, int out_f32, int vt_T,
                   int vt_B, int r_period, const float* ln_g, const float* ln_b, int out_f16);
/* (out_f16: bf16 launches store fp16 instead of bf16.  ln_g/ln_b non-null: post-norm LayerNorm over each output row fused into the epilogue; bf16,
 * N == 256 and enough rows for the large-tile kernel, else SPE_E_LAUNCH) */
/* kernel family that served this thread's last gemm launch: 0 the 128x128 kernel, 1 the large-tile
 * kernels (gemm2.hip), 2 the persistent streaming kernel for short-K problems (gemm_stream.hip),
 * 3 the patch-staged 3x3 conv (pconv.hip), 4 the projection + residual + LayerNorm (lnproj.hip),
 * 5 the fp32x6 three-way split kernel (gemm.hip), 6 its LDS-DMA form (gemm.hip gemm_x6d), 7 the fp32h3
 * scaled fp16 split kernel (gemm.hip gemm_h3d), 8 its persistent row-store form (gemm.hip gemm_h3p) */
int spe_debug_gemm_path(void);
/* fp32h3 (gemm.hip gemm_h3d): C = act((A . W^T) + bias + R) on fp32 A (LINEAR or CONV geometry as
 * spe_debug_gemm) with the weights given as the finalize form -- planes = fp16 [2][plane_rows][ldb]
 * holding hi, lo of W[n] * 2^e_n, sinv[n] = 2^-e_n -- and amax_a = device max |A| (nullable: scale
 * 1).  amax_c (nullable): max |stored C| * (amax_c_mul or 1) atomically maxed into it (float bits).
 * (Round 5 removed its LayerNorm-epilogue form: the model runs the persistent GEMM + the LayerNorm
 * kernel, measured faster.) */
int spe_debug_gemm_h3(void* stream, int mode, const void* A, int lda, int H, int W, int Cin, int KH, int KW, int stride,
                      int pad, int ldb, int M, int N, int K, const float* bias, const void* R, int ldr, int act_code,
                      void* C, int ldc, const void* planes, int plane_rows, const float* sinv, const float* amax_a,
                      float* amax_c, float amax_c_mul);
/* fp32h3 one-pass encoder FFN (ffn_h3.hip): y = LayerNorm(x + ReLU(x W1^T + b1) W2^T + b2) (eps 1e-5)
 * on fp32 x / y [M][256] (y may be x), F hidden units.  w1 = fp16 [2][F][ld1] hi, lo of W1[j] 2^e1_j;
 * meta1 = [F/32][64] floats: 2^-e1 of the chunk's 32 units, then their b1; w2 = fp16 [2][256][ld2]
 * hi, lo of W2[n] 2^e2_n with the columns of each 32-wide chunk permuted by spe_debug_ffn_h3_perm;
 * sinv2 = 2^-e2; amax_x = device bound on |x|; sh = the hidden activation's power-of-two scale. */
int spe_debug_ffn_h3(void* stream, const float* x, int ldx, float* y, int ldy, int M, int F, const void* w1, int ld1,
                     const float* meta1, const void* w2, int ld2, const float* sinv2, const float* b2,
                     const float* gamma, const float* beta, const float* amax_x, float sh);
/* position p (0..31) of a 32-wide hidden chunk in that column order -> the hidden unit it holds */
int spe_debug_ffn_h3_perm(int p);
/* the same launch with the weights also given pre-split (dtype SPE_DTYPE_F32X6_): planes = bf16
 * [3][plane_rows][ldb] holding hi, mid, lo of Bw (what spe_model_finalize writes for fp32x6 models) */
int spe_debug_gemm_planes(void* stream, int dtype, int mode, const void* A, int lda, const void* P, int ldp, int prow,
                          int H, int W, int Cin, int KH, int KW, int stride, int pad, const void* Bw, int ldb, int M,
                          int N, int K, const float* bias, const void* R, int ldr, int act_code, void* C, int ldc,
                          const void* planes, int plane_rows);
/* attention: dtype | 0x100 = V^T in the 16-bit DMA kernel's key order; dtype SPE_DTYPE_F32X3_ | 0x200 =
 * k and vt given as bf16 hi planes ([B*Tk][ldk] and [B][H][32][Tk]), each followed by its lo plane
 * (what the fp32x3 / fp32x6 models' projection epilogues write; Tk % 8 == 0); | 0x200 | 0x100 = those
 * planes with V^T in that key order (Tk % 16 == 0: the LDS-DMA split kernel, attn_split.hip), and
 * | 0x400 on top = the V^T planes as fp16 hi / lo (the fp32h3 model's form, here unscaled) (ABI 8) */
int spe_debug_attention(void* stream, int dtype, const void* q, int ldq, const void* k, int ldk, const void* vt,
                        void* o, int ldo, int B, int H, int Tq, int Tk, float scale);
int spe_debug_layernorm(void* stream, int dtype, const void* x, const float* gamma, const float* beta, void* out,
                        float* out_f32, int M, int D);
/* ffn (bf16 only): y = LayerNorm(x + W2 relu(W1 x + b1) + b2), D == 256, F % 32 == 0; x and y may
 * alias.  W1 [F][ld1], W2 [D][ld2], biases / LayerNorm affine fp32.  partial (nullable, fp32
 * [splits][M][D]) selects the split-over-F form used for few rows (splits divides F/32).  ld2 == 0
 * (ABI 7 addition): W2 is chunk-packed [F/32][D][32], the bf16 model's encoder form. */
int spe_debug_ffn(void* stream, const void* x, int ldx, const void* w1, int ld1, const float* b1, const void* w2,
                  int ld2, const float* b2, const float* gamma, const float* beta, void* y, int ldy, int M, int D,
                  int F, float* partial, int splits);
/* xattn (bf16 only, the decoder cross-attention against the memory): for image b, query q and
 * head h, u[b*Q+q][h*256 .. +256] = softmax_t(q'[b*Q+q][h*256 ..] . k[b*T+t]) . v[b*T+t] with the
 * scores already in the exp2 domain (k = memory + pos, v = memory, rows of 256).  wv non-null
 * ([256][256] bf16, bv fp32): o[b*Q+q][h*32 + j] = wv[h*32 + j] . u_h + bv[h*32 + j] is written
 * instead of u.  splits <= 0 picks the launch's own key split; partial_scratch: fp32,
 * splits * B * 8Q * 258.  (ABI 7: the measured-negative shared-pos variant and its k_shared
 * argument are gone.) */
int spe_debug_xattn(void* stream, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv, void* u,
                    int ldu, const void* wv, const float* bv, void* o, int ldo, int B, int Q, int T, int splits,
                    float* partial_scratch);
/* xattn_h3 (fp32h3, xattn_h3.hip, ABI 9 addition): the same cross-attention at fp32-level products --
 * q' fp32 [B*Q][ldq] (exp2 domain), mem fp32 [B*T][256], pos fp32 [T][256], keys mem + pos, values mem,
 * *mem_amax (device) >= max |mem|: mem is first written as fp16 hi / lo planes into plane_scratch
 * (B*T*2048 bytes), then o[b*Q+q][h*32 + j] = wv[h*32 + j] . u_h + bv[h*32 + j] (wv [256][256] fp32) is
 * written in fp32 and max |o| raised into *o_amax (nullable; an unsigned-max slot, zero it first).
 * splits <= 0: the launch's own key split; partial_scratch as spe_debug_xattn's. */
int spe_debug_xattn_h3(void* stream, const float* q, int ldq, const float* mem, const float* pos, const float* mem_amax,
                       const float* wv, const float* bv, float* o, int ldo, float* o_amax, int B, int Q, int T,
                       int splits, float* partial_scratch, void* plane_scratch);
/* upconv (bf16 models' neck, replaces the upsample + conv pair of REV/models/backbone.py:141
 * s16_latern(up16sto8s(xs16))): z [B*H*W][9*C] holds the per-tap products W_t . x at the low
 * resolution (t = kh*3 + kw); out [B][2H][2W] rows of stride ldo receive conv3x3(pad 1) of the
 * align_corners bilinear x2 upsample, i.e. sum over in-grid taps of the bilinear interpolation
 * of z's tap block.  C % 8 == 0 (bf16) / C % 4 == 0 (fp32). */
int spe_debug_upconv(void* stream, int dtype, const void* z, void* out, int ldo, int B, int H, int W, int C);
/* btail (bf16, the layer-1 bottleneck tail fused with the next block's conv1, btail.hip):
 * y [M][256] = relu(a [M][k1] . w3^T + b3 (+ r [M][256])), z [M][n2] = relu(y . w1p^T + b1) where
 * w1p [n2][256] holds conv1's columns in spe_debug_btail_perm order; (k1, n2, r) in
 * {(64, 64, r), (64, 128, r), (128, 64, null)}. */
int spe_debug_btail(void* stream, const void* a, int lda, int k1, const void* r, const void* w3, int ld3,
                    const float* b3, void* y, const void* w1p, int ld1, const float* b1, void* z, int n2, int M);
/* decsa (bf16 only, the decoder self-attention block, decsa.hip): in place over tgt [B*Q][ldt],
 * per image b: tgt = LayerNorm(tgt + MHA(q = k = tgt + query_pos, v = tgt) . wo^T + bo) with
 * 8 heads of 32 (d = 256), q|k = tgt . wqk^T + bqk + qpos ([Q][512] bf16, query_pos . wqk^T),
 * v = tgt . wv^T + bv, LayerNorm gamma g / beta b (eps 1e-5).  Q <= 64; weights bf16 rows. */
int spe_debug_decsa(void* stream, void* tgt, int ldt, int B, int Q, const void* wqk, int ldqk, const float* bqk,
                    const void* wv, int ldv, const float* bv, const void* qpos, const void* wo, int ldo,
                    const float* bo, const float* g, const float* b, float scale);
/* decproj (bf16 only, decsa.hip): in place over tgt [B*Q][ldt], tgt = LayerNorm(tgt + x . wo^T + bo)
 * per row (the decoder cross-attention's out-projection + norm2), x [B*Q][ldx] bf16, d = 256,
 * Q <= 64 (one workgroup per image). */
int spe_debug_decproj(void* stream, void* tgt, int ldt, const void* x, int ldx, int B, int Q, const void* wo, int ldo,
                      const float* bo, const float* g, const float* b);
/* decxproj (bf16 only, decsa.hip, ABI 7 addition): the cross-attention's tail in place over tgt:
 * merges the key-split partials spe_debug_xattn left in partial_scratch (same B, Q, T, splits),
 * o[b*Q+q][h*32 + j] = wv[h*32 + j] . u_h + bv[h*32 + j] rounded to bf16, then
 * tgt = LayerNorm(tgt + o . wo^T + bo) -- xattn's merge kernel and decproj as one launch, Q <= 48. */
int spe_debug_decxproj(void* stream, void* tgt, int ldt, float* partial_scratch, int splits, int T, int B, int Q,
                       const void* wv, int ldwv, const float* bv, const void* wo, int ldo, const float* bo,
                       const float* g, const float* b);
/* The decoder kernels (decsa, decproj, decxproj) read fragment-packed weights: bf16 rows
 * w [N][ld] (K = 256, N % 16 == 0) -> dst [N/16][8][64][8], lane l's A fragment of column tile t,
 * K-step ks at ((t*8 + ks)*64 + l)*8 (ABI 7 addition).  Their hooks take row-major weights with
 * ld > 0 (packed into scratch per call) or packed ones with ld == 0. */
int spe_debug_wfrag_pack(void* stream, const void* w, int ld, int N, void* dst);
/* decffn (bf16, decsa.hip + ffn.hip's reduce, ABI 7 addition): y [M][ldy] = LayerNorm(x + W2
 * relu(W1 x + b1) + b2) for few rows, d = 256, F % 256 == 0, through fp32 partials
 * [F/256][M][256]; x and y may alias.  w1 [F][ld1], w2 [256][ld2] row-major (or packed with ld 0:
 * w1 as spe_debug_wfrag_pack of [F] rows, w2 per 256-wide chunk of columns at chunk * 256 * 256). */
int spe_debug_decffn(void* stream, const void* x, int ldx, int M, int F, const void* w1, int ld1, const float* b1,
                     const void* w2, int ld2, const float* b2, const float* gamma, const float* beta, void* y, int ldy,
                     float* partial);
/* decq (bf16, decsa.hip, ABI 7 addition): y [M][ldy] = x . w^T + bias + r[m % period] over K = 256,
 * N % 256 == 0 (the decoder cross-attention's folded query projection); w [N][ldw] row-major or
 * packed with ldw 0; bias (fp32) and r (bf16 [period][ldr]) nullable. */
int spe_debug_decq(void* stream, const void* x, int ldx, int M, int N, const void* w, int ldw, const float* bias,
                   const void* r, int ldr, int period, void* y, int ldy);
/* the K-column order btail's second product expects: stored column k holds channel perm(k) */
int spe_debug_btail_perm(int k);
/* stempool (bf16, stempool.hip): out [B][Po][Po] rows of stride ldo (Po = S/4 for S % 4 == 0) =
 * maxpool3x3/s2/p1(relu(conv7x7/s2/p3(image) + bias)) from x = the zero-bordered pair-packed
 * input [B][S+6][S+6][4] and w [64][ldw] with k = (kh*8 + kw)*4 + ci (registry.cpp's stem). */
int spe_debug_stempool(void* stream, const void* x, const void* w, int ldw, const float* bias, void* out, int ldo,
                       int B, int S);

#ifdef __cplusplus
}
#endif
#endif
