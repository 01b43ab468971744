// Launch helpers of the native runtime (forward.cpp), shared by the DETR and the UNC RT-DETR
// launch sequences: every launch goes through run_gemm / run_attn / run_other, which bracket it
// with HIP events when the per-launch profiler is on (spe_model_profile_*, bench roofline).
#pragma once
#include <functional>

#include "model_state.h"

int run_other(spe_model* m, const char* kind, double flops, double bytes, hipStream_t s, const std::function<int()>& fn);
int run_gemm(spe_model* m, const char* kind, const GemmArgs& g, int mode, hipStream_t s);
int run_attn(spe_model* m, const char* kind, const AttnArgs& a, int dtype, hipStream_t s);
GemmArgs linear_args(const Conv& c, const void* A, int lda, int M, void* C, int ldc);
GemmArgs conv_args(const Conv& c, const void* X, int B, int H, int W, void* Y, int ldc);
int run_ffn(spe_model* m, const char* kind, const Conv& l1, const Conv& l2, const float* g, const float* b, void* x,
            int M, hipStream_t s, const void* pos = nullptr, void* ypos = nullptr, int period = 0,
            float* partial = nullptr, const void* w2_chunked = nullptr);
