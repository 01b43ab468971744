// Weight packing helpers of the native runtime (registry.cpp), shared by the DETR and the UNC
// RT-DETR model builders.  Every helper follows the two-pass finalize: with m->dmem null it only
// advances the device-block size, with it set it packs and uploads.
#pragma once
#include <string>
#include <vector>

#include "model_state.h"

uint16_t f2bf(float f);
int pad64(int k);
void* dalloc(spe_model* m, size_t bytes);
void* upload_rows(spe_model* m, const std::vector<float>& rows, int N, int K, int Kpad);   // fp32 [N][K] -> T [N][Kpad]
float* upload_f32(spe_model* m, const float* p, size_t n);
void* upload_T(spe_model* m, const std::vector<float>& v);
float* upload_key(spe_model* m, const std::string& k);
float* upload_transposed(spe_model* m, const std::string& k, int out, int in);
std::vector<int64_t> param_shape(const spe_model* m, const std::string& key);
void fold_conv(spe_model* m, const std::string& wkey, const std::string& bnkey, const std::string& biaskey,
               std::vector<float>& w, std::vector<float>& bias);
Conv pack_conv(spe_model* m, const std::vector<float>& w, const std::vector<float>& bias, int cout, int cin, int kh,
               int kw, int cin_pad, int stride, int pad);
Conv make_conv(spe_model* m, const std::string& wkey, const std::string& bnkey, const std::string& biaskey, int cin_pad,
               int stride, int pad);
Conv make_linear(spe_model* m, const std::string& wkey, const std::string& bkey, int r0, int n, int K);
