// kcpp_internal.h -- host-side declarations shared by the runtime translation units.
#pragma once
#include <stdint.h>

extern "C" {
int kcpp_weight_repack(int type, const void *src_ggml, void *dst_kcpp, int64_t K, int64_t N, int to_ggml, void *stream);
int kcpp_weight_synth(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, void *stream);
int kcpp_dequantize(int type, const void *w, float *y, int64_t K, int64_t N, void *stream);
int kcpp_quantize_act(int vtype, const float *x, int64_t ldx, void *out, int64_t K, int64_t M, void *stream);
int64_t kcpp_act_bytes(int wtype, int64_t K, int64_t M);
int kcpp_vec_dot_type(int wtype);
}
#include "../../include/kcpp_mi355x.h"
