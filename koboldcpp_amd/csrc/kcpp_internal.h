// kcpp_internal.h -- host-side declarations shared by the runtime translation units.
#pragma once
#include <stdint.h>

// bytes in front of the flash-attention workspace's partials (spare header words for in-launch hand-offs)
#define KCPP_FA_WS_HEADER 2048
// single-token decode attention: contexts up to this many keys would run the one-launch kernel (attn.hip fa_short_launch;
// off: one workgroup per kv head measured slower than the split pair at every size, 10.3 vs 7.8 us at 300 keys;
// runtime.cpp picks the regime per step, KCPP_FA_SHORT overrides)
#define KCPP_FA_SHORT_MAX 0

extern "C" {
int kcpp_weight_repack(int type, const void *src_ggml, void *dst_kcpp, int64_t K, int64_t N, int to_ggml, void *stream);
int kcpp_weight_synth(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, void *stream);
// columns [c0, c0 + M) (M <= 8) of an activation buffer of Mtot columns through the generic mat-vec (gemv.hip)
int gemv_cols(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, int64_t Mtot,
              int64_t c0, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *stream,
              const int32_t *eid = nullptr, int64_t ebytes = 0, int n_exp = 0, const float *escale = nullptr);
int kcpp_gemv_expert(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, float *Y,
                     const int32_t *eid, int64_t ebytes, int n_exp, const float *escale, int mode, void *stream);
// rows [row0, row0 + N) of the synthetic [K][N_full] tensor (a row-split slice)
int kcpp_weight_synth_rows(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, int64_t row0,
                           void *stream);
int kcpp_dequantize(int type, const void *w, float *y, int64_t K, int64_t N, void *stream);
int kcpp_quantize_act(int vtype, const float *x, int64_t ldx, void *out, int64_t K, int64_t M, void *stream);
int64_t kcpp_act_bytes(int wtype, int64_t K, int64_t M);
int kcpp_vec_dot_type(int wtype);
}
#include "../../include/kcpp_mi355x.h"
#include <hip/hip_runtime.h>

// arguments of the fused decode mat-vec (gemv_dec.hip)
struct DecArgs {
    const uint8_t *W[3];
    float *Y[3];
    int64_t N[3];
    int role[3];          // MODE 2: 0 = q, 1 = k, 2 = v
    int nseg;
    const uint8_t *W2;    // MODE 1: up weight
    int64_t K;
    const uint8_t *act;   // PRO 0
    const float *x;       // PRO 1/2 input row
    const float *nw;      // PRO 1 norm weight
    float eps;
    const float *res;     // MODE 0 residual (indexed like Y[0])
    uint16_t *q16, *kc, *vc;
    int64_t ekv;
    int D;
    const int32_t *pos;
    const float2 *rope_tab;
    // mixture of experts (mul_mat_id at batch 1): W, W2 are expert 0 of [n_expert] equal slices of
    // `ebytes`; the expert index is read on the device (eid[0]); MODE 0 scales the product by escale[0]
    const int32_t *eid;
    int64_t ebytes;
    const float *escale;
    // PRO 0 in the RS kernels: column act_col of an activation buffer holding act_mtot (0 = 1) columns
    int64_t act_mtot, act_col;
    // MoE: the number of expert slices; an expert id read on the device is clamped to [0, n_exp) so that a bad
    // router id cannot address past the tensor (the reference asserts, ggml-cuda.cu mul_mat_id); 0 = unchecked
    int64_t n_exp;
    // MODE 0 in the RS kernels: added to the (scaled) product before the residual -- the MoE slot chain
    // ((w0 o0 + w1 o1) + ...) + x of k_moe_combine, carried through the expert down projections
    const float *pre;
    // MoE, RS kernels: segment 1's expert index (two top-k slots' gate|up in one launch: segments 0 / 1 = slots 0 / 1
    // over the same expert tensors, the same activation); null: every segment takes eid
    const int32_t *eid1;
    // MoE, RS GLU with two slots: route inside the launch (k_moe_route's math on the prologue's normalised row; NE <= 8,
    // top-2, K <= 4096) instead of reading eid / eid1; workgroup 0 stores the ids and weights for the down projections
    const void *route_w;      // ffn_gate_inp [NE][K], F32 or F16
    int route_wt;             // KT_F32 / KT_F16
    int route_ne;
    int32_t *route_ids;
    float *route_wts;
};
// the ggml plugin's fused nodes (ggml_backend.cpp fuse_*): the intermediate nodes' outputs, written beside Y so that
// the graph's every tensor holds what the unfused node sequence leaves.  MODE 0: p0 = the product before the residual
// (the MUL_MAT node under an ADD; null without one), h0 = the product as f16 (a CPY into a contiguous F16 cache view;
// null without one).  MODE 1: p0 = gate, p1 = silu(gate), p2 = up.  A separate kernel parameter of the RS kernels'
// AUX instances (kcpp_gemv_rs_aux), so the runtime's launches and their DecArgs carry none of it.
// RopeP (MODE 0, pairs of rows): the ROPE node (mode NORM, n_dims = D) that follows the product -- out = its f32
// output, rows (2i, 2i+1) of each D-row head rotated by pair (i mod D/2) at position pos[0] (ggml_rope_cs); h0 then
// holds the roped values as f16 (the CPY of the ROPE into the cache)
struct RopeP {
    float *out;
    const int32_t *pos;
    const float *ff;
    int D;
    float theta_scale, freq_scale, ext_factor, attn_factor, mscale_ext, corr0, corr1;
};
// yn / rn (PRO 1 launches; rn may be null): the RMS_NORM and MUL nodes in front of this, stored by workgroup 0 from
// the prologue's normalised row (r = x * scale, y = r * w: the nodes' own bits)
struct AuxOut {
    float *p0, *p1, *p2;
    uint16_t *h0;
    RopeP rope;
    float *rn, *yn;
};


// top-NU of NE <= 8 router logits exactly as ggml's soft_max (ggml_float sum) + argsort (exchange order) + the
// normalisation by the selected weights' sum (llm_build_moe_ffn, src/llama.cpp:9416-9470); shared by k_moe_route
// (moe.hip) and the routed RS GLU launch (gemv_rs.hip) so both choose bit-identical experts and weights
__device__ __forceinline__ void moe_topk8(const float *logit, int NE, int NU, int *idx_out, float *w_out) {
    float p[8], pv[8];
    int idx[8];
    float mx = -INFINITY;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        p[e] = e < NE ? logit[e] : -INFINITY;
        mx = fmaxf(mx, p[e]);
    }
    double sum = 0.0;
#pragma unroll
    for (int e = 0; e < 8; ++e)
        if (e < NE) { p[e] = expf(p[e] - mx); sum += (double)p[e]; }
    const float inv = (float)(1.0 / sum);
#pragma unroll
    for (int e = 0; e < 8; ++e) { p[e] *= inv; pv[e] = p[e]; idx[e] = e; }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (j >= NU) break;
#pragma unroll
        for (int k = j + 1; k < 8; ++k) {
            if (k >= NE) break;
            if (pv[j] < pv[k]) {
                const int ti = idx[j]; idx[j] = idx[k]; idx[k] = ti;
                const float tv = pv[j]; pv[j] = pv[k]; pv[k] = tv;
            }
        }
    }
    double ws = 0.0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < NU) ws += (double)pv[j];
    const float wsum = (float)ws;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (j < NU) { idx_out[j] = idx[j]; w_out[j] = pv[j] / wsum; }
}
// the expert slice offset of a DecArgs (0 without an expert id); `id` defaults to eid
__device__ __forceinline__ int64_t dec_expert_offset(const DecArgs &a, const int32_t *id = nullptr) {
    if (!id) id = a.eid;
    if (!id) return 0;
    int e = __builtin_amdgcn_readfirstlane(id[0]);
    if (a.n_exp > 0) e = e < 0 ? 0 : (e >= (int)a.n_exp ? (int)a.n_exp - 1 : e);
    return (int64_t)e * a.ebytes;
}
extern "C" int kcpp_gemv_dec(int type, const void *args, int mode, int pro, int rows_per_wave, void *stream);
// coalesced Q4_K variant (gemv_stream.hip); -3 = not covered
extern "C" int kcpp_gemv_stream(int type, const void *args, int mode, int pro, void *stream);
// VALU-lean unit-per-lane Q4_K variant (gemv_q4k.hip); -3 = not covered
extern "C" int kcpp_gemv_q4k(const void *args, int mode, int pro, void *stream);


// MFMA prefill flash attention (attn_mfma.hip); -3 = shape not covered (needs D = 128, H = 4 * HKV)
extern "C" int kcpp_flash_attn_prefill_mfma(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out,
                                            int T, int H, int HKV, int D, int n_past, float scale, void *stream);
extern "C" int kcpp_flash_attn_prefill_mfma_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out,
                                               void *qta, void *ws, int T, int H, int HKV, int D, int n_past, float scale,
                                               void *stream);
extern "C" int64_t kcpp_fa_split_ws_bytes(int H);
extern "C" int kcpp_flash_attn_dec_ta(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qta,
                                      void *ws, int H, int HKV, int D, int n_past, const int32_t *n_past_dev,
                                      int n_kv_max, float scale, void *stream);
// decode mat-vec over the row-major RS layouts (gemv_rs.hip); -3 = not covered
extern "C" int kcpp_gemv_rs(int type, const void *args, int mode, int pro, void *stream);
// ROPE's host constants {theta_scale, corr0, corr1, mscale_ext} (ggml_ops.hip; the CPU op's own expressions)
extern "C" void kcpp_ggml_rope_consts(int n_dims, int n_ctx_orig, float freq_base, float freq_scale, float attn_factor,
                                      float beta_fast, float beta_slow, float *out);
// the same single-token launch (mode 0 / 1, quantize prologue) storing the intermediate nodes' tensors too (AuxOut)
extern "C" int kcpp_gemv_rs_aux(int type, const void *args, int mode, const AuxOut *aux, void *stream);
extern "C" int kcpp_rs_supported(int type, int64_t K);



struct kcpp_model;
// single-token stage hand-off by the stages' own kernels (link.hip; the layer-split engine in expose.cpp): this stage's
// wait / pull / report words and the peers it writes (peer memory on another GPU).  in_lag: 1 on stage 0 (its input is
// the previous step's token), else 0; out_lag: 0 on the last stage (stage 0 pulls its token in the same step), else 1.
struct KLink {
    unsigned *stepctr;            // this stage's linked-step counter (local)
    const unsigned *ready_in;     // local: the producer's published step
    const unsigned *copied_out;   // local: the step the consumer has pulled this stage's output for
    unsigned *ready_out;          // the consumer's ready_in
    unsigned *copied_report;      // the producer's copied_out
    const float *src_x;           // stage >= 1: the producer's residual row, n floats
    float *dst_x;
    int n;
    const int32_t *src_tok;       // stage 0: the last stage's greedy token
    int32_t *dst_tok;
    int in_lag, out_lag;
    unsigned *err;                // local: set when a wait gave up (bounded poll); the host checks it after a sync
};
int kcpp_link_wait(const KLink &L, hipStream_t s);
int kcpp_link_publish(const KLink &L, hipStream_t s);
// the stage's single-token graph bracketed by the link kernels (runtime.cpp); -3 when graphs are off (row split)
int kcpp_model_set_link(kcpp_model *m, const KLink *L);
int kcpp_model_step_linked(kcpp_model *m, int n_past);
// one query of FLASH_ATTN_EXT in the ggml graph form on the split decode kernel (attn.hip; the b1 backend's decode)
extern "C" int kcpp_flash_attn_ext_dec(const float *q, int64_t q_nb2, const uint16_t *kc, const uint16_t *vc, int64_t k_ld,
                                       int64_t k_hs, const uint16_t *mask, float *out, void *ws, int H, int HKV, int D,
                                       int n_kv, float scale, void *stream);
