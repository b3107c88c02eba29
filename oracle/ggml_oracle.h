/*
 * ggml_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's CPU ggml path for the Llama
 * token-generation hot path.  It is the parity checker
 * for the HIP kernels and the "port" CPU baseline; the product library never
 * links, loads or calls it.  Pinned against the reference itself through
 * tests/golden/ fixtures produced by oracle/_ref (reference ggml compiled from
 * /root/reference sources) -- see tests/test_oracle_golden.py.
 *
 * x86 semantics are restated (the GPU box's host is x86-64 with AVX2):
 *   - quantize_row_q8_0 follows the AVX2 branch (ggml-quants.c:940-1000):
 *     id = 127/amax, round-half-to-even;
 *   - quantize_row_q8_K = quantize_row_q8_K_ref (ggml-quants.c:3786-3823, 3836);
 *   - f32->f16 is round-to-nearest-even (F16C).
 */
#ifndef GGML_ORACLE_H
#define GGML_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

float    orc_fp16_to_fp32(uint16_t h);
uint16_t orc_fp32_to_fp16(float f);

/* dequantize_row_{q4_0,q8_0,q4_K,q5_K,q6_K} (ggml-quants.c:1523,1617,2556,2764,2978), f16, f32 */
void orc_dequantize_row(int type, const void *x, float *y, int64_t k);

/* activation quantization: vec_dot_type of `wtype` (ggml.c:793-959) */
int  orc_vec_dot_type(int wtype);
int64_t orc_row_bytes(int type, int64_t k);
void orc_quantize_row_q8_K(const float *x, void *y, int64_t k);
void orc_quantize_row_q8_0(const float *x, void *y, int64_t k);
void orc_quantize_row_q4_0(const float *x, void *y, int64_t k);   /* quantize_row_q4_0_ref, ggml-quants.c:669 */
void orc_quantize_row(int vtype, const float *x, void *y, int64_t k);

/* ggml_vec_dot_<wtype>_<vec_dot_type> for one row (ggml-quants.c:3922,5519,7714,8282,8919) */
float orc_vec_dot(int wtype, int n, const void *w, const void *a);

/* dst[m*N + n] = W[n,:] . X[m,:]  (ggml_compute_forward_mul_mat, ggml.c:12486-12707) */
void orc_mul_mat(int wtype, const void *W, int64_t K, int64_t N, const float *X, int64_t M,
                 float *dst, int nthreads);

/* ggml_compute_forward_rms_norm_f32 (ggml.c:12059) followed by ggml_mul with w (may be NULL) */
void orc_rms_norm(const float *x, const float *w, float *y, int64_t ne0, int64_t nrows, float eps);

/* ggml_compute_forward_rope_f32, NORM mode (ggml.c:14272-14378); x is [n_tokens][n_heads][head_dim] */
void orc_rope(const float *x, float *y, int64_t head_dim, int64_t n_heads, int64_t n_tokens,
              const int32_t *pos, int n_dims, float freq_base, float freq_scale,
              const float *freq_factors, float ext_factor, float attn_factor,
              float beta_fast, float beta_slow, int n_ctx_orig);

/* ggml_compute_forward_flash_attn_ext_f16 with F16 K/V (ggml.c:15667-15860).
 * q   [n_q][n_head][D] f32, k/v [n_kv][n_head_kv][D] f16 (row stride kv_stride elements),
 * mask [n_q][n_kv] f16 (may be NULL), out [n_q][n_head][D] f32 */
void orc_flash_attn_ext(const float *q, const uint16_t *k, const uint16_t *v, int64_t kv_stride,
                        const uint16_t *mask, float *out, int D, int n_q, int n_head,
                        int n_kv, int n_head_kv, float scale, int nthreads);

/* the same with a quantized K and V (Q8_0 / Q4_0 ggml block rows; ggml.c:15748-15851): Q quantized to Q8_0,
 * integer-block dot, V dequantized and accumulated in f32.  Row p of kv head hk at base + p*row_bytes +
 * hk*orc_row_bytes(type, D). */
void orc_flash_attn_ext_q(const float *q, const void *k, const void *v, int64_t k_row_bytes, int64_t v_row_bytes,
                          int ktype, int vtype, const uint16_t *mask, float *out, int D, int n_q, int n_head,
                          int n_kv, int n_head_kv, float scale, int nthreads);

/* diagnostic: 1 = accumulate V in f32 in orc_flash_attn_ext (NOT the reference's f16 VKQ16) */
void orc_set_fa_f32_accum(int on);

/* ---------------- Llama forward (build_llama, src/llama.cpp:10453-10620) ---------------- */
typedef struct {
    int n_vocab, n_embd, n_head, n_head_kv, n_layer, n_ff, n_ctx;
    float eps, rope_base, rope_freq_scale;
    int n_expert, n_expert_used;     /* 0 = dense FFN; else mixture of experts (llm_build_moe_ffn) */
} orc_hparams;

/* weights: 3 + LW*n_layer entries (LW = 9 dense, 10 MoE) in this order:
 *   tok_embd, output_norm, output, then per layer
 *   attn_norm, wq, wk, wv, wo, ffn_norm, ffn_gate, ffn_up, ffn_down (, ffn_gate_inp)
 * MoE: ffn_gate/up/down hold n_expert consecutive [K][N] slices (ggml's [K, N, n_expert] _exps
 * tensors); ffn_gate_inp is the [n_embd, n_expert] router. */
typedef struct orc_llama orc_llama;
orc_llama *orc_llama_create(const orc_hparams *hp, const void *const *data, const int *types, int nthreads);
void       orc_llama_free(orc_llama *m);
/* KV cache types (koboldcpp --quantkv): KT_F16 (default) or KT_Q8_0 / KT_Q4_0 for both; call before eval */
int        orc_llama_set_kv_types(orc_llama *m, int type_k, int type_v);
/* evaluate n_tokens at positions n_past.. ; writes last-token logits (n_vocab) */
int        orc_llama_eval(orc_llama *m, const int32_t *tokens, int n_tokens, int n_past, float *logits);
/* optional debug: copy hidden state of last token after last layer's ffn (n_embd) */
void       orc_llama_last_hidden(orc_llama *m, float *out);

#ifdef __cplusplus
}
#endif
#endif
