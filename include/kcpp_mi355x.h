/*
 * kcpp_mi355x.h -- C ABI of koboldcpp_amd/koboldcpp_hipblas.so (MI355X / gfx950 ggml backend).
 *
 * Plain pointers and sizes only.  Device pointers are HIP device addresses; `stream` is a
 * hipStream_t (NULL = default stream).  Every function returns 0 on success, <0 on error
 * (never aborts across the ABI: mirrors the reference's "return failure, never throw" rule,
 * SURVEY.md §8b b2).
 *
 * Three layers:
 *   1. kernel entry points (what ggml_cuda_compute_forward dispatches to in the reference,
 *      ggml/src/ggml-cuda.cu:2145-2349) -- used by the parity tests;
 *   2. the Llama runtime (the part of src/llama.cpp + ggml-backend scheduling this backend
 *      executes on the device: build_llama :10453, llama_decode_internal :17114);
 *   3. the koboldcpp drop-in ABI (expose.cpp/expose.h) -- declared in include/kcpp_expose.h.
 *
 * Tensor data layouts: weights live in the "kcpp layout" (same byte count as ggml; Q6_K, Q4_0,
 * Q8_0 are split into structure-of-arrays streams -- koboldcpp_amd/csrc/kcpp_common.h);
 * activations, KV caches and outputs follow ggml's row-major order.
 */
#ifndef KCPP_MI355X_H
#define KCPP_MI355X_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---------- 1. kernels ---------- */

/* ggml layout <-> kcpp layout (to_ggml=0: ggml->kcpp).  Replaces ggml_backend_cuda_buffer_set_tensor /
 * get_tensor byte copies (ggml/src/ggml-cuda.cu:471-484) for quantized weights. */
int kcpp_weight_repack(int type, const void *src, void *dst, int64_t K, int64_t N, int to_ggml, void *stream);
/* deterministic synthetic weights (include/kcpp_synth.h) written directly in kcpp layout */
int kcpp_weight_synth(int type, uint64_t seed, uint64_t tid, void *dst, int64_t K, int64_t N, void *stream);
/* dequantize a whole kcpp-layout tensor to f32 [N][K] (ggml_get_to_fp32_cuda, convert.cu) */
int kcpp_dequantize(int type, const void *w, float *y, int64_t K, int64_t N, void *stream);
/* get_rows of a quantized table (k_get_rows, getrows.cu:5): y[t] = dequant(W[ids[t]]) */
int kcpp_get_rows(int type, const void *w, int64_t K, int64_t N, const int32_t *ids, int64_t T, float *y,
                  int64_t ldy, void *stream);

/* activation quantization to the CPU vec_dot_type of the weight (Q8_K or Q8_0), bit-exact with
 * quantize_row_q8_K_ref / quantize_row_q8_0 (ggml-quants.c:3786,940).  Replaces quantize_q8_1
 * (ggml/src/ggml-cuda/quantize.cu:4-38). */
int64_t kcpp_act_bytes(int wtype, int64_t K, int64_t M);
int kcpp_vec_dot_type(int wtype);
int kcpp_quantize_act(int vtype, const float *x, int64_t ldx, void *out, int64_t K, int64_t M, void *stream);
/* Q8_K of silu(g) * u with g = x[m][i], u = x[m][uoff + i] (fused gate|up GEMM output; = k_silu_mul + quantize) */
int kcpp_quantize_act_glu(const float *x, int64_t ldx, int64_t uoff, void *out, int64_t K, int64_t M, void *stream);

/* Quantized mat-vec for M <= 8 columns (replaces mul_mat_vec_q, mmvq.cu:50-202):
 *   mode 0: Y[c][n] = W[n].x[c] (+ res[c][n])     mode 1: Y[c][n] = silu(W[n].x[c]) * (W2[n].x[c]) */
int kcpp_gemv(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
              int64_t ldy, const float *res, int64_t ldr, int mode, void *stream);

/* Batched quantized mat-mul on MFMA for M > 8 (replaces mul_mat_q / the hipBLAS dequant path,
 * mmq.cuh:2572-2905, ggml-cuda.cu:1186-1284).  act from kcpp_quantize_act (mode 0/1 as gemv). */
int64_t kcpp_gemm_workspace_bytes(int type, int64_t K, int64_t N, int64_t M);
int kcpp_gemm(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
              int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, void *stream);
/* Q6_K prefill image (same MUL_MAT role as kcpp_gemm on KT_Q6_K_RS, int8 matrix cores): the exact weight integers
 * sc*(q-32) of a Q6_K_RS matrix as two int8 planes, N*K*2 bytes (0 = shape not covered: N % 128, K % 256).
 * kcpp_gemm_q6p gives kcpp_gemm(KT_Q6_K_RS, ...)'s results bit for bit (M > 32; ws of kcpp_gemm_workspace_bytes). */
int64_t kcpp_q6p_image_bytes(int64_t K, int64_t N);
int kcpp_q6p_build(const void *W, int64_t K, int64_t N, void *img, void *stream);
int kcpp_gemm_q6p(const void *img, const void *W, const void *img2, const void *W2, int64_t K, int64_t N, const void *act,
                  int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, void *stream);
/* Grouped expert GEMM for MoE prefill (replaces ggml_cuda_mul_mat_id's per-expert loop, ggml-cuda.cu:2003-2139):
 * ng groups of cnt_host[e] rows (act: Q8_K of all M rows, grouped back to back; cnt_dev the same counts on the
 * device), group e against W + e*wstride (and W2 + e*wstride); mode 0 plain, 1 silu(g)*u with up [M][N] scratch.
 * Q4_K / Q5_K and their RS layouts; Q6_K_RS in mode 0 with ws of kcpp_gemm_grouped_ws_bytes (else ws unused,
 * may be NULL); Y is [M][N]. */
int64_t kcpp_gemm_grouped_ws_bytes(int type, int64_t K, int64_t M, int ng);
int kcpp_gemm_grouped(int type, const void *W, const void *W2, int64_t wstride, int64_t K, int64_t N, const void *act,
                      int64_t M, const int32_t *cnt_host, const int32_t *cnt_dev, int ng, float *Y, float *up, int mode,
                      void *ws, void *stream);
/* Q4_K GEMM kernel generation for later kcpp_gemm calls: 3 (= 0, the default; env KCPP_GEMM_V) = 128(64) x 128
 * tiles, LDS-DMA activation, register-dequantized weights; 2 = 128(256) x 64 tiles, LDS weights.  Same results
 * bit for bit.  Returns the previous value. */
int kcpp_gemm_set_variant(int v);
/* Q8_0 at M <= 32 over nseg <= 3 weights whose outputs sit back to back in Y's columns (q|k|v of one layer,
 * one activation quantization and one launch instead of three); every N_i but the last a multiple of 128;
 * ws from kcpp_gemm_workspace_bytes(KT_Q8_0, K, sum N_i, M) */
/* silu(W.x) * (W2.x) for Q8_0 weights at M <= 32, emitted directly as Q8_0 activations (the down projection's
   input; = kcpp_gemm(mode 1) then kcpp_quantize_act(Q8_0), bit for bit).  ws as for kcpp_gemm(KT_Q8_0, K, N, M). */
int kcpp_gemm_q80_glu_q80(const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, void *qout,
                          void *ws, void *stream);
int kcpp_gemm_q80_segs(const void *const *W, const int64_t *N, int nseg, int64_t K, const void *act, int64_t M, float *Y,
                       int64_t ldy, void *ws, void *stream);

/* Fused single-token mat-vec (koboldcpp_amd/csrc/gemv_dec.hip): args points at a DecArgs struct
 * (koboldcpp_amd/csrc/kcpp_internal.h, size kcpp_gemv_dec_args_size()).  mode 0 plain(+res),
 * 1 silu-GLU, 2 RoPE + K/V-cache store; pro 0 act given, 1 rms_norm+quantize prologue, 2 quantize. */
int kcpp_gemv_dec(int type, const void *args, int mode, int pro, int rows_per_wave, void *stream);
int64_t kcpp_gemv_dec_args_size(void);
/* the coalesced-streaming Q4_K variant kcpp_gemv_dec dispatches to (koboldcpp_amd/csrc/gemv_stream.hip);
 * returns -3 when the type/shape/mode is not covered.  Exposed for the parity tests and tools. */
int kcpp_gemv_stream(int type, const void *args, int mode, int pro, void *stream);
/* the VALU-lean unit-per-lane Q4_K variant (koboldcpp_amd/csrc/gemv_q4k.hip), tried first for Q4_K;
 * -3 when not covered */
int kcpp_gemv_q4k(const void *args, int mode, int pro, void *stream);
/* single-token mat-vec over the row-major decode layouts KT_Q4_K_RS / KT_Q6_K_RS (type ids 112 / 114,
 * koboldcpp_amd/csrc/gemv_rs.hip); kcpp_gemv_dec dispatches these types here.  kcpp_rs_supported(type, K)
 * says whether a [K x N] weight of Q4_K / Q6_K (or its RS id) can be held in the RS layout. */
int kcpp_gemv_rs(int type, const void *args, int mode, int pro, void *stream);
/* q|k|v decode projection (mode 2, rms_norm + Q8_K prologue) with segments 0, 1 (q, k) in KT_Q4_K_RS and segment 2
 * (v) in KT_Q6_K_RS -- the Q4_K_M "more bits" layers -- in one launch; -3 when the shape is not covered */
int kcpp_gemv_rs_qkv_mixed(const void *args, void *stream);
/* decode q|k|v with q in an RS layout (Q4_K / Q5_K / Q6_K, qargs) and k|v in Q8_0 (kvargs) -- Mixtral's Q5_K_M
 * policy -- as one grid holding both mat-vec launches' workgroups (mode 2 each, results identical to the two
 * kcpp_gemv_dec calls); -3 when not covered */
int kcpp_gemv_qkv_dual(const void *qargs, int qtype, const void *kvargs, void *stream);
int kcpp_rs_supported(int type, int64_t K);

/* rms_norm (ggml.c:12059) * w, optionally quantized to Q8_K in the same pass (q8k_out) */
int kcpp_rms_norm(const float *x, int64_t ldx, const float *w, float *y, int64_t ldy, void *q8k_out, int64_t ne0,
                  int64_t nrows, float eps, void *stream);
/* split-K partials [KS][Mp][ne0] summed in split order (+ res) into x, then kcpp_rms_norm(x, w, -> q8k_out): one
 * launch, bit for bit the reduce followed by the norm (the residual GEMM's reduce and the next ggml RMS_NORM + MUL) */
int kcpp_reduce_rms_norm(const float *part, int KS, int64_t Mp, const float *res, int64_t ldr, float *x, int64_t ldx,
                         const float *w, void *q8k_out, int64_t ne0, int64_t nrows, float eps, void *stream);
/* kcpp_gemm (mode 0) / kcpp_gemm_q6p followed by kcpp_rms_norm(Y, norm_w, -> q8k_out), the norm folded into the
 * GEMM's split-K reduce when it splits (results identical to the two calls) */
int kcpp_gemm_rms_norm(int type, const void *W, int64_t K, int64_t N, const void *act, int64_t M, float *Y, int64_t ldy,
                       const float *res, int64_t ldr, void *ws, void *stream, const float *norm_w, float eps, void *q8k_out);
int kcpp_gemm_q6p_rms_norm(const void *img, const void *W, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
                           int64_t ldy, const float *res, int64_t ldr, void *ws, void *stream, const float *norm_w, float eps,
                           void *q8k_out);
/* rms_norm * w quantized to Q8_0 in the same pass (= kcpp_rms_norm then kcpp_quantize_act(Q8_0), bit for bit) */
int kcpp_rms_norm_q80(const float *x, int64_t ldx, const float *w, void *q80_out, int64_t ne0, int64_t nrows, float eps,
                      void *stream);
/* the same quantized into the KT_Q8_0_TA activation layout of KT_Q8_0_T weights (kcpp_common.h) */
int kcpp_rms_norm_q80t(const float *x, int64_t ldx, const float *w, void *q80t_out, int64_t ne0, int64_t nrows, float eps,
                       void *stream);
/* mat-mul of KT_Q8_0_T weights (Q8_0 in 32-row tile fragments, kcpp_common.h) with a KT_Q8_0_TA activation of M tokens
 * (any M; replaces ggml_cuda_op_mul_mat's MMQ / MMVQ for Q8_0, ggml-cuda.cu:1882-1947): mode 0, up to 3 weight segments
 * [K][Ns[i]] whose rows sit back to back in Y's columns, Y (+ res); mode 1 (one segment, W2 = up): h = silu(W act) *
 * (W2 act) as f32 into Y, or, with qout, quantized to the KT_Q8_0_TA activation of h (K = Ns[0]).  ws:
 * kcpp_gemm_workspace_bytes(KT_Q8_0_T, K, sum Ns, M) bytes, zero before its first use (split-K tickets). */
int64_t kcpp_q80t_ws_bytes(int64_t K, int64_t N, int64_t M);
int kcpp_gemm_q80t(const void *const *Ws, const int64_t *Ns, int nseg, const void *W2, int64_t K, const void *act,
                   int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr, int mode, void *qout, void *ws,
                   void *stream);
/* q|k|v (3 segments, Ns = {H D, HKV D, HKV D}) as kcpp_gemm_q80t mode 0 with kcpp_rope_kv fused into the epilogue
 * (llama.cpp's ggml_rope_ext of Qcur/Kcur + the ggml_cpy of K/V into the cache, src/llama.cpp:9180-9202): rope(q) ->
 * q16 [M][H D] f16, rope(k) and v -> kc / vc [pos][HKV D] f16 at pos_dev[t] (or n_past + t); bit-identical to the GEMM
 * then kcpp_rope_kv. */
int kcpp_gemm_q80t_qkv_rope(const void *const *Ws, const int64_t *Ns, int64_t K, const void *act, int64_t M,
                            const void *rope_tab, int n_past, const int32_t *pos_dev, int head_dim, uint16_t *q16,
                            uint16_t *kc, uint16_t *vc, void *ws, void *stream);
/* host-side table of (cos, sin) per [pos][D/2], exactly as ggml_rope_cache_init (ggml.c:14246) */
int kcpp_rope_table(float *tab_host, int n_pos, int n_dims, float freq_base, float freq_scale, const float *freq_factors,
                    float ext_factor, float attn_factor, float beta_fast, float beta_slow, int n_ctx_orig);
/* rope(q), rope(k) (NORM mode) + f16 store of K and V into the caches at positions pos.. */
/* one position's (cos, sin) pairs of the table above; p may be negative (a K-shift distance) */
int kcpp_rope_row(float *row_host, int p, int n_dims, float freq_base, float freq_scale, float ext_factor,
                  float attn_factor, float beta_fast, float beta_slow, int n_ctx_orig);
/* K-shift of cache rows: ks = f16(rope(f32(kc), cs)) per adjacent pair (ggml_compute_forward_rope_f16, NORM),
 * vs = vc; rows x D f16 each, cs = D floats (cos, sin per pair, device) */
int kcpp_kv_shift_rows(const uint16_t *kc, const uint16_t *vc, uint16_t *ks, uint16_t *vs, int64_t rows, int D,
                       const float *cs, void *stream);
int kcpp_rope_kv(const float *qkv, int64_t ldqkv, float *q_out, uint16_t *q16, uint16_t *kc, uint16_t *vc, int T,
                 int H, int HKV, int D, int n_past, const int32_t *pos_dev, const void *rope_tab, void *stream);
/* flash attention over the f16 cache (ggml_cuda_flash_attn_ext, fattn.cu:298-345) */
/* force_path: 0 auto, 1 decode (T = 1: k_fa_dec4 splits + k_fa_comb4), 2 FMA-tiled prefill, 3 MFMA prefill
 * (D = 128, H = 4 HKV), 6 decode through the 64-key chunked kernel even at T = 1 */
int64_t kcpp_fa_workspace_bytes(int T, int H, int n_kv_max);
int kcpp_flash_attn(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qout, void *ws,
                    int T, int H, int HKV, int D, int n_past, const int32_t *n_past_dev, int n_kv_max, float scale,
                    int force_path, void *stream);
/* strict-parity attention: the reference CPU's order (ggml.c:15667-15875) with its f16 V accumulator, one serial
 * chain per (query, head, dim) -- bit-for-bit the AVX2 build's arithmetic up to exp rounding (attn_exact.hip).
 * Same layouts and causal window as kcpp_flash_attn; D = 128. */
int kcpp_flash_attn_exact(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, int T, int H,
                          int HKV, int D, int n_past, const int32_t *n_past_dev, float scale, void *stream);
/* the same in the ggml op's graph form (arguments as kcpp_flash_attn_ext, no workspace): the b1 backend's strict mode */
int kcpp_flash_attn_ext_exact(const float *q, int64_t q_nb1, int64_t q_nb2, const uint16_t *kc, const uint16_t *vc,
                              const uint16_t *mask, int64_t mask_ld, float *out, int T, int H, int HKV, int D, int n_kv,
                              float scale, void *stream);
/* quantized KV cache (koboldcpp --quantkv 1/2 = q8_0/q4_0 K and V, gpttype_adapter.cpp:1958-1959; attn_kvq.hip).
 * Per-layer cache layout: Q8_0 = qs int8 [n_ctx][ekv] ++ d f16 [n_ctx][ekv/32]; Q4_0 = qs [n_ctx][ekv/2] (ggml
 * nibble order per 32-block) ++ d f16 [n_ctx][ekv/32].  kcpp_kv_cache_bytes(KT_F16 / KT_Q8_0 / KT_Q4_0, ...). */
int64_t kcpp_kv_cache_bytes(int type, int64_t n_ctx, int64_t ekv);
/* RoPE (mode NORM, table as kcpp_rope_table) of the q and k heads in place in f32 q|k|v rows (stride ld) */
int kcpp_rope_qk_inplace(float *qkv, int64_t ld, int T, int H, int HKV, int D, int n_past, const int32_t *pos_dev,
                         const void *rope_tab, void *stream);
/* K (column koff) and V (column voff) of T f32 rows into the quantized caches at n_past + t (pos_dev[0] + t when
 * given): quantize_row_q8_0 (AVX2 rounding) / quantize_row_q4_0_ref, ggml-quants.c */
int kcpp_kv_store_q(int tk, int tv, const float *qkv, int64_t ld, int64_t koff, int64_t voff, int T, int64_t ekv,
                    void *kc, void *vc, int64_t n_ctx, int n_past, const int32_t *pos_dev, void *stream);
/* causal attention of T f32 query rows (stride ldq, head h at h*D) over quantized caches, positions
 * [0, n_past + t]: q quantized to Q8_0, s = sum_b d_k d_q (integer dot), V dequantized, f32 accumulation
 * (ggml_compute_forward_flash_attn_ext_f16 with a quantized K/V, ggml.c:15750-15840); D = 64 or 128 */
int kcpp_flash_attn_q(int tk, int tv, const float *q, int64_t ldq, const void *kc, const void *vc, float *out, int T,
                      int H, int HKV, int D, int64_t n_ctx, int n_past, const int32_t *n_past_dev, float scale,
                      void *stream);
/* single-token decode attention with explicit cache strides in elements (key p of kv head hk at
 * kc + p*kv_ld + hk*kv_hs); variant 0: 64-key chunks + combine, 3: the production k_fa_dec4 splits +
 * k_fa_comb4 (A/B measurement entry, tools/fa_dec_bench.py) */
int kcpp_fa_decode_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, int64_t kv_ld, int64_t kv_hs,
                      float *out, void *qout, void *ws, int H, int HKV, int n_past, const int32_t *n_past_dev,
                      int n_kv_max, float scale, int variant, void *stream);
/* diagnostic: per-workgroup phase stamps of the split-KV decode kernel (s_memrealtime, 8 per workgroup) into p
 * (device, or NULL to disable); tools only */
void kcpp_fa_set_stamps(void *p);
/* the MFMA prefill kernel alone (koboldcpp_amd/csrc/attn_mfma.hip); -3 when the shape is not covered */
int kcpp_flash_attn_prefill_mfma(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, int T, int H,
                                 int HKV, int D, int n_past, float scale, void *stream);
/* the same with, for T <= 64 and ws (kcpp_fa_workspace_bytes, zero before first use), the keys split over ~512
 * workgroups merged in-launch by the last split; out (f32 [T][H D], may be NULL) and/or qta (the KT_Q8_0_TA
 * activation of attn_output for KT_Q8_0_T weights, replacing kcpp_quantize_act; may be NULL).  -3 = not covered. */
int kcpp_flash_attn_prefill_mfma_ex(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qta,
                                    void *ws, int T, int H, int HKV, int D, int n_past, float scale, void *stream);
int64_t kcpp_fa_split_ws_bytes(int H);
/* single-token decode attention (the k_fa_dec5 + k_fa_comb4 pair) with the combine writing the KT_Q8_0_TA activation of
 * the token (qta) -- bit-identical to kcpp_quantize_act(KT_Q8_0_TA) of its f32 output; n_kv_max = the caches' row count
 * when n_past_dev is given (the graph-replayable form); -3 = not covered */
int kcpp_flash_attn_dec_ta(const uint16_t *q16, const uint16_t *kc, const uint16_t *vc, float *out, void *qta, void *ws,
                           int H, int HKV, int D, int n_past, const int32_t *n_past_dev, int n_kv_max, float scale,
                           void *stream);
/* MFMA prefill kernel generation: 2 (default; env KCPP_FA_MFMA_V) = next tile prefetched, V read through the
 * LDS transpose; 1 = the first version; 0 = the default.  Bit-identical outputs.  Returns the previous value. */
int kcpp_fa_prefill_set_variant(int v);
/* MoE router (llm_build_moe_ffn, src/llama.cpp:9435-9460): logits = W_router . x (W F16 -> x rounded
 * to f16 like the CPU vec_dot_f16, or F32), softmax, top-k (argsort descending), weights normalized to
 * sum 1; ids/weights [T][k] */
int kcpp_moe_route(const float *x, int64_t ldx, const void *w_router, int wtype, int64_t K, int n_expert, int k,
                   int32_t *ids, float *weights, int T, void *stream);
/* the router on rms_norm(x) * norm_w computed in the same launch (k_rms_norm's arithmetic; K <= 4096,
 * n_expert <= 8); -3 when not covered */
int kcpp_moe_route_norm(const float *x, int64_t ldx, const float *norm_w, float eps, const void *w_router, int wtype,
                        int64_t K, int n_expert, int k, int32_t *ids, float *weights, int T, void *stream);
/* MoE helpers: dst[i] = src[rows[i]] (row gather); dst[rows[i]] = w[i] * src[i] (weighted scatter into
 * the token's top-k slot row); combine: x[i] = ((slots[0][i] + slots[1][i]) + ...) + x[i] over k slots
 * spaced slot_stride floats (the ggml_add chain of llm_build_moe_ffn, src/llama.cpp:9500-9515) */
int kcpp_moe_gather(const float *src, int64_t lds, const int32_t *rows, int n, int64_t E, float *dst, void *stream);
int kcpp_moe_scatter(float *dst, int64_t ldd, const float *src, const int32_t *rows, const float *w, int n, int64_t E,
                     void *stream);
int kcpp_moe_combine(float *x, const float *slots, int64_t slot_stride, int k, int64_t n, void *stream);
int kcpp_add(float *y, const float *a, const float *b, int64_t n, void *stream);
int kcpp_silu_mul(float *y, const float *g, const float *u, int64_t n, void *stream);

/* ---------- 1b. general-layout ggml node kernels (the b1 backend, csrc/ggml_backend.cpp) ----------
 * A tensor is described by its ggml shape and byte strides (ggml_tensor.ne / .nb); data pointers are
 * device pointers.  Each entry follows the reference CPU op named in csrc/ggml_ops.hip. */
typedef struct kcpp_tdesc {
    int64_t ne[4];
    int64_t nb[4];
} kcpp_tdesc;
enum { KCPP_BIN_ADD = 0, KCPP_BIN_SUB = 1, KCPP_BIN_MUL = 2, KCPP_BIN_DIV = 3 };
enum { KCPP_UN_SILU = 0, KCPP_UN_SCALE = 1, KCPP_UN_NEG = 2, KCPP_UN_RELU = 3 };
/* d = a (op) b, b broadcast over d's shape by modulo (ggml_can_repeat) */
int kcpp_ggml_binary(int op, const void *a, const kcpp_tdesc *ta, const void *b, const kcpp_tdesc *tb, void *d,
                     const kcpp_tdesc *td, void *stream);
/* d = f(a); KCPP_UN_SCALE multiplies by param */
int kcpp_ggml_unary(int op, const void *a, const kcpp_tdesc *ta, void *d, const kcpp_tdesc *td, float param,
                    void *stream);
/* element-order copy with conversion (KT_F32 / KT_F16 each side); shapes may differ, counts equal */
int kcpp_ggml_cpy(int stype, const void *src, const kcpp_tdesc *ts, int dtype, void *dst, const kcpp_tdesc *td,
                  void *stream);
int kcpp_ggml_rms_norm(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, float eps, void *stream);
/* b1 fusion: rms_norm then MUL by the broadcast weight w (build_norm), one launch writing both outputs: r = the norm
 * node's tensor, y = the MUL node's; each element the two nodes' bits.  Rows contiguous (nb[0] = 4), else -2 */
int kcpp_ggml_rms_norm_mul(const void *x, const kcpp_tdesc *tx, void *r, const kcpp_tdesc *tr, void *y,
                           const kcpp_tdesc *ty, const float *w, const kcpp_tdesc *tw, float eps, void *stream);
/* GGML_OP_ROPE f32, mode 0 (NORM) or 2 (NEOX); pos int32 [ne2]; freq_factors may be null */
/* b1 fusion: the same ROPE also storing each value as f16 at its linear element index in y16 (the CPY of the roped
 * tensor into a contiguous F16 cache view that follows it); y must be contiguous */
int kcpp_ggml_rope_f16(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, void *y16, const int32_t *pos,
                       const float *freq_factors, int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale,
                       float ext_factor, float attn_factor, float beta_fast, float beta_slow, void *stream);
int kcpp_ggml_rope(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, const int32_t *pos,
                   const float *freq_factors, int n_dims, int mode, int n_ctx_orig, float freq_base, float freq_scale,
                   float ext_factor, float attn_factor, float beta_fast, float beta_slow, void *stream);
/* softmax(x * scale + mask[row % mask_rows]) per row; mask KT_F16 / KT_F32 or null */
int kcpp_ggml_soft_max(const void *x, const kcpp_tdesc *tx, const void *mask, int mask_type, int64_t mask_ld,
                       int64_t mask_rows, void *y, const kcpp_tdesc *ty, float scale, void *stream);
int kcpp_ggml_argsort(const void *x, const kcpp_tdesc *tx, int32_t *d, int64_t ld, int desc, void *stream);
int kcpp_ggml_sum_rows(const void *x, const kcpp_tdesc *tx, void *y, const kcpp_tdesc *ty, void *stream);
/* dst[:, i10, i11, i12] = src[:, ids[i10, i11, i12], i11, i12] for KT_F32 / KT_F16 sources */
int kcpp_ggml_get_rows(int stype, const void *src, const kcpp_tdesc *ts, const int32_t *ids, const kcpp_tdesc *ti,
                       void *dst, const kcpp_tdesc *td, void *stream);
/* mul_mat with a KT_F16 (src1 rounded to f16, vec_dot_f16), KCPP_MM_F16_X32 (F16 weight x f32 src1 without
 * rounding: the reference CPU's tinyBLAS route when built with AVX2/F16C, llamafile/sgemm.cpp:1094-1103) or KT_F32
 * weight, any strides, batched */
#define KCPP_MM_F16_X32 0x101
int kcpp_ggml_mul_mat_f(int wtype, const void *w, const kcpp_tdesc *tw, const float *x, const kcpp_tdesc *tx, float *d,
                        const kcpp_tdesc *td, void *stream);
/* GGML_OP_FLASH_ATTN_EXT in the graph's own form: q f32 (byte strides q_nb1 per query, q_nb2 per head), K/V f16
 * cache views [n_kv][HKV][128], optional f16 mask [T][n_kv] (row stride mask_ld; -inf keys skipped), out f32
 * [T][H][128]; ws of kcpp_fa_ext_workspace_bytes */
int64_t kcpp_fa_ext_workspace_bytes(int T, int H, int n_kv, int D);
/* f32 row moves (the MoE mat-mul's gather / scatter): dst row i <- src row i, K floats, each side addressed by byte
 * offsets (offs != NULL) or by a byte stride (ld) */
int kcpp_rows_move_f32(const void *src, const int64_t *soffs, int64_t sld, void *dst, const int64_t *doffs, int64_t dld,
                       int64_t K, int n, void *stream);
int kcpp_flash_attn_ext(const float *q, int64_t q_nb1, int64_t q_nb2, const uint16_t *kc, const uint16_t *vc,
                        const uint16_t *mask, int64_t mask_ld, float *out, void *ws, int T, int H, int HKV, int D,
                        int n_kv, float scale, void *stream);
/* the same over quantized K / V views (--quantkv): tk / tv = KT_Q8_0 / KT_Q4_0, views of ggml blocks at byte strides
 * nb1 (position) / nb2 (kv head); q quantized to Q8_0 per 32-block and integer block dots, V dequantized, f32
 * accumulation (ggml_compute_forward_flash_attn_ext_f16's quantized branch, ggml.c:15748-15851); D 64 or 128 */
/* GGML_OP_CPY f32 -> Q8_0 / Q4_0 (KT_ ids) of n contiguous values (n % 32 == 0) into ggml blocks: the reference's
 * from_float (quantize_row_q8_0 AVX2 / quantize_row_q4_0_ref), byte for byte */
int kcpp_cpy_f32_q(int type, const float *src, int64_t n, void *dst, void *stream);
int kcpp_flash_attn_ext_q(int tk, int tv, const float *q, int64_t q_nb1, int64_t q_nb2, const void *kc, int64_t k_nb1,
                          int64_t k_nb2, const void *vc, int64_t v_nb1, int64_t v_nb2, const uint16_t *mask,
                          int64_t mask_ld, float *out, int T, int H, int HKV, int D, int n_kv, float scale, void *stream);

/* ---------- 2. Llama runtime ---------- */
typedef struct kcpp_hparams {
    int n_vocab, n_embd, n_head, n_head_kv, n_layer, n_ff, n_ctx;
    float eps, rope_base, rope_freq_scale;
    int n_expert, n_expert_used;     /* 0 = dense FFN; else Mixtral-style MoE (llm_build_moe_ffn) */
} kcpp_hparams;

typedef struct kcpp_model kcpp_model;

/* Layer range [il0, il1) lives on `device`; embed/output flags say whether this stage owns the
 * token embedding / output head (layer split, src/llama.cpp:7000-7036).  types[] has 3+LW*n_layer
 * entries (LW = 9 dense, 10 MoE) in canonical order: tok_embd, output_norm, output, then per layer
 * attn_norm, wq, wk, wv, wo, ffn_norm, ffn_gate, ffn_up, ffn_down (, ffn_gate_inp).  With MoE the
 * ffn_gate/up/down entries are the [K, N, n_expert] _exps tensors (n_expert consecutive [K, N]
 * slices, synthetic tid = index * 256 + expert) and ffn_gate_inp is the F16/F32 router. */
kcpp_model *kcpp_model_create(const kcpp_hparams *hp, const int *types, int device, int il0, int il1, int has_embed,
                              int has_output, int max_ubatch);
/* weights: synthetic (seed) or uploaded from host ggml-layout bytes (tensor index = canonical order) */
int kcpp_model_synth_weights(kcpp_model *m, uint64_t seed);
int kcpp_model_set_tensor(kcpp_model *m, int index, const void *ggml_bytes, int64_t nbytes);
void kcpp_model_free(kcpp_model *m);

/* One llama_decode of T tokens at n_past (T may exceed the ubatch: split internally).
 * If the stage has the embedding, `tokens` are used; otherwise the stage's input hidden state
 * must have been placed with kcpp_model_hidden_in.  If the stage has the output head, the last
 * token's logits are copied to logits_host (may be NULL). */
int kcpp_model_decode(kcpp_model *m, const int32_t *tokens, int T, int n_past, float *logits_host);
/* the same, enqueued on the stage's stream without any host synchronisation (pipeline driver: stages chained by
 * events / RCCL, one host sync per step) */
int kcpp_model_decode_async(kcpp_model *m, const int32_t *tokens, int T, int n_past);
int kcpp_model_device(kcpp_model *m);
/* device pointers of this stage's residual stream [max_ubatch][n_embd] f32 (pipeline handoff) */
float *kcpp_model_hidden(kcpp_model *m);
/* copy n floats of the residual stream starting at float offset (debug / pipeline host path) */
int kcpp_model_read_hidden(kcpp_model *m, float *host, int64_t n_floats, int64_t offset);
void *kcpp_model_stream(kcpp_model *m);
/* stream-ordered copy of n_floats of the residual stream at float offset to/from buf (device or host
 * memory): dir 0 = buf -> stage input, 1 = stage output -> buf.  Pipeline handoff (replaces
 * ggml_backend_cuda_cpy_tensor_async, ggml/src/ggml-cuda.cu:2392-2445). */
int kcpp_model_hidden_io(kcpp_model *m, void *buf, int64_t n_floats, int64_t offset, int dir);
/* copy the last decode's logits [n_vocab] f32 to host memory (stage with the output head) */
int kcpp_model_read_logits(kcpp_model *m, float *host);
/* wait for all work queued on the stage's stream */
int kcpp_model_sync(kcpp_model *m);
/* per-stage step without embedding/out: run layers on the hidden buffer for T tokens */
int kcpp_model_forward_hidden(kcpp_model *m, int T, int n_past);
/* greedy argmax of the last logits on device (avoids the 0.5 MB logits copy); also becomes the
 * next decode_greedy step's input token */
int kcpp_model_argmax(kcpp_model *m, int32_t *token_out);
/* the greedy token the last single-token step computed on device (every step of the stage with the output head ends
 * in its argmax): 4-byte read + stream sync, no launch */
int kcpp_model_read_argmax(kcpp_model *m, int32_t *token_out);
/* the same enqueued on the stage's stream (no host synchronisation): the token lands in kcpp_model_argmax_dev */
int kcpp_model_argmax_async(kcpp_model *m);
/* one single-token step at n_past whose input token is already in kcpp_model_token_dev (stage with the embedding;
 * other stages take their hidden input as for decode_async); enqueued, no host synchronisation.  The stage with
 * the output head computes the step's greedy token into kcpp_model_argmax_dev (and, when it also owns the
 * embedding, into kcpp_model_token_dev: the next step's input).  Replaces the per-token host hop of the
 * pipeline's greedy loop (the reference reads the token on the host: llama_sampling + llama_decode). */
int kcpp_model_step_dev(kcpp_model *m, int n_past);
int32_t *kcpp_model_token_dev(kcpp_model *m);
int32_t *kcpp_model_argmax_dev(kcpp_model *m);
/* one greedy generation step at n_past: input = the previous argmax (device-resident), the step's
 * own argmax computed in the same graph replay and returned (one host sync per token).
 * Requires a stage owning both the embedding and the output head. */
int kcpp_model_decode_greedy(kcpp_model *m, int n_past, int32_t *token_out);
/* the same step with the host one token behind the device: returns the PREVIOUS step's token (-1 on the first call
 * after a drain) once its 4-byte read has landed, while this step is already queued; kcpp_model_greedy_drain returns
 * the last step's token and resets the readback ring */
int kcpp_model_decode_greedy_lagged(kcpp_model *m, int n_past, int32_t *token_out);
int kcpp_model_greedy_drain(kcpp_model *m, int32_t *token_out);
/* context shift (koboldcpp PurgeMissingTokens, gpttype_adapter.cpp:1504-1571: llama_kv_cache_seq_rm(p0, p0+diff)
 * + seq_add(p0+diff, n_past, -diff) + the K-shift of build_k_shift): cache rows [p0+diff, n_past) move to
 * [p0, n_past-diff) and K is re-rotated by position -diff (rope f16, mode NORM).  Synchronous. */
int kcpp_model_kv_shift(kcpp_model *m, int p0, int diff, int n_past);
/* rope frequency factors (rope_freqs.weight of Llama-3.1 / 3.2 GGUFs, n = head_dim / 2 F32 values): every rope of
 * the model and the context-shift K re-rotation divide the angle by them, as ggml_rope_ext with its freq_factors
 * operand (src/llama.cpp:7171, 10269, 10490; ggml.c ggml_rope_cache_init).  Rebuilds the rope table; synchronous. */
int kcpp_model_set_rope_freqs(kcpp_model *m, const float *freq_factors, int n);
/* koboldcpp's automatic RoPE base for a context beyond the trained one (CalcGradientAIRopeFreqBase,
 * gpttype_adapter.cpp:1598-1640); solar = the reference's ARCH_SOLAR rule (model_adapter.cpp:309) */
float kcpp_gradient_ai_rope_base(float original_rope_base, int n_ctx_train, int n_ctx_desired, int solar);
/* enable/disable hipGraph replay for single-token decode (default on) */
int kcpp_model_set_graphs(kcpp_model *m, int enable);
/* single-token decode through the fused mat-vec path (default on); off = one kernel per op */
int kcpp_model_set_fused_decode(kcpp_model *m, int enable);
/* 1: attention through kcpp_flash_attn_exact (reference order, f16 accumulation; strict-parity mode, slow);
 * 0 (default, or KCPP_FA_EXACT=1 at creation): the split-KV / MFMA kernels */
int kcpp_model_set_fa_exact(kcpp_model *m, int enable);
/* MoE: the expert ids the model's last MoE layer routed the last prefill's tokens to, n = T * n_expert_used
 * int32 ([token][slot], the router's top-k order); diagnostics for routing-aware parity tests */
int kcpp_model_moe_ids(kcpp_model *m, int32_t *out, int n);
/* MoE diagnostics: enable (1) / disable (0) a trace of single-token routing -- each MoE layer of the stage copies its
 * top-k expert ids into [layer][n_expert_used] every decode step; _read returns the last step's n ids */
int kcpp_model_moe_trace(kcpp_model *m, int enable);
int kcpp_model_moe_trace_read(kcpp_model *m, int32_t *out, int n);
/* MoE single-token decode fusions (bit 0: route inside the two-slot gate|up launch, else k_moe_route; bit 1: both
 * slots' down projections in one launch, else two chained launches; default 3); diagnostics */
int kcpp_model_set_fused_route(kcpp_model *m, int on);
/* enqueued so far (graph captures count once): routed gate|up launches (low 32 bits), two-slot down launches (high) */
int64_t kcpp_model_fused_route_count(kcpp_model *m);
/* MoE prefill: grouped expert GEMMs (1, default) or the per-expert loop (0); returns the previous setting.
 * kcpp_model_moe_grouped_count: grouped layers run so far (diagnostics) */
int kcpp_model_set_moe_grouped(kcpp_model *m, int on);
int64_t kcpp_model_moe_grouped_count(kcpp_model *m);
/* K / V cache types (llama_context_params type_k / type_v): KT_F16 (default) or quantized KT_Q8_0 / KT_Q4_0 for
 * both (koboldcpp --quantkv).  Reallocates and clears the caches; quantized caches run single-token decode
 * through the unfused per-op path and refuse kcpp_model_kv_shift (koboldcpp turns context shift off with
 * --quantkv, koboldcpp.py).  Returns -1 for other combinations. */
int kcpp_model_set_kv_types(kcpp_model *m, int type_k, int type_v);
/* row split (koboldcpp --rowsplit -> LLAMA_SPLIT_MODE_ROW, gpttype_adapter.cpp:1892; replaces the split buffer type
 * ggml_backend_cuda_split_buffer_type, ggml-cuda.cu:659-955, and ggml_cuda_op_mul_mat's per-device row ranges,
 * :1403-1700): the rows of every layer matrix and of the output matrix are spread over devices[0..n) by
 * tensor_split (proportions; all zero = equal), bounds rounded to 128 rows; everything else stays on the stage's
 * device.  n lanes may name the same GPU (each extra lane gets its own stream and buffers).  Call after create,
 * before the weights are set.  Turns graph replay and the fused single-token path off; refuses MoE (-3). */
int kcpp_model_set_row_split(kcpp_model *m, int n, const int *devices, const float *tensor_split);
/* the row range [lo, hi) of an nrows matrix on device id of n (host only; get_row_split, ggml-cuda.cu:638-651) */
int kcpp_row_split_range(int64_t nrows, int n, const float *tensor_split, int id, int64_t *lo, int64_t *hi);
int64_t kcpp_model_weight_bytes(kcpp_model *m);
/* bench.py --gpus N: the drop-in engine of load_model (layer-split stages over n_dev GPUs by tensor_split, RCCL or
 * event-ordered hand-off, pipelined ubatches: koboldcpp_amd/csrc/expose.cpp) on synthetic weights: prefill n_prompt
 * ids in ubatches of ub, then n_warm + n_steps greedy tokens with the token moved home on device (no host
 * synchronisation inside a step).  out = {prefill_s, decode_s of the n_steps tokens, n_past at the end, 1 if the
 * hand-off ran on RCCL}.  0 ok, -1 fewer than n_dev GPUs visible. */
int kcpp_engine_bench(const kcpp_hparams *hp, const int *types, int n_types, int n_dev, const float *tensor_split,
                      uint64_t seed, int n_prompt, int ub, int n_warm, int n_steps, double *out);
/* bench / test hook: the model load_model() holds gets the runtime's synthetic weights (kcpp_model_synth_weights per
 * stage; bench.py's generate() leg loads a sparse full-size GGUF, then this); 0 on success, -1 without a model */
int kcpp_expose_synth_weights(uint64_t seed);
/* test hook: the pipeline schedule's enqueue order (prefill, argmax, token home, `steps` greedy steps) for n_stages
 * stages, recorded by the schedule's trace backend into out (host only, no device calls) */
int kcpp_pipeline_trace(int n_stages, int ub, int T, int n_past, int steps, char *out, int cap);
/* test hook: load_model's layer placement (src/llama.cpp:7010-7036): out[i] = device of layer i, out[n_layer] =
 * the output head's device */
int kcpp_split_layers(int n_layer, int n_dev, const float *tensor_split, int *out);
const char *kcpp_last_error(void);

/* GGUF parse + tensor-table bounds validation alone (load_model's first step): 0 ok, -1 with the reason in err */
int kcpp_gguf_check(const char *path, char *err, int err_len);
/* host-only tokenizer probes (tests): the BPE pre-tokenizer of GGUF pre type `pre` (llm_tokenizer_bpe's
 * regex_exprs, src/llama-vocab.cpp:597-712; custom splits src/unicode.cpp:248-492) -> byte end offsets of the
 * words; and the GGUF vocabulary's full tokenization as generate() uses it (special tokens parsed,
 * tokenizer_st_partition src/llama-vocab.cpp:1544).  Return the count, -1 on error. */
int kcpp_pretokenize(const char *pre, const char *text, int64_t *ends, int cap);
int kcpp_tokenize_probe(const char *gguf_path, const char *text, int add_bos, int32_t *out, int cap);
/* every vocabulary id's streamed text (llama_token_to_piece_impl with special = false, src/llama-vocab.cpp:2007)
 * concatenated into out (<= cap bytes), ends[i] = end offset of id i; returns n_vocab, -1 on a load error (host only) */
int kcpp_pieces_probe(const char *gguf_path, char *out, int64_t cap, int64_t *ends, int n_ends);
/* the vocabulary's special ids as generate() uses them: out = {bos, eos, eot} (eot -1 when the vocabulary has none;
 * llm_load_vocab's EOT detection, src/llama.cpp:6606, 6642-6661).  0 ok, -1 on a load error */
int kcpp_tokenizer_special_ids(const char *gguf_path, int32_t *out);
/* generate()'s restated sampler chain (SampleLogits, gpttype_adapter.cpp:1338-1434) on caller logits, for the
 * host-side parity test (koboldcpp_amd/csrc/expose.cpp documents fp / ip / restarts); returns the drawn token */
int kcpp_sampler_probe(const float *logits, int n_vocab, int n_ctx, const float *fp, const int *ip, const int *order,
                       int n_order, const int *ctx_toks, int n_ctx_toks, const int *last_n, int n_last,
                       const int *restarts, int n_restart_ints, unsigned seed, float *mu, int *out_ids, float *out_p,
                       int cap, int *out_n);

#ifdef __cplusplus
}
#endif
#endif
