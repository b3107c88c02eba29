/*
 * ref_b1.c -- TEST / DIAGNOSTIC INFRASTRUCTURE ONLY (never part of bench.py's timed region).
 *
 * Decode throughput of a full Llama graph driven through the ggml backend plugin (b1) by the REFERENCE host
 * library, as a koboldcpp build that links koboldcpp_hipblas.so as its ROCm backend would run it: the reference
 * ggml (oracle/_ref/libggml_ref.so) builds build_llama's graph every token (src/llama.cpp:10453-10620 as restated in
 * ref_llama.c, flash attention on, KV cache f16, n_kv padded to 256 as llama_kv_cache does for flash attention),
 * ggml_backend_sched (ggml-backend.cpp) splits and allocates it over {our backend, the reference CPU backend} and
 * dispatches every node through our vtables (ggml_backend_cuda_init from the plugin, dlopen'ed), and the host reads
 * the logits and takes the argmax each token.  Weights: include/kcpp_synth.h's synthetic blocks, written with
 * ggml_backend_tensor_set into our buffer type; the KV cache rows below n_past are zeros (a decode step's cost
 * depends on the cache length, not its contents).
 *
 * usage: ref_b1 <plugin.so> <n_layer> <n_past> <n_steps> [types: "q4_k_m"]
 * prints one JSON line: decode tok/s, ms/token, nodes per graph, graph splits.
 */
#include "ggml.h"
#include "ggml-alloc.h"
#include "ggml-backend.h"
#include "../include/kcpp_synth.h"

#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Llama-3-8B shape; Q4_K_M per-tensor policy (llama_tensor_get_type, as tests/refharness.py q4_k_m_types):
   Q6_K attn_v / ffn_down on the "more bits" layers, Q4_K elsewhere, Q6_K output, Q4_K token embedding */
enum { NV = 128256, NE = 4096, NH = 32, NHKV = 8, NFF = 14336, NCTX = 4096 };

static int more_bits(int il, int nl) { return il < nl / 8 || il >= 7 * nl / 8 || (il - nl / 8) % 3 == 2; }

int main(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "usage: ref_b1 <plugin.so> <n_layer> <n_past> <n_steps>\n"); return 1; }
    const int n_layer = atoi(argv[2]), n_past0 = atoi(argv[3]), n_steps = atoi(argv[4]);
    if (n_layer < 1 || n_layer > 256 || n_past0 < 0 || n_past0 + n_steps + 1 > NCTX) return 1;
    void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 2; }
    ggml_backend_t (*cuda_init)(int) = (ggml_backend_t (*)(int))dlsym(h, "ggml_backend_cuda_init");
    if (!cuda_init) { fprintf(stderr, "no ggml_backend_cuda_init\n"); return 2; }
    ggml_backend_t be = cuda_init(0), cpu = ggml_backend_cpu_init();
    if (!be || !cpu) return 3;
    ggml_backend_cpu_set_n_threads(cpu, 8);

    const int D = NE / NH, EKV = NHKV * D;
    const int nw = 3 + 9 * n_layer;
    int *types = malloc(sizeof(int) * nw);
    int64_t (*shape)[2] = malloc(sizeof(*shape) * nw);
    types[0] = GGML_TYPE_Q4_K; shape[0][0] = NE; shape[0][1] = NV;
    types[1] = GGML_TYPE_F32; shape[1][0] = NE; shape[1][1] = 1;
    types[2] = GGML_TYPE_Q6_K; shape[2][0] = NE; shape[2][1] = NV;
    for (int il = 0; il < n_layer; ++il) {
        int *t = types + 3 + 9 * il;
        int64_t (*s)[2] = shape + 3 + 9 * il;
        const int mb = more_bits(il, n_layer);
        t[0] = GGML_TYPE_F32; s[0][0] = NE; s[0][1] = 1;
        t[1] = GGML_TYPE_Q4_K; s[1][0] = NE; s[1][1] = NE;
        t[2] = GGML_TYPE_Q4_K; s[2][0] = NE; s[2][1] = EKV;
        t[3] = mb ? GGML_TYPE_Q6_K : GGML_TYPE_Q4_K; s[3][0] = NE; s[3][1] = EKV;
        t[4] = GGML_TYPE_Q4_K; s[4][0] = NE; s[4][1] = NE;
        t[5] = GGML_TYPE_F32; s[5][0] = NE; s[5][1] = 1;
        t[6] = GGML_TYPE_Q4_K; s[6][0] = NE; s[6][1] = NFF;
        t[7] = GGML_TYPE_Q4_K; s[7][0] = NE; s[7][1] = NFF;
        t[8] = mb ? GGML_TYPE_Q6_K : GGML_TYPE_Q4_K; s[8][0] = NFF; s[8][1] = NE;
    }
    /* weights + caches in our buffer type (no_alloc context, ggml_backend_alloc_ctx_tensors) */
    struct ggml_init_params wp = { (size_t)(nw + 2 * n_layer + 8) * ggml_tensor_overhead(), NULL, true };
    struct ggml_context *wctx = ggml_init(wp);
    struct ggml_tensor **w = malloc(sizeof(*w) * nw), **kc = malloc(sizeof(*kc) * n_layer), **vc = malloc(sizeof(*vc) * n_layer);
    for (int i = 0; i < nw; ++i) w[i] = ggml_new_tensor_2d(wctx, (enum ggml_type)types[i], shape[i][0], shape[i][1]);
    for (int il = 0; il < n_layer; ++il) {
        kc[il] = ggml_new_tensor_1d(wctx, GGML_TYPE_F16, (int64_t)EKV * NCTX);
        vc[il] = ggml_new_tensor_1d(wctx, GGML_TYPE_F16, (int64_t)EKV * NCTX);
    }
    double t0 = now_s();
    ggml_backend_buffer_t wbuf = ggml_backend_alloc_ctx_tensors(wctx, be);
    if (!wbuf) { fprintf(stderr, "weight allocation failed\n"); return 4; }
    ggml_backend_buffer_clear(wbuf, 0);
    size_t maxb = 0;
    for (int i = 0; i < nw; ++i) if (ggml_nbytes(w[i]) > maxb) maxb = ggml_nbytes(w[i]);
    uint8_t *stage = malloc(maxb);
    for (int i = 0; i < nw; ++i) {
        const int bb = ks_block_bytes(types[i]);
        const int64_t nbl = (int64_t)(ggml_nbytes(w[i]) / bb);
        #pragma omp parallel for
        for (int64_t b = 0; b < nbl; ++b) ks_fill_block(types[i], 1234, (uint64_t)i, (uint64_t)b, stage + b * bb);
        ggml_backend_tensor_set(w[i], stage, 0, ggml_nbytes(w[i]));
    }
    free(stage);
    const double t_load = now_s() - t0;

    ggml_backend_t bes[2] = { be, cpu };
    ggml_backend_sched_t sched = ggml_backend_sched_new(bes, NULL, 2, 8192, false);
    const size_t cmem = (size_t)8192 * ggml_tensor_overhead() + ggml_graph_overhead_custom(8192, false);
    uint8_t *cbuf = malloc(cmem);
    float *logits = malloc(sizeof(float) * NV);
    int tok = 16, n_nodes = 0, n_splits = 0;
    double t_tg = 0.0, t_build = 0.0, t_alloc = 0.0, t_in = 0.0, t_comp = 0.0, t_out = 0.0;   /* per-phase host time */
    const float kq_scale = 1.0f / sqrtf((float)D);
    for (int step = -2; step < n_steps; ++step) {           /* two untimed warm-up steps */
        const int n_past = n_past0 + (step < 0 ? 0 : step);
        const double ts = now_s();
        /* llama_kv_cache: n_kv = the cells in use padded to 256 (flash attention), masked beyond n_past */
        int n_kv = (n_past + 1 + 255) / 256 * 256;
        if (n_kv > NCTX) n_kv = NCTX;
        struct ggml_init_params ip = { cmem, cbuf, true };
        struct ggml_context *ctx = ggml_init(ip);
        struct ggml_cgraph *gf = ggml_new_graph_custom(ctx, 8192, false);
        struct ggml_tensor *inp_tokens = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, 1);
        struct ggml_tensor *inp_pos = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, 1);
        struct ggml_tensor *kq_mask = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, n_kv, GGML_KQ_MASK_PAD);
        ggml_set_input(inp_tokens); ggml_set_input(inp_pos); ggml_set_input(kq_mask);
        struct ggml_tensor *inpL = ggml_get_rows(ctx, w[0], inp_tokens);
        for (int il = 0; il < n_layer; ++il) {
            struct ggml_tensor **lw = w + 3 + 9 * il;
            struct ggml_tensor *inpSA = inpL;
            struct ggml_tensor *cur = ggml_mul(ctx, ggml_rms_norm(ctx, inpL, 1e-5f), lw[0]);
            struct ggml_tensor *Qcur = ggml_mul_mat(ctx, lw[1], cur);
            struct ggml_tensor *Kcur = ggml_mul_mat(ctx, lw[2], cur);
            struct ggml_tensor *Vcur = ggml_mul_mat(ctx, lw[3], cur);
            Qcur = ggml_rope_ext(ctx, ggml_reshape_3d(ctx, Qcur, D, NH, 1), inp_pos, NULL, D, 0, NCTX, 500000.0f, 1.0f,
                                 0.0f, 1.0f, 32.0f, 1.0f);
            Kcur = ggml_rope_ext(ctx, ggml_reshape_3d(ctx, Kcur, D, NHKV, 1), inp_pos, NULL, D, 0, NCTX, 500000.0f, 1.0f,
                                 0.0f, 1.0f, 32.0f, 1.0f);
            struct ggml_tensor *kview = ggml_view_1d(ctx, kc[il], EKV, ggml_row_size(GGML_TYPE_F16, EKV) * n_past);
            struct ggml_tensor *vview = ggml_view_1d(ctx, vc[il], EKV, ggml_row_size(GGML_TYPE_F16, EKV) * n_past);
            ggml_build_forward_expand(gf, ggml_cpy(ctx, Kcur, kview));
            ggml_build_forward_expand(gf, ggml_cpy(ctx, ggml_reshape_2d(ctx, Vcur, EKV, 1), vview));
            struct ggml_tensor *q = ggml_permute(ctx, Qcur, 0, 2, 1, 3);
            struct ggml_tensor *k = ggml_view_3d(ctx, kc[il], D, n_kv, NHKV, ggml_row_size(GGML_TYPE_F16, EKV),
                                                 ggml_row_size(GGML_TYPE_F16, D), 0);
            struct ggml_tensor *v = ggml_view_3d(ctx, vc[il], D, n_kv, NHKV, ggml_row_size(GGML_TYPE_F16, EKV),
                                                 ggml_row_size(GGML_TYPE_F16, D), 0);
            cur = ggml_flash_attn_ext(ctx, q, k, v, kq_mask, kq_scale, 0.0f, 0.0f);
            ggml_flash_attn_ext_set_prec(cur, GGML_PREC_F32);
            cur = ggml_reshape_2d(ctx, cur, NE, 1);
            cur = ggml_mul_mat(ctx, lw[4], cur);
            struct ggml_tensor *ffn_inp = ggml_add(ctx, cur, inpSA);
            cur = ggml_mul(ctx, ggml_rms_norm(ctx, ffn_inp, 1e-5f), lw[5]);
            struct ggml_tensor *up = ggml_mul_mat(ctx, lw[7], cur);
            struct ggml_tensor *gate = ggml_mul_mat(ctx, lw[6], cur);
            cur = ggml_mul(ctx, ggml_silu(ctx, gate), up);
            cur = ggml_mul_mat(ctx, lw[8], cur);
            inpL = ggml_add(ctx, cur, ffn_inp);
        }
        struct ggml_tensor *out = ggml_mul_mat(ctx, w[2], ggml_mul(ctx, ggml_rms_norm(ctx, inpL, 1e-5f), w[1]));
        ggml_set_output(out);
        ggml_build_forward_expand(gf, out);
        const double t1 = now_s();
        ggml_backend_sched_reset(sched);
        if (!ggml_backend_sched_alloc_graph(sched, gf)) { fprintf(stderr, "sched alloc failed\n"); return 5; }
        const double t2 = now_s();
        const int32_t pos = n_past;
        ggml_backend_tensor_set(inp_tokens, &tok, 0, 4);
        ggml_backend_tensor_set(inp_pos, &pos, 0, 4);
        ggml_fp16_t *mask = malloc(sizeof(ggml_fp16_t) * n_kv * GGML_KQ_MASK_PAD);
        for (int r = 0; r < GGML_KQ_MASK_PAD; ++r)
            for (int j = 0; j < n_kv; ++j)
                mask[(size_t)r * n_kv + j] = ggml_fp32_to_fp16((r == 0 && j <= n_past) ? 0.0f : -INFINITY);
        ggml_backend_tensor_set(kq_mask, mask, 0, sizeof(ggml_fp16_t) * n_kv * GGML_KQ_MASK_PAD);
        free(mask);
        const double t3 = now_s();
        if (ggml_backend_sched_graph_compute(sched, gf) != GGML_STATUS_SUCCESS) { fprintf(stderr, "compute failed\n"); return 6; }
        ggml_backend_sched_synchronize(sched);
        const double t4 = now_s();
        ggml_backend_tensor_get(out, logits, 0, sizeof(float) * NV);
        int b = 0;
        for (int i = 1; i < NV; ++i) if (logits[i] > logits[b]) b = i;
        tok = b;
        n_nodes = ggml_graph_n_nodes(gf);
        n_splits = ggml_backend_sched_get_n_splits(sched);
        ggml_free(ctx);
        if (step >= 0) {
            const double t5 = now_s();
            t_tg += t5 - ts;
            t_build += t1 - ts; t_alloc += t2 - t1; t_in += t3 - t2; t_comp += t4 - t3; t_out += t5 - t4;
        }
    }
    printf("{\"b1_decode_tok_s\": %.2f, \"ms_per_token\": %.4f, \"n_layer\": %d, \"n_past\": %d, \"steps\": %d, "
           "\"graph_nodes\": %d, \"sched_splits\": %d, \"load_s\": %.1f, \"last_token\": %d, \"ms_build\": %.4f, "
           "\"ms_sched_alloc\": %.4f, \"ms_inputs\": %.4f, \"ms_compute_sync\": %.4f, \"ms_logits_argmax\": %.4f}\n",
           n_steps / t_tg, t_tg / n_steps * 1e3, n_layer, n_past0, n_steps, n_nodes, n_splits, t_load, tok,
           t_build / n_steps * 1e3, t_alloc / n_steps * 1e3, t_in / n_steps * 1e3, t_comp / n_steps * 1e3,
           t_out / n_steps * 1e3);
    ggml_backend_sched_free(sched);
    ggml_backend_buffer_free(wbuf);
    ggml_free(wctx);
    ggml_backend_free(cpu);
    ggml_backend_free(be);
    return 0;
}
