/*
 * ref_llama.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Our harness over the REFERENCE ggml library (oracle/_ref/libggml_ref.so, compiled
 * from /root/reference/ggml/src by oracle/Makefile).  It rebuilds the Llama graph
 * exactly as build_llama() does (src/llama.cpp:10453-10620, llm_build_kv/kqv
 * :9180-9634, llm_build_ffn :9289-9414) with the reference ops, on synthetic
 * weights from include/kcpp_synth.h, and runs the reference CPU backend:
 *   - golden logits / greedy tokens for tests/golden (parity pinning),
 *   - the "reference" CPU baseline timing for bench.py.
 *
 * Also exposes single-op modes used to pin the C restatement (oracle/ggml_oracle.c).
 *
 * usage: ref_llama llama <cfg.txt>      (see write_cfg in tests/refharness.py)
 *        ref_llama op <opname> <in.bin> <out.bin> [args...]
 */
#include "ggml.h"
#include "../include/kcpp_synth.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

typedef struct {
    int n_vocab, n_embd, n_head, n_head_kv, n_layer, n_ff, n_ctx;
    float eps, rope_base, rope_freq_scale;
    unsigned long long seed;
    int n_expert, n_expert_used;   /* MoE (llm_build_moe_ffn) when n_expert > 0 */
    int *types;            /* 3 + LW*n_layer, LW = 9 dense / 10 MoE (+ ffn_gate_inp) */
    int nthreads;
    int n_prompt, n_gen, ubatch;
    int *prompt;
    char out[1024];
    int n_forced;          /* optional: teacher-forced decode tokens (else the greedy argmax) */
    int *forced;
    char hidden_out[1024]; /* optional: per-layer residual stream of the prefill ubatch(es) */
} cfg_t;

static int read_cfg(const char *path, cfg_t *c) {
    FILE *f = fopen(path, "r");
    if (!f) return -1;
    int ok = fscanf(f, "%d %d %d %d %d %d %d %f %f %f %llu %d %d", &c->n_vocab, &c->n_embd, &c->n_head,
                    &c->n_head_kv, &c->n_layer, &c->n_ff, &c->n_ctx, &c->eps, &c->rope_base,
                    &c->rope_freq_scale, &c->seed, &c->n_expert, &c->n_expert_used);
    if (ok != 13) { fclose(f); return -2; }
    int nw = 3 + (c->n_expert ? 10 : 9) * c->n_layer;
    c->types = malloc(sizeof(int) * nw);
    for (int i = 0; i < nw; ++i) if (fscanf(f, "%d", &c->types[i]) != 1) { fclose(f); return -3; }
    if (fscanf(f, "%d %d %d %d", &c->nthreads, &c->n_prompt, &c->n_gen, &c->ubatch) != 4) { fclose(f); return -4; }
    c->prompt = malloc(sizeof(int) * (c->n_prompt > 0 ? c->n_prompt : 1));
    for (int i = 0; i < c->n_prompt; ++i) if (fscanf(f, "%d", &c->prompt[i]) != 1) { fclose(f); return -5; }
    if (fscanf(f, "%1023s", c->out) != 1) { fclose(f); return -6; }
    c->n_forced = 0; c->forced = NULL; c->hidden_out[0] = 0;
    if (fscanf(f, "%d", &c->n_forced) == 1 && c->n_forced > 0) {
        c->forced = malloc(sizeof(int) * c->n_forced);
        for (int i = 0; i < c->n_forced; ++i) if (fscanf(f, "%d", &c->forced[i]) != 1) { fclose(f); return -7; }
    }
    if (fscanf(f, "%1023s", c->hidden_out) != 1) c->hidden_out[0] = 0;
    fclose(f);
    return 0;
}

typedef struct {
    cfg_t c;
    struct ggml_context *wctx;
    struct ggml_tensor **w;        /* weights in the canonical order */
    struct ggml_tensor **kc, **vc; /* per-layer f16 caches [EKV * n_ctx] */
} model_t;

static void fill_tensor(struct ggml_tensor *t, int type, unsigned long long seed, int tid) {
    const int64_t nbl = ggml_nbytes(t) / ks_block_bytes(type);
    uint8_t *p = (uint8_t *)t->data;
    const int bb = ks_block_bytes(type);
    #pragma omp parallel for
    for (int64_t b = 0; b < nbl; ++b) ks_fill_block(type, seed, (uint64_t)tid, (uint64_t)b, p + b * bb);
}

/* KV cache types (koboldcpp --quantkv: gpttype_adapter.cpp:1958-1959 -> llama_kv_cache type_k / type_v):
 * env REF_KV_TYPES="tk tv" with ggml type ids (1 = F16 default, 8 = Q8_0, 2 = Q4_0) */
static int g_tk = GGML_TYPE_F16, g_tv = GGML_TYPE_F16;
/* optional rope frequency factors (env REF_ROPE_FREQS = path of D/2 f32 values): the model's rope_freqs.weight, fed
   to every rope of build_llama (src/llama.cpp:7171 create_tensor, :10269 build_rope_factors, :10490 ggml_rope_ext)
   and to the K-shift (build_k_shift) */
static float *g_rope_ff = NULL;
static int g_rope_nff = 0;
static struct ggml_tensor *rope_factors(struct ggml_context *ctx) {
    if (!g_rope_ff) return NULL;
    struct ggml_tensor *t = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, g_rope_nff);
    memcpy(t->data, g_rope_ff, sizeof(float) * g_rope_nff);
    return t;
}

static int load_model(model_t *m) {
    cfg_t *c = &m->c;
    const int E = c->n_embd, D = E / c->n_head, EKV = c->n_head_kv * D, F = c->n_ff, V = c->n_vocab;
    const int LW = c->n_expert ? 10 : 9;
    const int nw = 3 + LW * c->n_layer;
    const int NE = c->n_expert ? c->n_expert : 1;
    size_t total = 0;
    int64_t shapes[3 + 10 * 256][3];
    for (int i = 0; i < nw; ++i) shapes[i][2] = 1;
    shapes[0][0] = E; shapes[0][1] = V;
    shapes[1][0] = E; shapes[1][1] = 1;
    shapes[2][0] = E; shapes[2][1] = V;
    for (int il = 0; il < c->n_layer; ++il) {
        int64_t (*s)[3] = shapes + 3 + LW * il;
        s[0][0] = E; s[0][1] = 1;
        s[1][0] = E; s[1][1] = E;
        s[2][0] = E; s[2][1] = EKV;
        s[3][0] = E; s[3][1] = EKV;
        s[4][0] = E; s[4][1] = E;
        s[5][0] = E; s[5][1] = 1;
        s[6][0] = E; s[6][1] = F;
        s[7][0] = E; s[7][1] = F;
        s[8][0] = F; s[8][1] = E;
        if (c->n_expert) {
            s[6][2] = s[7][2] = s[8][2] = NE;          /* _exps tensors [K, N, n_expert] */
            s[9][0] = E; s[9][1] = NE; s[9][2] = 1;    /* ffn_gate_inp */
        }
    }
    for (int i = 0; i < nw; ++i)
        total += ggml_row_size((enum ggml_type)c->types[i], shapes[i][0]) * shapes[i][1] * shapes[i][2] + 256;
    total += (size_t)2 * c->n_layer * ((size_t)EKV * c->n_ctx * 2 + 256);
    total += (size_t)(nw + 2 * c->n_layer + 16) * ggml_tensor_overhead();
    struct ggml_init_params ip = { total, NULL, false };
    m->wctx = ggml_init(ip);
    if (!m->wctx) return -1;
    m->w = malloc(sizeof(*m->w) * nw);
    for (int i = 0; i < nw; ++i) {
        if (shapes[i][2] > 1) {
            /* expert e of tensor i: synthetic tid = i * 256 + e (the convention of tests/refharness.py) */
            m->w[i] = ggml_new_tensor_3d(m->wctx, (enum ggml_type)c->types[i], shapes[i][0], shapes[i][1], shapes[i][2]);
            const size_t slice = ggml_row_size((enum ggml_type)c->types[i], shapes[i][0]) * shapes[i][1];
            const int bb = ks_block_bytes(c->types[i]);
            for (int64_t e = 0; e < shapes[i][2]; ++e) {
                uint8_t *p = (uint8_t *)m->w[i]->data + e * slice;
                const int64_t nbl = slice / bb;
                #pragma omp parallel for
                for (int64_t b = 0; b < nbl; ++b) ks_fill_block(c->types[i], c->seed, (uint64_t)(i * 256 + e), (uint64_t)b, p + b * bb);
            }
        } else {
            m->w[i] = ggml_new_tensor_2d(m->wctx, (enum ggml_type)c->types[i], shapes[i][0], shapes[i][1]);
            fill_tensor(m->w[i], c->types[i], c->seed, i);
        }
    }
    m->kc = malloc(sizeof(*m->kc) * c->n_layer);
    m->vc = malloc(sizeof(*m->vc) * c->n_layer);
    for (int il = 0; il < c->n_layer; ++il) {
        m->kc[il] = ggml_new_tensor_1d(m->wctx, (enum ggml_type)g_tk, (int64_t)EKV * c->n_ctx);
        m->vc[il] = ggml_new_tensor_1d(m->wctx, (enum ggml_type)g_tv, (int64_t)EKV * c->n_ctx);
        memset(m->kc[il]->data, 0, ggml_nbytes(m->kc[il]));
        memset(m->vc[il]->data, 0, ggml_nbytes(m->vc[il]));
    }
    return 0;
}

static float *g_router = NULL;   /* MoE router logits of the hidden-dump layers (run_llama with a hidden file) */

/* one llama_decode of T tokens at n_past; returns logits of the last token.  With hid != NULL the
 * residual stream after every layer but the last ([n_layer-1][T][E]) is written there (layer outputs =
 * the next layer's input; the last layer keeps only the last token, src/llama.cpp out_ids), and with
 * g_router the MoE router logits of those layers ([n_layer-1][T][n_expert]). */
static int eval(model_t *m, const int *tokens, int T, int n_past, float *logits, float *hid) {
    cfg_t *c = &m->c;
    const int E = c->n_embd, H = c->n_head, HKV = c->n_head_kv, D = E / H, EKV = HKV * D, F = c->n_ff;
    const int n_kv = n_past + T;
    const int T_pad = GGML_PAD(T, GGML_KQ_MASK_PAD);
    size_t mem = (size_t)T * c->n_layer * ((size_t)E * 16 + (size_t)F * 4 + (size_t)EKV * 6) * sizeof(float)
               + (size_t)n_kv * T_pad * 2 + (size_t)c->n_vocab * 8 + (size_t)T * 16
               + (size_t)(c->n_layer * 64 + 64) * ggml_tensor_overhead() + ggml_graph_overhead_custom(8192, false)
               + (size_t)64 * 1024 * 1024 + (size_t)T * F * 8 + (size_t)T * E * 8
               + (c->n_expert ? (size_t)T * c->n_layer * ((size_t)F * 4 + (size_t)E * 3 + 64) * c->n_expert_used * sizeof(float)
                                + (size_t)c->n_layer * 64 * ggml_tensor_overhead() : 0);
    struct ggml_init_params ip = { mem, NULL, false };
    struct ggml_context *ctx = ggml_init(ip);
    if (!ctx) return -1;
    struct ggml_cgraph *gf = ggml_new_graph_custom(ctx, 8192, false);

    struct ggml_tensor *inp_tokens = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, T);
    memcpy(inp_tokens->data, tokens, sizeof(int) * T);
    struct ggml_tensor *inp_pos = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, T);
    for (int t = 0; t < T; ++t) ((int32_t *)inp_pos->data)[t] = n_past + t;
    struct ggml_tensor *rope_ff = rope_factors(ctx);
    struct ggml_tensor *kq_mask = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, n_kv, T_pad);
    for (int t = 0; t < T_pad; ++t)
        for (int j = 0; j < n_kv; ++j)
            ((ggml_fp16_t *)kq_mask->data)[(int64_t)t * n_kv + j] =
                ggml_fp32_to_fp16((t < T && j <= n_past + t) ? 0.0f : -INFINITY);
    struct ggml_tensor *inp_out = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, 1);
    ((int32_t *)inp_out->data)[0] = T - 1;

    const float kq_scale = 1.0f / sqrtf((float)D);
    struct ggml_tensor *inpL = ggml_get_rows(ctx, m->w[0], inp_tokens);   /* llm_build_inp_embd */
    struct ggml_tensor *lay_out[256], *rlog[256];
    for (int il = 0; il < c->n_layer; ++il) {
        struct ggml_tensor **lw = m->w + 3 + (c->n_expert ? 10 : 9) * il;
        struct ggml_tensor *inpSA = inpL;
        struct ggml_tensor *cur = ggml_mul(ctx, ggml_rms_norm(ctx, inpL, c->eps), lw[0]);
        struct ggml_tensor *Qcur = ggml_mul_mat(ctx, lw[1], cur);
        struct ggml_tensor *Kcur = ggml_mul_mat(ctx, lw[2], cur);
        struct ggml_tensor *Vcur = ggml_mul_mat(ctx, lw[3], cur);
        Qcur = ggml_rope_ext(ctx, ggml_reshape_3d(ctx, Qcur, D, H, T), inp_pos, rope_ff, D, 0, c->n_ctx,
                             c->rope_base, c->rope_freq_scale, 0.0f, 1.0f, 32.0f, 1.0f);
        Kcur = ggml_rope_ext(ctx, ggml_reshape_3d(ctx, Kcur, D, HKV, T), inp_pos, rope_ff, D, 0, c->n_ctx,
                             c->rope_base, c->rope_freq_scale, 0.0f, 1.0f, 32.0f, 1.0f);
        /* llm_build_kv_store (src/llama.cpp:9180-9202), FA => V not transposed */
        struct ggml_tensor *kview = ggml_view_1d(ctx, m->kc[il], (int64_t)T * EKV, ggml_row_size((enum ggml_type)g_tk, EKV) * n_past);
        struct ggml_tensor *vview = ggml_view_1d(ctx, m->vc[il], (int64_t)T * EKV, ggml_row_size((enum ggml_type)g_tv, EKV) * n_past);
        ggml_build_forward_expand(gf, ggml_cpy(ctx, Kcur, kview));
        ggml_build_forward_expand(gf, ggml_cpy(ctx, ggml_reshape_2d(ctx, Vcur, EKV, T), vview));
        /* llm_build_kqv, FA branch (src/llama.cpp:9517-9634) */
        struct ggml_tensor *q = ggml_permute(ctx, Qcur, 0, 2, 1, 3);
        struct ggml_tensor *k = ggml_view_3d(ctx, m->kc[il], D, n_kv, HKV, ggml_row_size((enum ggml_type)g_tk, EKV),
                                             ggml_row_size((enum ggml_type)g_tk, D), 0);
        struct ggml_tensor *v = ggml_view_3d(ctx, m->vc[il], D, n_kv, HKV, ggml_row_size((enum ggml_type)g_tv, EKV),
                                             ggml_row_size((enum ggml_type)g_tv, D), 0);
        cur = ggml_flash_attn_ext(ctx, q, k, v, kq_mask, kq_scale, 0.0f, 0.0f);
        ggml_flash_attn_ext_set_prec(cur, GGML_PREC_F32);
        cur = ggml_reshape_2d(ctx, cur, E, T);
        cur = ggml_mul_mat(ctx, lw[4], cur);
        if (il == c->n_layer - 1) {           /* skip unused tokens in the last layer */
            cur = ggml_get_rows(ctx, cur, inp_out);
            inpSA = ggml_get_rows(ctx, inpSA, inp_out);
        }
        struct ggml_tensor *ffn_inp = ggml_add(ctx, cur, inpSA);
        cur = ggml_mul(ctx, ggml_rms_norm(ctx, ffn_inp, c->eps), lw[5]);
        if (c->n_expert) {
            /* mixture of experts as llm_build_moe_ffn (src/llama.cpp:9416), llama arch: norm_w = true */
            const int NE = c->n_expert, NU = c->n_expert_used;
            const int64_t T = cur->ne[1];                  /* 1 in the last layer (out_ids) */
            struct ggml_tensor *logits = ggml_mul_mat(ctx, lw[9], cur);                 /* [NE, T] */
            rlog[il] = logits;
            if (hid && g_router && il < c->n_layer - 1) ggml_build_forward_expand(gf, logits);
            struct ggml_tensor *probs = ggml_soft_max(ctx, logits);
            struct ggml_tensor *sel = ggml_top_k(ctx, probs, NU);                        /* [NU, T] */
            struct ggml_tensor *wts = ggml_get_rows(ctx, ggml_reshape_3d(ctx, probs, 1, NE, T), sel);
            wts = ggml_reshape_2d(ctx, wts, NU, T);
            wts = ggml_div(ctx, wts, ggml_sum_rows(ctx, wts));
            wts = ggml_reshape_3d(ctx, wts, 1, NU, T);
            struct ggml_tensor *cur3 = ggml_reshape_3d(ctx, cur, E, 1, T);
            struct ggml_tensor *up = ggml_mul_mat_id(ctx, lw[7], cur3, sel);             /* [F, NU, T] */
            struct ggml_tensor *gate = ggml_mul_mat_id(ctx, lw[6], cur3, sel);
            struct ggml_tensor *par = ggml_mul(ctx, up, ggml_silu(ctx, gate));
            struct ggml_tensor *ex = ggml_mul_mat_id(ctx, lw[8], par, sel);              /* [E, NU, T] */
            ex = ggml_mul(ctx, ex, wts);
            struct ggml_tensor *moe = ggml_view_2d(ctx, ex, E, T, ex->nb[2], 0);
            for (int i = 1; i < NU; ++i) moe = ggml_add(ctx, moe, ggml_view_2d(ctx, ex, E, T, ex->nb[2], i * ex->nb[1]));
            cur = moe;
        } else {
            struct ggml_tensor *up = ggml_mul_mat(ctx, lw[7], cur);
            struct ggml_tensor *gate = ggml_mul_mat(ctx, lw[6], cur);
            cur = ggml_mul(ctx, ggml_silu(ctx, gate), up);
            cur = ggml_mul_mat(ctx, lw[8], cur);
        }
        inpL = ggml_add(ctx, cur, ffn_inp);
        lay_out[il] = inpL;
        if (hid && il < c->n_layer - 1) ggml_build_forward_expand(gf, inpL);
    }
    struct ggml_tensor *cur = ggml_mul(ctx, ggml_rms_norm(ctx, inpL, c->eps), m->w[1]);
    cur = ggml_mul_mat(ctx, m->w[2], cur);
    ggml_build_forward_expand(gf, cur);
    enum ggml_status st = ggml_graph_compute_with_ctx(ctx, gf, c->nthreads);
    if (st != GGML_STATUS_SUCCESS) { ggml_free(ctx); return -2; }
    memcpy(logits, cur->data, sizeof(float) * c->n_vocab);
    if (hid)
        for (int il = 0; il < c->n_layer - 1; ++il)
            memcpy(hid + (size_t)il * T * E, lay_out[il]->data, sizeof(float) * (size_t)T * E);
    if (hid && g_router)      /* router logits of the same layers (MoE): [n_layer-1][T][n_expert] */
        for (int il = 0; il < c->n_layer - 1; ++il)
            memcpy(g_router + (size_t)il * T * c->n_expert, rlog[il]->data, sizeof(float) * (size_t)T * c->n_expert);
    ggml_free(ctx);
    return 0;
}

/* context shift between the prompt and the decode (env REF_KSHIFT="p0 diff", koboldcpp PurgeMissingTokens,
   gpttype_adapter.cpp:1504-1571): llama_kv_cache_seq_rm(p0, p0 + diff) + seq_add(p0 + diff, n_past, -diff), then
   build_k_shift (src/llama.cpp:10144-10190): ggml_rope_ext_inplace on the F16 K cache of the moved cells with
   position -diff.  The reference leaves the moved cells where they are and masks the erased ones; here the cells
   are compacted (rows [p0 + diff, n_past) -> [p0, n_past - diff), K through the same rope op), which the
   attention sees identically up to the order it visits keys.  F16 caches only. */
static int kv_shift(model_t *m, int p0, int diff, int n_past) {
    cfg_t *c = &m->c;
    const int D = c->n_embd / c->n_head, HKV = c->n_head_kv, EKV = HKV * D, n = n_past - p0 - diff;
    if (g_tk != GGML_TYPE_F16 || g_tv != GGML_TYPE_F16 || p0 < 0 || diff <= 0 || n < 0) return -1;
    if (n == 0) return 0;
    struct ggml_init_params ip = {(size_t)n * EKV * 16 + (1 << 20), NULL, false};
    for (int il = 0; il < c->n_layer; ++il) {
        struct ggml_context *ctx = ggml_init(ip);
        struct ggml_tensor *k = ggml_new_tensor_3d(ctx, GGML_TYPE_F16, D, HKV, n);
        struct ggml_tensor *pos = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, n);
        memcpy(k->data, (const uint8_t *)m->kc[il]->data + (size_t)(p0 + diff) * EKV * 2, (size_t)n * EKV * 2);
        for (int i = 0; i < n; ++i) ((int32_t *)pos->data)[i] = -diff;
        struct ggml_tensor *r = ggml_rope_ext_inplace(ctx, k, pos, rope_factors(ctx), D, 0, c->n_ctx, c->rope_base, c->rope_freq_scale,
                                                      0.0f, 1.0f, 32.0f, 1.0f);
        struct ggml_cgraph *gf = ggml_new_graph(ctx);
        ggml_build_forward_expand(gf, r);
        if (ggml_graph_compute_with_ctx(ctx, gf, c->nthreads) != GGML_STATUS_SUCCESS) { ggml_free(ctx); return -2; }
        memcpy((uint8_t *)m->kc[il]->data + (size_t)p0 * EKV * 2, r->data, (size_t)n * EKV * 2);
        memmove((uint8_t *)m->vc[il]->data + (size_t)p0 * EKV * 2, (const uint8_t *)m->vc[il]->data + (size_t)(p0 + diff) * EKV * 2,
                (size_t)n * EKV * 2);
        ggml_free(ctx);
    }
    return 0;
}

static int argmax(const float *x, int n) {
    int b = 0;
    for (int i = 1; i < n; ++i) if (x[i] > x[b]) b = i;
    return b;
}

static int run_llama(const char *cfgpath) {
    model_t m; memset(&m, 0, sizeof(m));
    int rc = read_cfg(cfgpath, &m.c);
    if (rc) { fprintf(stderr, "bad cfg %d\n", rc); return 1; }
    double t0 = now_s();
    if (load_model(&m)) { fprintf(stderr, "load failed\n"); return 2; }
    double t_load = now_s() - t0;
    cfg_t *c = &m.c;
    FILE *out = fopen(c->out, "wb");
    if (!out) return 3;
    float *logits = malloc(sizeof(float) * c->n_vocab);
    int n_past = 0;
    /* REF_SKIP_PREFIX=n (bench.py's cpu_baseline at the GPU's context depth): the first n prompt positions are
       taken as already in the (zeroed) KV cache, not computed -- a decode step's cost depends on the cache length,
       not its contents -- so the timed work is the rest of the prompt at positions n.. and the decode after it */
    const char *skip = getenv("REF_SKIP_PREFIX");
    int p0 = skip ? atoi(skip) : 0;
    if (p0 < 0 || p0 >= c->n_prompt) p0 = 0;
    n_past = p0;
    double tp0 = now_s();
    FILE *hout = c->hidden_out[0] ? fopen(c->hidden_out, "wb") : NULL;
    float *hid = hout ? malloc(sizeof(float) * (size_t)(c->n_layer > 1 ? c->n_layer - 1 : 1) * c->ubatch * c->n_embd) : NULL;
    FILE *rout = NULL;
    if (hout && c->n_expert) {  /* MoE: the router logits beside the hidden states, <hidden_out>.router */
        char rp[1100];
        snprintf(rp, sizeof rp, "%s.router", c->hidden_out);
        rout = fopen(rp, "wb");
        g_router = malloc(sizeof(float) * (size_t)(c->n_layer > 1 ? c->n_layer - 1 : 1) * c->ubatch * c->n_expert);
    }
    for (int i = p0; i < c->n_prompt; i += c->ubatch) {
        int T = c->n_prompt - i < c->ubatch ? c->n_prompt - i : c->ubatch;
        if (eval(&m, c->prompt + i, T, n_past, logits, hid)) return 4;
        if (hout) fwrite(hid, sizeof(float), (size_t)(c->n_layer - 1) * T * c->n_embd, hout);
        if (rout) fwrite(g_router, sizeof(float), (size_t)(c->n_layer - 1) * T * c->n_expert, rout);
        n_past += T;
    }
    if (hout) { fclose(hout); free(hid); }
    if (rout) { fclose(rout); free(g_router); g_router = NULL; }
    double t_pp = now_s() - tp0;
    fwrite(logits, sizeof(float), c->n_vocab, out);
    int tok = argmax(logits, c->n_vocab);
    const char *ks = getenv("REF_KSHIFT");
    if (ks && *ks) {
        int sp0 = 0, sdiff = 0;
        if (sscanf(ks, "%d %d", &sp0, &sdiff) != 2 || kv_shift(&m, sp0, sdiff, n_past)) return 6;
        n_past -= sdiff;
    }
    double tg0 = now_s();
    for (int g = 0; g < c->n_gen; ++g) {
        if (g < c->n_forced) tok = c->forced[g];
        if (eval(&m, &tok, 1, n_past, logits, NULL)) return 5;
        n_past += 1;
        fwrite(logits, sizeof(float), c->n_vocab, out);
        tok = argmax(logits, c->n_vocab);
    }
    double t_tg = now_s() - tg0;
    fclose(out);
    printf("{\"load_s\": %.3f, \"prefill_s\": %.6f, \"decode_s\": %.6f, \"n_prompt\": %d, \"n_gen\": %d, \"threads\": %d, "
           "\"skip_prefix\": %d}\n", t_load, t_pp, t_tg, c->n_prompt, c->n_gen, c->nthreads, p0);
    return 0;
}

/* ---------------------------- single-op modes ---------------------------- */
static void *read_all(const char *p, size_t *n) {
    FILE *f = fopen(p, "rb"); if (!f) return NULL;
    fseek(f, 0, SEEK_END); *n = ftell(f); fseek(f, 0, SEEK_SET);
    void *b = malloc(*n ? *n : 1); if (fread(b, 1, *n, f) != *n) { fclose(f); free(b); return NULL; }
    fclose(f); return b;
}
static int write_all(const char *p, const void *b, size_t n) {
    FILE *f = fopen(p, "wb"); if (!f) return -1;
    fwrite(b, 1, n, f); fclose(f); return 0;
}

/* op rope <in f32 [T][H][D]> <out> D H T base freq_scale  (positions = 0..T-1 scaled by pos_mul) */
/* op rmsnorm <in f32 [R][N]> <out> N R eps */
/* op fattn <in: q f32 [T][H][D] | k f16 [n_kv][HKV][D] | v f16 | mask f16 [T][n_kv]> <out> D T H HKV n_kv */
/* op mulmat <in: W bytes | X f32 [M][K]> <out> type K N M */
static int run_op(int argc, char **argv) {
    const char *op = argv[2];
    size_t nin; uint8_t *in = read_all(argv[3], &nin);
    if (!in) return 10;
    struct ggml_init_params ip = { (size_t)1 << 30, NULL, false };
    struct ggml_context *ctx = ggml_init(ip);
    struct ggml_cgraph *gf = ggml_new_graph(ctx);
    struct ggml_tensor *res = NULL;
    if (!strcmp(op, "rope")) {
        int D = atoi(argv[5]), H = atoi(argv[6]), T = atoi(argv[7]);
        float base = atof(argv[8]), fs = atof(argv[9]); int pos_mul = atoi(argv[10]);
        struct ggml_tensor *x = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, D, H, T);
        memcpy(x->data, in, ggml_nbytes(x));
        struct ggml_tensor *pos = ggml_new_tensor_1d(ctx, GGML_TYPE_I32, T);
        for (int t = 0; t < T; ++t) ((int32_t *)pos->data)[t] = t * pos_mul;
        res = ggml_rope_ext(ctx, x, pos, NULL, D, 0, 4096, base, fs, 0.0f, 1.0f, 32.0f, 1.0f);
    } else if (!strcmp(op, "rmsnorm")) {
        int N = atoi(argv[5]), R = atoi(argv[6]); float eps = atof(argv[7]);
        struct ggml_tensor *x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, N, R);
        memcpy(x->data, in, ggml_nbytes(x));
        res = ggml_rms_norm(ctx, x, eps);
    } else if (!strcmp(op, "fattn")) {
        int D = atoi(argv[5]), T = atoi(argv[6]), H = atoi(argv[7]), HKV = atoi(argv[8]), NKV = atoi(argv[9]);
        int T_pad = GGML_PAD(T, GGML_KQ_MASK_PAD);
        struct ggml_tensor *q = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, D, H, T);
        struct ggml_tensor *k = ggml_new_tensor_3d(ctx, GGML_TYPE_F16, D, HKV, NKV);
        struct ggml_tensor *v = ggml_new_tensor_3d(ctx, GGML_TYPE_F16, D, HKV, NKV);
        struct ggml_tensor *mask = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, NKV, T_pad);
        size_t off = 0;
        memcpy(q->data, in + off, ggml_nbytes(q)); off += ggml_nbytes(q);
        memcpy(k->data, in + off, ggml_nbytes(k)); off += ggml_nbytes(k);
        memcpy(v->data, in + off, ggml_nbytes(v)); off += ggml_nbytes(v);
        memset(mask->data, 0, ggml_nbytes(mask));
        memcpy(mask->data, in + off, (size_t)T * NKV * 2);
        struct ggml_tensor *qp = ggml_permute(ctx, q, 0, 2, 1, 3);
        struct ggml_tensor *kp = ggml_permute(ctx, k, 0, 2, 1, 3);
        struct ggml_tensor *vp = ggml_permute(ctx, v, 0, 2, 1, 3);
        res = ggml_flash_attn_ext(ctx, qp, kp, vp, mask, 1.0f / sqrtf((float)D), 0.0f, 0.0f);
    } else if (!strcmp(op, "cpyq")) {            /* ggml_cpy f32 [R][N] -> type (the KV-cache store); out raw bytes */
        int type = atoi(argv[5]), N = atoi(argv[6]), R = atoi(argv[7]);
        struct ggml_tensor *x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, N, R);
        memcpy(x->data, in, ggml_nbytes(x));
        struct ggml_tensor *y = ggml_new_tensor_2d(ctx, (enum ggml_type)type, N, R);
        res = ggml_cpy(ctx, x, y);
    } else if (!strcmp(op, "fattnq")) {          /* fattn with K / V of types tk / tv ([n_kv][HKV*D] block rows) */
        int D = atoi(argv[5]), T = atoi(argv[6]), H = atoi(argv[7]), HKV = atoi(argv[8]), NKV = atoi(argv[9]);
        int tk = atoi(argv[10]), tv = atoi(argv[11]);
        int T_pad = GGML_PAD(T, GGML_KQ_MASK_PAD);
        struct ggml_tensor *q = ggml_new_tensor_3d(ctx, GGML_TYPE_F32, D, H, T);
        struct ggml_tensor *k = ggml_new_tensor_3d(ctx, (enum ggml_type)tk, D, HKV, NKV);
        struct ggml_tensor *v = ggml_new_tensor_3d(ctx, (enum ggml_type)tv, D, HKV, NKV);
        struct ggml_tensor *mask = ggml_new_tensor_2d(ctx, GGML_TYPE_F16, NKV, T_pad);
        size_t off = 0;
        memcpy(q->data, in + off, ggml_nbytes(q)); off += ggml_nbytes(q);
        memcpy(k->data, in + off, ggml_nbytes(k)); off += ggml_nbytes(k);
        memcpy(v->data, in + off, ggml_nbytes(v)); off += ggml_nbytes(v);
        memset(mask->data, 0, ggml_nbytes(mask));
        memcpy(mask->data, in + off, (size_t)T * NKV * 2);
        res = ggml_flash_attn_ext(ctx, ggml_permute(ctx, q, 0, 2, 1, 3), ggml_permute(ctx, k, 0, 2, 1, 3),
                                  ggml_permute(ctx, v, 0, 2, 1, 3), mask, 1.0f / sqrtf((float)D), 0.0f, 0.0f);
    } else if (!strcmp(op, "mulmat")) {
        int type = atoi(argv[5]), K = atoi(argv[6]), N = atoi(argv[7]), M = atoi(argv[8]);
        struct ggml_tensor *w = ggml_new_tensor_2d(ctx, (enum ggml_type)type, K, N);
        struct ggml_tensor *x = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, M);
        memcpy(w->data, in, ggml_nbytes(w));
        memcpy(x->data, in + ggml_nbytes(w), ggml_nbytes(x));
        res = ggml_mul_mat(ctx, w, x);
    } else {
        return 11;
    }
    ggml_build_forward_expand(gf, res);
    int nth = getenv("REF_THREADS") ? atoi(getenv("REF_THREADS")) : 4;
    if (ggml_graph_compute_with_ctx(ctx, gf, nth) != GGML_STATUS_SUCCESS) return 12;
    write_all(argv[4], res->data, ggml_nbytes(res));
    ggml_free(ctx);
    return 0;
}

int main(int argc, char **argv) {
    if (getenv("REF_KV_TYPES") && sscanf(getenv("REF_KV_TYPES"), "%d %d", &g_tk, &g_tv) != 2) return 2;
    if (getenv("REF_ROPE_FREQS") && getenv("REF_ROPE_FREQS")[0]) {
        size_t n;
        g_rope_ff = (float *)read_all(getenv("REF_ROPE_FREQS"), &n);
        if (!g_rope_ff || n % 4) return 2;
        g_rope_nff = (int)(n / 4);
    }
    if (argc >= 3 && !strcmp(argv[1], "llama")) return run_llama(argv[2]);
    if (argc >= 5 && !strcmp(argv[1], "op")) return run_op(argc, argv);
    fprintf(stderr, "usage: ref_llama llama <cfg> | op <name> <in> <out> args...\n");
    return 1;
}
