// runtime.cpp -- Llama forward on one MI355X (one pipeline stage of the layer split).
//
// The reference executes build_llama (src/llama.cpp:10453-10620) as a ggml graph through
// ggml_backend_sched -> ggml_backend_cuda_graph_compute (ggml-cuda.cu:2508), one kernel per
// node with host dispatch per node (CUDA graphs are compiled out on HIP, common.cuh:580-582).
// Here the same computation is a fixed, fused launch sequence per layer:
//   rms_norm*w -> Q8_K           (1 launch)
//   wq | wk | wv  mat-vec        (3 launches into one packed qkv row)
//   rope(q,k) + K/V f16 store    (1)
//   flash-attn split-KV + combine(+Q8_K quant)  (2)
//   wo mat-vec + residual add    (1)
//   rms_norm*w -> Q8_K           (1)
//   gate|up mat-vec + silu*mul   (1)
//   quantize -> down + residual  (2)
// and single-token decode is captured once into a hipGraph and replayed (n_past and the token
// id are read from device memory, so one graph serves every position).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kcpp_mi355x.h"
#include "../../include/kcpp_synth.h"
#include "kcpp_internal.h"

static thread_local std::string g_err;
extern "C" const char *kcpp_last_error(void) { return g_err.c_str(); }

#define RT_CHECK(expr)                                                                                 \
    do {                                                                                               \
        hipError_t _e = (expr);                                                                        \
        if (_e != hipSuccess) {                                                                        \
            char _b[512];                                                                              \
            snprintf(_b, sizeof _b, "HIP %s at %s:%d (%s)", hipGetErrorName(_e), __FILE__, __LINE__, #expr); \
            g_err = _b;                                                                                \
            fprintf(stderr, "[kcpp] %s\n", _b);                                                        \
            return -1;                                                                                 \
        }                                                                                              \
    } while (0)
#define RC(expr)                                                                                       \
    do {                                                                                               \
        int _r = (expr);                                                                               \
        if (_r != 0) {                                                                                 \
            char _b[512];                                                                              \
            snprintf(_b, sizeof _b, "rc=%d at %s:%d (%s)", _r, __FILE__, __LINE__, #expr);             \
            g_err = _b;                                                                                \
            fprintf(stderr, "[kcpp] %s\n", _b);                                                        \
            return _r;                                                                                 \
        }                                                                                              \
    } while (0)

// one device's rows of a row-split matrix (LLAMA_SPLIT_MODE_ROW, ggml_backend_cuda_split_buffer,
// ggml-cuda.cu:659-955): rows [lo, hi) of the [K][N] tensor, stored as a [K][hi - lo] tensor in the device layout
struct RowSlice { int lane = 0; int64_t lo = 0, hi = 0; void *d = nullptr; };

struct KTensor {
    int type = KT_F32;
    int64_t K = 0, N = 0;
    void *d = nullptr;
    size_t bytes = 0;
    bool owned = true;               // false: a slice of a fused group allocation
    int slices = 1;                  // MoE _exps tensors: n_expert consecutive [K][N] slices
    size_t slice_bytes = 0;
    std::vector<RowSlice> rs;        // non-empty: row split, the rows live in these slices (d is null)
    void *dec = nullptr;             // KT_Q8_0_T weights: a second copy in the row-major KT_Q8_0 layout for the fused
                                     // single-token chain (gemv_dec), owned
    void *pre = nullptr;             // KT_Q6_K_RS layer weights: the int8 two-plane prefill image (kcpp_q6p_build)
    bool pre_owned = false;          // false: a slice of the layer's q|k|v or gate|up image group
};

// a row-split execution lane: one device of the split.  The first lane on the stage's own device runs inline on
// its stream and buffers; every other lane (other GPUs, or further lanes on the same GPU) has its own stream,
// activation copy, output rows and GEMM workspace, fenced against the stage stream by events.
struct Lane {
    int dev = 0;
    bool inline_main = false;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    void *act = nullptr, *ws = nullptr;
    float *y = nullptr;
};

struct KLayer {
    KTensor t[10];  // attn_norm, wq, wk, wv, wo, ffn_norm, gate, up, down (, ffn_gate_inp for MoE)
    uint16_t *kc = nullptr, *vc = nullptr;
    // prefill fusion: same-type row-major (Q4_K/Q5_K) weights sharing one input are stored back to back,
    // so q|k(|v) and gate|up each run as ONE GEMM over the concatenated rows (one activation conversion,
    // 6x/2x more workgroups for the narrow k/v shapes)
    void *qkv_base = nullptr, *glu_base = nullptr;
    int nqkv = 0;                    // 2: q|k contiguous, 3: q|k|v contiguous
    bool glu_fused = false;
};

struct kcpp_model {
    kcpp_hparams hp;
    std::vector<int> types;
    int device = 0, il0 = 0, il1 = 0, has_embed = 1, has_output = 1, ub = 512;
    hipStream_t stream = nullptr;
    KTensor tok_embd, output_norm, output;
    std::vector<KLayer> layers;      // only [il0, il1)
    // workspace
    float *x = nullptr, *qkv = nullptr, *attn = nullptr, *h = nullptr, *logits = nullptr;
    float *hglu = nullptr;           // [ubatch][2 n_ff] fused gate|up GEMM output (prefill)
    uint16_t *q16 = nullptr;
    void *act = nullptr, *act2 = nullptr, *fa_ws = nullptr, *gemm_ws = nullptr;
    void *gemm_ws2 = nullptr;               // prefill: attn_v GEMM on the side stream (q|k fused layers)
    size_t act_sz = 0, gemm_ws_sz = 0;
    int32_t *tok_dev = nullptr, *pos_dev = nullptr, *argmax_dev = nullptr;   // pos_dev = {position, epoch}
    void *argmax_ws = nullptr;       // ARGMAX_BLOCKS (value, index) partials
    int32_t *moe_ids = nullptr;      // [ubatch][n_expert_used] selected experts (device)
    float *moe_w = nullptr;          // [ubatch][n_expert_used] normalized weights (device)
    int32_t *moe_rows = nullptr;     // prefill, grouped by expert: [ubatch*k] token rows ++ [ubatch*k] slot rows
    float *moe_rw = nullptr;         // [ubatch*k] routing weight of each grouped entry
    float *moe_slots = nullptr;      // [k][ubatch][n_embd] weighted expert outputs, summed in top-k order
    int32_t *moe_trace = nullptr;    // [n_layer of the stage][n_expert_used] single-token routing (diagnostics)
    bool no_fused_route = false;     // MoE decode: route in k_moe_route instead of inside the gate|up launch (A/B tests)
    int64_t n_fused_route = 0;       // routed gate|up launches enqueued (tests: the fused path really ran)
    bool no_pair_down = false;       // MoE decode: the two slots' down projections as two chained launches (A/B tests)
    int64_t n_pair_down = 0;         // two-slot down launches enqueued
    bool no_moe_grouped = false;     // MoE prefill: per-expert GEMM loop instead of the grouped launches (A/B tests)
    int64_t n_moe_grouped = 0;       // grouped MoE prefill layers run
    float *moe_gx = nullptr, *moe_gh = nullptr, *moe_gup = nullptr, *moe_geo = nullptr;   // grouped prefill: [ubatch*k]
    void *moe_gact = nullptr;        // rows (gathered input, GLU output, up scratch, down output), their Q8_K
    void *moe_gws = nullptr;         // grouped Q6_K down: fragment image of the padded layout
    int32_t *moe_gcnt = nullptr, *moe_gcnt_h = nullptr;   // per-expert row counts (device, pinned host)
    int32_t *moe_ids_h = nullptr;    // pinned host copies (prefill routing)
    float *moe_w_h = nullptr;
    int32_t *moe_rows_h = nullptr;
    float *moe_rw_h = nullptr;
    float2 *rope_tab = nullptr;
    std::vector<float> rope_ff;             // rope frequency factors (rope_freqs.weight); empty: none
    void *kv_scratch = nullptr;             // context shift: moved K/V rows (n_ctx x EKV x 2 f16, lazily)
    float *shift_cs = nullptr;              // context shift: (cos, sin) pairs of the shift distance
    int32_t *pin = nullptr;          // pinned host {token, n_past}
    hipEvent_t ev_tok[2] = {nullptr, nullptr};   // decode_greedy_lagged: token readback ring (pin[4 + k % 2])
    int lag_k = 0;                   // lagged steps enqueued since the last drain
    int pos_val = -1;                // the value pos_dev holds once the enqueued work has run (-1: unknown)
    float *logits_pin = nullptr;
    bool use_graphs = true;
    bool fused_decode = true;        // single-token path through gemv_dec (norm/rope/KV fused)
    bool q81 = false;                // Q4_1 / Q5_1 weights (Q8_1 activations): decode on the per-op path
    bool q80t = false;               // Q8_0 layer weights in the tile layout KT_Q8_0_T (gemm_q80t.hip) at every batch size
    bool no_dual_qkv = false;        // KCPP_DUAL_QKV=0: q (RS) and k|v (Q8_0) as two launches (A/B)
    bool no_norm_fold = false;       // KCPP_NORM_FOLD=0: the residual GEMMs never carry the next rms_norm (A/B)
    bool q80_dec = false;            // ... plus their KT_Q8_0 decode copies (KTensor::dec): single tokens on the fused chain
    bool fa_exact = false;           // attention in the reference CPU's order with f16 accumulation (attn_exact.hip)
    int kv_tk = KT_F16, kv_tv = KT_F16;   // cache types (--quantkv: Q8_0 / Q4_0, attn_kvq.hip)
    hipGraphExec_t g_exec[2] = {nullptr, nullptr};   // single-token graph per attention regime (dec_short)
    // layer-split engine: the single-token graph bracketed by the stage hand-off kernels (link.hip), captured lazily
    KLink link{};
    bool has_link = false;
    hipGraphExec_t g_link[2] = {nullptr, nullptr};
    // single-token attention regime: contexts up to short_max keys take the one-launch kernel (kcpp_flash_attn
    // force_path 7, no combine); chosen per step from the host-known position, each regime its own graph
    bool dec_short = false;
    int short_max = 0;
    hipStream_t side = nullptr;             // second branch of the decode step (independent q|k|v launches)
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int64_t weight_bytes = 0;
    std::vector<Lane> lanes;                // row split (kcpp_model_set_row_split); empty: every matrix whole here
    hipEvent_t ev_in = nullptr;             // row split: the stage stream has produced a mat-mul's inputs
};

static int ensure_graph(kcpp_model *m);
static void drop_graphs(kcpp_model *m) {
    for (int r = 0; r < 2; ++r) {
        if (m->g_exec[r]) { (void)hipGraphExecDestroy(m->g_exec[r]); m->g_exec[r] = nullptr; }
        if (m->g_link[r]) { (void)hipGraphExecDestroy(m->g_link[r]); m->g_link[r] = nullptr; }
    }
}
static int launch_argmax(kcpp_model *m, bool step_pos);
static int launch_pos_step(kcpp_model *m);

static int64_t tensor_bytes(int type, int64_t K, int64_t N) {
    return K / ks_block_elems(type) * N * ks_block_bytes(type);
}

static int per_layer(const kcpp_hparams &hp) { return hp.n_expert > 0 ? 10 : 9; }
static int n_tensors(const kcpp_hparams &hp) { return 3 + per_layer(hp) * hp.n_layer; }
static int n_slices(const kcpp_hparams &hp, int idx) {
    if (idx < 3 || hp.n_expert <= 0) return 1;
    const int j = (idx - 3) % 10;
    return (j >= 6 && j <= 8) ? hp.n_expert : 1;
}

static void shape_of(const kcpp_hparams &hp, int idx, int64_t &K, int64_t &N) {
    const int64_t E = hp.n_embd, F = hp.n_ff, V = hp.n_vocab, EKV = (int64_t)hp.n_head_kv * (E / hp.n_head);
    if (idx == 0) { K = E; N = V; return; }
    if (idx == 1) { K = E; N = 1; return; }
    if (idx == 2) { K = E; N = V; return; }
    switch ((idx - 3) % per_layer(hp)) {
    case 0: K = E; N = 1; return;
    case 1: K = E; N = E; return;
    case 2: K = E; N = EKV; return;
    case 3: K = E; N = EKV; return;
    case 4: K = E; N = E; return;
    case 5: K = E; N = 1; return;
    case 6: K = E; N = F; return;
    case 7: K = E; N = F; return;
    case 8: K = F; N = E; return;
    default: K = E; N = hp.n_expert; return;    // ffn_gate_inp (router)
    }
}

static KTensor *tensor_at(kcpp_model *m, int idx) {
    if (idx == 0) return m->has_embed ? &m->tok_embd : nullptr;
    if (idx == 1) return m->has_output ? &m->output_norm : nullptr;
    if (idx == 2) return m->has_output ? &m->output : nullptr;
    const int LW = per_layer(m->hp);
    const int il = (idx - 3) / LW, j = (idx - 3) % LW;
    if (il < m->il0 || il >= m->il1) return nullptr;
    return &m->layers[il - m->il0].t[j];
}

static int alloc_tensor(kcpp_model *m, KTensor &t, int type, int64_t K, int64_t N, int slices = 1) {
    t.type = type; t.K = K; t.N = N;
    t.slices = slices;
    t.slice_bytes = (size_t)tensor_bytes(type, K, N);
    t.bytes = t.slice_bytes * slices;
    RT_CHECK(hipMalloc(&t.d, (t.bytes + 255) & ~(size_t)255));
    m->weight_bytes += t.bytes;
    return 0;
}

// one position's (cos, sin) pairs: ggml_rope_cache_init + rope_yarn (ggml.c:14216-14260); p may be negative
// (a K-shift distance), n_dims == head dim for Llama
static void rope_row(float *row, float p, int n_dims, float freq_base, float freq_scale, const float *freq_factors,
                     float ext_factor, float attn_factor, float beta_fast, float beta_slow, int n_ctx_orig) {
    const float theta_scale = powf(freq_base, -2.0f / n_dims);
    auto corr_dim = [&](float n_rot) { return n_dims * logf(n_ctx_orig / (n_rot * 2 * (float)M_PI)) / (2 * logf(freq_base)); };
    float corr0 = fmaxf(0, floorf(corr_dim(beta_fast))), corr1 = fminf(n_dims - 1, ceilf(corr_dim(beta_slow)));
    float theta = p;
    for (int i0 = 0; i0 < n_dims; i0 += 2) {
        const float ff = freq_factors ? freq_factors[i0 / 2] : 1.0f;
        const float theta_extrap = theta / ff;
        const float theta_interp = freq_scale * theta_extrap;
        float th = theta_interp, mscale = attn_factor;
        if (ext_factor != 0.0f) {
            const float y = (i0 / 2 - corr0) / fmaxf(0.001f, corr1 - corr0);
            const float ramp_mix = (1 - fminf(1, fmaxf(0, y))) * ext_factor;
            th = theta_interp * (1 - ramp_mix) + theta_extrap * ramp_mix;
            mscale *= 1.0f + 0.1f * logf(1.0f / freq_scale);
        }
        row[i0 + 0] = cosf(th) * mscale;
        row[i0 + 1] = sinf(th) * mscale;
        theta *= theta_scale;
    }
}

extern "C" int kcpp_rope_table(float *tab, int n_pos, int n_dims, float freq_base, float freq_scale,
                               const float *freq_factors, float ext_factor, float attn_factor, float beta_fast,
                               float beta_slow, int n_ctx_orig) {
    for (int p = 0; p < n_pos; ++p)
        rope_row(tab + (int64_t)p * n_dims, (float)p, n_dims, freq_base, freq_scale, freq_factors, ext_factor, attn_factor,
                 beta_fast, beta_slow, n_ctx_orig);
    return 0;
}

extern "C" int kcpp_rope_row(float *row, int p, int n_dims, float freq_base, float freq_scale, float ext_factor,
                             float attn_factor, float beta_fast, float beta_slow, int n_ctx_orig) {
    rope_row(row, (float)p, n_dims, freq_base, freq_scale, nullptr, ext_factor, attn_factor, beta_fast, beta_slow, n_ctx_orig);
    return 0;
}

// Context shift (koboldcpp PurgeMissingTokens: llama_kv_cache_seq_rm(p0, p0 + diff) +
// llama_kv_cache_seq_add(p0 + diff, n_past, -diff), then the K-shift of build_k_shift on the next decode):
// cache rows [p0 + diff, n_past) move to [p0, n_past - diff), K re-rotated by position -diff.  The caches are
// position-indexed here, so the rows move (through a scratch copy) instead of the cells being relabelled.
extern "C" int kcpp_model_kv_shift(kcpp_model *m, int p0, int diff, int n_past) {
    if (!m || p0 < 0 || diff <= 0 || p0 + diff > n_past || n_past > m->hp.n_ctx) { g_err = "kv_shift: bad range"; return -1; }
    if (m->kv_tk != KT_F16) { g_err = "kv_shift: quantized KV cache (context shift is off with --quantkv)"; return -1; }
    hipSetDevice(m->device);
    const int64_t E = m->hp.n_embd, H = m->hp.n_head, HKV = m->hp.n_head_kv, D = E / H, EKV = HKV * D;
    const int64_t count = n_past - p0 - diff;
    if (count == 0) return 0;
    if (!m->kv_scratch && hipMalloc(&m->kv_scratch, (size_t)m->hp.n_ctx * EKV * 2 * 2) != hipSuccess) {
        g_err = "kv_shift scratch";
        return -2;
    }
    if (!m->shift_cs && hipMalloc(&m->shift_cs, (size_t)D * 4) != hipSuccess) { g_err = "kv_shift cs"; return -2; }
    std::vector<float> row((size_t)D);
    rope_row(row.data(), (float)-diff, (int)D, m->hp.rope_base, m->hp.rope_freq_scale,
             m->rope_ff.empty() ? nullptr : m->rope_ff.data(), 0.0f, 1.0f, 32.0f, 1.0f, m->hp.n_ctx);
    RT_CHECK(hipMemcpyAsync(m->shift_cs, row.data(), (size_t)D * 4, hipMemcpyHostToDevice, m->stream));
    uint16_t *ks = (uint16_t *)m->kv_scratch, *vs = ks + (size_t)m->hp.n_ctx * EKV;
    for (auto &L : m->layers) {
        RC(kcpp_kv_shift_rows(L.kc + (p0 + diff) * EKV, L.vc + (p0 + diff) * EKV, ks, vs, count * HKV, (int)D, m->shift_cs,
                              m->stream));
        RT_CHECK(hipMemcpyAsync(L.kc + p0 * EKV, ks, (size_t)count * EKV * 2, hipMemcpyDeviceToDevice, m->stream));
        RT_CHECK(hipMemcpyAsync(L.vc + p0 * EKV, vs, (size_t)count * EKV * 2, hipMemcpyDeviceToDevice, m->stream));
    }
    RT_CHECK(hipStreamSynchronize(m->stream));     // the host row above must outlive its copy
    return 0;
}

extern "C" int kcpp_model_set_rope_freqs(kcpp_model *m, const float *ff, int n) {
    const int64_t D = m->hp.n_embd / m->hp.n_head;
    if (!ff || n != D / 2) { g_err = "rope_freqs: need head_dim / 2 values"; return -1; }
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    m->rope_ff.assign(ff, ff + n);
    std::vector<float> tab((size_t)m->hp.n_ctx * D);
    kcpp_rope_table(tab.data(), m->hp.n_ctx, (int)D, m->hp.rope_base, m->hp.rope_freq_scale, m->rope_ff.data(), 0.0f, 1.0f,
                    32.0f, 1.0f, m->hp.n_ctx);
    RT_CHECK(hipMemcpy(m->rope_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    return 0;
}

extern "C" kcpp_model *kcpp_model_create(const kcpp_hparams *hp, const int *types, int device, int il0, int il1,
                                         int has_embed, int has_output, int max_ubatch) {
    if (hipSetDevice(device) != hipSuccess) { g_err = "hipSetDevice failed"; return nullptr; }
    // the split-KV decode attention merges at most 2048 chunks of 64 keys (attn.hip FA_MAX_CHUNKS)
    if (hp->n_ctx < 1 || hp->n_ctx > 131072) { g_err = "n_ctx must be in [1, 131072]"; return nullptr; }
    kcpp_model *m = new kcpp_model();
    m->hp = *hp;
    // on-device layout per tensor: dense Q4_K / Q5_K / Q6_K mat-mul weights whose K the RS kernels cover are held in
    // the row-major decode layouts (KT_Q4_K_RS / KT_Q5_K_RS / KT_Q6_K_RS, gemv_rs.hip), expert slices too (each slice
    // its own RS tensor: the RS kernels take the device-resident expert index, the GEMMs read RS planes); the token
    // embedding (row gathers), the router and everything else keep the kcpp layout.
    m->types.resize(n_tensors(*hp));
    for (int idx = 0; idx < n_tensors(*hp); ++idx) {
        int t = types[idx];
        int64_t K, N;
        shape_of(*hp, idx, K, N);
        const bool dense = idx >= 2 && N > 1 && (idx == 2 || (idx - 3) % per_layer(*hp) <= 8);
        if (dense && (t == KT_Q4_K || t == KT_Q5_K || t == KT_Q6_K) && kcpp_rs_supported(t, K))
            t = t == KT_Q4_K ? KT_Q4_K_RS : (t == KT_Q5_K ? KT_Q5_K_RS : KT_Q6_K_RS);
        m->types[idx] = t;
    }
    // an all-Q8_0 dense model (BASELINE config 3) holds its layer matrices (and a Q8_0 output head) in the tile layout
    // KT_Q8_0_T: one int8 MFMA kernel at every batch size, 1 KiB-contiguous weight fragments (gemm_q80t.hip)
    if (hp->n_expert == 0 && hp->n_layer > 0) {
        bool all = true;
        for (int il = 0; il < hp->n_layer && all; ++il)
            for (int j : {1, 2, 3, 4, 6, 7, 8}) {
                const int idx = 3 + per_layer(*hp) * il + j;
                int64_t K, N;
                shape_of(*hp, idx, K, N);
                all = all && m->types[idx] == KT_Q8_0 && K % 128 == 0 && N % 32 == 0;
            }
        if (all) {
            for (int il = 0; il < hp->n_layer; ++il)
                for (int j : {1, 2, 3, 4, 6, 7, 8}) m->types[3 + per_layer(*hp) * il + j] = KT_Q8_0_T;
            int64_t K, N;
            shape_of(*hp, 2, K, N);
            if (m->types[2] == KT_Q8_0 && K % 128 == 0 && N % 32 == 0) m->types[2] = KT_Q8_0_T;
            m->q80t = true;
        }
    }
    types = m->types.data();
    for (int idx = 0; idx < n_tensors(*hp); ++idx)
        m->q81 |= types[idx] == KT_Q4_1 || types[idx] == KT_Q5_1;

    m->device = device; m->il0 = il0; m->il1 = il1; m->has_embed = has_embed; m->has_output = has_output;
    m->ub = max_ubatch > 0 ? max_ubatch : 512;
    m->fa_exact = getenv("KCPP_FA_EXACT") && atoi(getenv("KCPP_FA_EXACT")) != 0;
    auto fail = [&](const char *what) { g_err = what; kcpp_model_free(m); return (kcpp_model *)nullptr; };
    if (hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    if (hipStreamCreateWithFlags(&m->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_join, hipEventDisableTiming) != hipSuccess)
        return fail("side stream");
    const int64_t E = hp->n_embd, F = hp->n_ff, H = hp->n_head, HKV = hp->n_head_kv, D = E / H, EKV = HKV * D;
    const int64_t UB = m->ub;
    m->layers.resize(il1 - il0);
    auto rowmajor = [](int t) { return t == KT_Q4_K || t == KT_Q5_K || t == KT_Q4_K_RS || t == KT_Q5_K_RS || t == KT_Q6_K_RS; };
    auto alloc_group = [&](void *&base, int idx0, int n) -> int {
        size_t tot = 0;
        for (int j = 0; j < n; ++j) { int64_t K, N; shape_of(*hp, idx0 + j, K, N); tot += (size_t)tensor_bytes(types[idx0 + j], K, N); }
        if (hipMalloc(&base, (tot + 255) & ~(size_t)255) != hipSuccess) return -1;
        size_t off = 0;
        for (int j = 0; j < n; ++j) {
            KTensor &t = *tensor_at(m, idx0 + j);
            int64_t K, N; shape_of(*hp, idx0 + j, K, N);
            t.type = types[idx0 + j]; t.K = K; t.N = N; t.bytes = (size_t)tensor_bytes(t.type, K, N);
            t.d = (uint8_t *)base + off; t.owned = false;
            off += t.bytes;
            m->weight_bytes += t.bytes;
        }
        return 0;
    };
    for (int il = il0; il < il1; ++il) {
        KLayer &L = m->layers[il - il0];
        const int b = 3 + per_layer(*hp) * il;
        if (rowmajor(types[b + 1]) && types[b + 2] == types[b + 1]) {
            L.nqkv = types[b + 3] == types[b + 1] ? 3 : 2;
            if (alloc_group(L.qkv_base, b + 1, L.nqkv)) return fail("qkv alloc");
        }
        if (hp->n_expert <= 0 && rowmajor(types[b + 6]) && types[b + 7] == types[b + 6]) {
            L.glu_fused = true;
            if (alloc_group(L.glu_base, b + 6, 2)) return fail("glu alloc");
        }
    }
    for (int idx = 0; idx < n_tensors(*hp); ++idx) {
        KTensor *t = tensor_at(m, idx);
        if (!t || t->d) continue;
        int64_t K, N;
        shape_of(*hp, idx, K, N);
        if (alloc_tensor(m, *t, types[idx], K, N, n_slices(*hp, idx))) return fail("weight alloc");
    }
    for (auto &L : m->layers) {
        const size_t kvb = (size_t)hp->n_ctx * EKV * 2;
        if (hipMalloc(&L.kc, kvb) != hipSuccess || hipMalloc(&L.vc, kvb) != hipSuccess) return fail("kv alloc");
        hipMemset(L.kc, 0, kvb); hipMemset(L.vc, 0, kvb);
    }
    // activation buffers sized for the widest vec_dot input (K = F) at UB columns
    m->act_sz = (size_t)std::max({kcpp_act_bytes(KT_Q4_K, std::max(E, F), UB), kcpp_act_bytes(KT_Q8_0, std::max(E, F), UB),
                                  kcpp_act_bytes(KT_Q4_1, std::max(E, F), UB), kcpp_act_bytes(KT_Q8_0_T, std::max(E, F), UB)});
    m->gemm_ws_sz = 0;
    for (int idx = 0; idx < n_tensors(*hp); ++idx) {
        int64_t K, N; shape_of(*hp, idx, K, N);
        if (types[idx] == KT_F32 || types[idx] == KT_F16) continue;
        m->gemm_ws_sz = std::max<size_t>(m->gemm_ws_sz, (size_t)kcpp_gemm_workspace_bytes(types[idx], K, N, UB));
        // fused shapes (q|k|v: N = E + 2 EKV; gate|up: N = 2 F)
        m->gemm_ws_sz = std::max<size_t>(m->gemm_ws_sz, (size_t)kcpp_gemm_workspace_bytes(types[idx], E, E + 2 * EKV, UB));
        m->gemm_ws_sz = std::max<size_t>(m->gemm_ws_sz, (size_t)kcpp_gemm_workspace_bytes(types[idx], E, 2 * F, UB));
    }
    bool ok = hipMalloc(&m->x, UB * E * 4) == hipSuccess && hipMalloc(&m->qkv, UB * (E + 2 * EKV) * 4) == hipSuccess &&
              hipMalloc(&m->attn, UB * E * 4) == hipSuccess && hipMalloc(&m->h, UB * F * 4) == hipSuccess &&
              hipMalloc(&m->hglu, UB * 2 * F * 4) == hipSuccess &&
              hipMalloc(&m->q16, UB * E * 2) == hipSuccess && hipMalloc(&m->act, m->act_sz) == hipSuccess &&
              hipMalloc(&m->act2, m->act_sz) == hipSuccess &&
              hipMalloc(&m->fa_ws, kcpp_fa_workspace_bytes(std::max<int>(16, 1), H, hp->n_ctx)) == hipSuccess &&
              hipMalloc(&m->tok_dev, UB * 4) == hipSuccess && hipMalloc(&m->pos_dev, 64) == hipSuccess &&
              hipMalloc(&m->argmax_dev, 64) == hipSuccess && hipMalloc(&m->argmax_ws, 256 * 8) == hipSuccess &&
              hipMalloc(&m->rope_tab, (size_t)hp->n_ctx * D / 2 * sizeof(float2)) == hipSuccess &&
              hipHostMalloc((void **)&m->pin, 64, hipHostMallocDefault) == hipSuccess &&
              (m->gemm_ws_sz == 0 || hipMalloc(&m->gemm_ws, m->gemm_ws_sz) == hipSuccess);
    if (!ok) return fail("workspace alloc");
    // the KT_Q8_0_T GEMM's split-K tickets live in the workspace and must start at zero (each launch leaves them zero)
    if (m->gemm_ws && hipMemset(m->gemm_ws, 0, m->gemm_ws_sz) != hipSuccess) return fail("gemm ws memset");
    // all-Q8_0 models: the tile layout serves every batch size, and single-token steps run the fused row-major chain
    // (norm / RoPE / K-V / residual / GLU fused into the mat-vecs) on a second copy in the KT_Q8_0 layout -- 398 vs 372
    // tok/s on Llama-3-8B Q8_0 for 7.4 GB more HBM (the layer matrices and the head stored twice; KCPP_Q80_DEC=0:
    // one copy, single tokens on the tile GEMM)
    if (m->q80t && !(getenv("KCPP_Q80_DEC") && atoi(getenv("KCPP_Q80_DEC")) == 0)) {
        bool ok2 = true;
        for (int idx = 2; idx < n_tensors(*hp) && ok2; ++idx) {
            KTensor *t = tensor_at(m, idx);
            if (!t || t->type != KT_Q8_0_T || t->slices != 1) continue;
            ok2 = hipMalloc(&t->dec, (size_t)tensor_bytes(KT_Q8_0, t->K, t->N)) == hipSuccess;
        }
        if (!ok2) {                               // not enough memory for the copies: one copy, tile GEMM decode
            for (int idx = 2; idx < n_tensors(*hp); ++idx) {
                KTensor *t = tensor_at(m, idx);
                if (t && t->dec) { hipFree(t->dec); t->dec = nullptr; }
            }
            (void)hipGetLastError();
        }
        m->q80_dec = ok2;
    }
    // Q6_K layer matrices: the int8 prefill image beside the RS weights (k_gemm_q6p: int8 matrix cores, q6v3's bits;
    // 2 B per weight more, e.g. +1.9 GB on Llama-3-8B Q4_K_M).  Fused q|k|v / gate|up groups get one image each, so
    // the group's GEMM reads one contiguous image.  KCPP_Q6P=0: no images (q6v3).
    m->no_norm_fold = getenv("KCPP_NORM_FOLD") && atoi(getenv("KCPP_NORM_FOLD")) == 0;
    m->no_dual_qkv = getenv("KCPP_DUAL_QKV") && atoi(getenv("KCPP_DUAL_QKV")) == 0;
    m->short_max = getenv("KCPP_FA_SHORT") ? atoi(getenv("KCPP_FA_SHORT")) : KCPP_FA_SHORT_MAX;
    if (!(getenv("KCPP_Q6P") && atoi(getenv("KCPP_Q6P")) == 0)) {
        bool ok3 = true;
        auto img_group = [&](KTensor *ts, const int *js, int n) {
            size_t tot = 0;
            for (int i = 0; i < n; ++i) {
                const KTensor &t = ts[js[i]];
                if (t.type != KT_Q6_K_RS || t.slices != 1 || !t.d || !kcpp_q6p_image_bytes(t.K, t.N)) return;
                tot += (size_t)kcpp_q6p_image_bytes(t.K, t.N);
            }
            void *base = nullptr;
            if (hipMalloc(&base, tot) != hipSuccess) { ok3 = false; return; }
            size_t off = 0;
            for (int i = 0; i < n; ++i) {
                KTensor &t = ts[js[i]];
                t.pre = (uint8_t *)base + off; t.pre_owned = i == 0;
                off += (size_t)kcpp_q6p_image_bytes(t.K, t.N);
            }
        };
        for (auto &L : m->layers) {
            static const int qkv[3] = {1, 2, 3}, glu[2] = {6, 7};
            if (L.nqkv >= 2) img_group(L.t, qkv, L.nqkv);
            if (L.glu_fused) img_group(L.t, glu, 2);
            for (int j = 1; j <= 8 && ok3; ++j) {
                if (j == 5 || L.t[j].pre) continue;
                const int one[1] = {j};
                img_group(L.t, one, 1);
            }
        }
        if (!ok3) {                               // not enough memory: no images anywhere
            for (auto &L : m->layers)
                for (auto &t : L.t) {
                    if (t.pre && t.pre_owned) hipFree(t.pre);
                    t.pre = nullptr; t.pre_owned = false;
                }
            (void)hipGetLastError();
        }
    }
    if (hp->n_expert > 0) {
        const int NU = hp->n_expert_used;
        if (NU < 1 || NU > hp->n_expert || hp->n_expert > 64) return fail("bad n_expert / n_expert_used");
        if (hipMalloc(&m->moe_ids, UB * NU * 4) != hipSuccess || hipMalloc(&m->moe_w, UB * NU * 4) != hipSuccess ||
            hipMalloc(&m->moe_rows, 2 * UB * NU * 4) != hipSuccess || hipMalloc(&m->moe_rw, UB * NU * 4) != hipSuccess ||
            hipMalloc(&m->moe_slots, NU * UB * E * 4) != hipSuccess ||
            hipHostMalloc((void **)&m->moe_ids_h, UB * NU * 4, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&m->moe_w_h, UB * NU * 4, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&m->moe_rows_h, 2 * UB * NU * 4, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void **)&m->moe_rw_h, UB * NU * 4, hipHostMallocDefault) != hipSuccess)
            return fail("moe workspace alloc");
    }
    // flash-attention tickets must start at zero (the merging workgroup resets its own)
    if (hipMemset(m->fa_ws, 0, kcpp_fa_workspace_bytes(16, H, hp->n_ctx)) != hipSuccess) return fail("fa ws memset");
    {   // pos_dev = {position, step counter}
        const int32_t pe[2] = {0, 1};
        if (hipMemcpy(m->pos_dev, pe, 8, hipMemcpyHostToDevice) != hipSuccess) return fail("pos");
    }
    if (has_output) {
        if (hipMalloc(&m->logits, (size_t)hp->n_vocab * 4) != hipSuccess) return fail("logits alloc");
        if (hipHostMalloc((void **)&m->logits_pin, (size_t)hp->n_vocab * 4, hipHostMallocDefault) != hipSuccess)
            return fail("logits pin");
    }
    std::vector<float> tab((size_t)hp->n_ctx * D);
    kcpp_rope_table(tab.data(), hp->n_ctx, (int)D, hp->rope_base, hp->rope_freq_scale, nullptr, 0.0f, 1.0f, 32.0f, 1.0f,
                    hp->n_ctx);
    if (hipMemcpy(m->rope_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return fail("rope tab");
    return m;
}

extern "C" void kcpp_model_free(kcpp_model *m) {
    if (!m) return;
    hipSetDevice(m->device);
    drop_graphs(m);
    auto F = [](void *p) { if (p) hipFree(p); };
    F(m->moe_trace);
    auto FS = [&](KTensor &t) {
        for (auto &r : t.rs) { hipSetDevice(m->lanes[r.lane].dev); F(r.d); }
        hipSetDevice(m->device);
    };
    F(m->tok_embd.d); F(m->output_norm.d); F(m->output.d); FS(m->output); F(m->output.dec);
    for (auto &L : m->layers) {
        for (auto &t : L.t) { if (t.owned) F(t.d); FS(t); F(t.dec); if (t.pre_owned) F(t.pre); }
        F(L.qkv_base); F(L.glu_base); F(L.kc); F(L.vc);
    }
    F(m->hglu); F(m->moe_ids); F(m->moe_w); F(m->moe_rows); F(m->moe_rw); F(m->moe_slots);
    F(m->moe_gx); F(m->moe_gh); F(m->moe_gup); F(m->moe_geo); F(m->moe_gact); F(m->moe_gcnt); F(m->moe_gws);
    for (void *p : {(void *)m->moe_ids_h, (void *)m->moe_w_h, (void *)m->moe_rows_h, (void *)m->moe_rw_h,
                    (void *)m->moe_gcnt_h})
        if (p) hipHostFree(p);
    F(m->x); F(m->qkv); F(m->attn); F(m->h); F(m->logits); F(m->q16); F(m->act); F(m->act2); F(m->fa_ws);
    F(m->gemm_ws); F(m->gemm_ws2); F(m->tok_dev); F(m->pos_dev); F(m->argmax_dev); F(m->argmax_ws); F(m->rope_tab);
    F(m->kv_scratch); F(m->shift_cs);
    if (m->pin) hipHostFree(m->pin);
    for (hipEvent_t &ev : m->ev_tok) if (ev) hipEventDestroy(ev);
    if (m->logits_pin) hipHostFree(m->logits_pin);
    if (m->stream) hipStreamDestroy(m->stream);
    if (m->side) hipStreamDestroy(m->side);
    if (m->ev_fork) hipEventDestroy(m->ev_fork);
    if (m->ev_join) hipEventDestroy(m->ev_join);
    if (m->ev_in) hipEventDestroy(m->ev_in);
    for (auto &ln : m->lanes) {
        if (ln.inline_main) continue;
        hipSetDevice(ln.dev);
        F(ln.act); F(ln.ws); F(ln.y);
        if (ln.s) hipStreamDestroy(ln.s);
        if (ln.done) hipEventDestroy(ln.done);
    }
    hipSetDevice(m->device);
    delete m;
}

extern "C" int kcpp_model_synth_weights(kcpp_model *m, uint64_t seed) {
    RT_CHECK(hipSetDevice(m->device));
    for (int idx = 0; idx < n_tensors(m->hp); ++idx) {
        KTensor *t = tensor_at(m, idx);
        if (!t) continue;
        if (!t->rs.empty()) {                  // row split: each slice holds its rows of the same tensor
            for (const RowSlice &r : t->rs) {
                const Lane &ln = m->lanes[r.lane];
                RT_CHECK(hipSetDevice(ln.dev));
                RC(kcpp_weight_synth_rows(t->type, seed, (uint64_t)idx, r.d, t->K, r.hi - r.lo, r.lo,
                                          ln.inline_main ? m->stream : ln.s));
                RT_CHECK(hipStreamSynchronize(ln.inline_main ? m->stream : ln.s));
            }
            RT_CHECK(hipSetDevice(m->device));
        } else if (t->slices == 1) {
            RC(kcpp_weight_synth(t->type, seed, (uint64_t)idx, t->d, t->K, t->N, m->stream));
            if (t->dec) RC(kcpp_weight_synth(KT_Q8_0, seed, (uint64_t)idx, t->dec, t->K, t->N, m->stream));
            if (t->pre) RC(kcpp_q6p_build(t->d, t->K, t->N, t->pre, m->stream));
        } else {                               // expert e: tid = idx * 256 + e (tests/refharness.py)
            for (int e = 0; e < t->slices; ++e)
                RC(kcpp_weight_synth(t->type, seed, (uint64_t)idx * 256 + e, (uint8_t *)t->d + e * t->slice_bytes, t->K,
                                     t->N, m->stream));
        }
    }
    RT_CHECK(hipStreamSynchronize(m->stream));
    return 0;
}

// host GGUF bytes of `slices` [K][N] tensors -> device layout at dst on device dev
static int upload(int dev, hipStream_t s, int type, int64_t K, int64_t N, int slices, size_t slice_bytes,
                  const void *src, void *dst) {
    const size_t bytes = (size_t)tensor_bytes(type, K, N) * slices;
    if (!slice_bytes) slice_bytes = bytes;
    if (bytes == 0) return 0;
    RT_CHECK(hipSetDevice(dev));
    if (type == KT_Q6_K || type == KT_Q3_K || type == KT_Q2_K || type == KT_Q4_0 || type == KT_Q4_1 || type == KT_Q5_0 || type == KT_Q5_1 || type == KT_Q8_0 ||
        type == KT_IQ4_NL || type == KT_IQ4_XS ||
        type == KT_Q4_K_RS || type == KT_Q5_K_RS ||
        type == KT_Q6_K_RS || type == KT_Q8_0_T) {
        void *stage = nullptr;
        RT_CHECK(hipMalloc(&stage, bytes));
        RT_CHECK(hipMemcpyAsync(stage, src, bytes, hipMemcpyHostToDevice, s));
        for (int e = 0; e < slices; ++e)         // structure-of-arrays layout per expert slice
            RC(kcpp_weight_repack(type, (uint8_t *)stage + e * slice_bytes, (uint8_t *)dst + e * slice_bytes, K, N, 0, s));
        RT_CHECK(hipStreamSynchronize(s));
        RT_CHECK(hipFree(stage));
    } else {
        RT_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
        RT_CHECK(hipStreamSynchronize(s));
    }
    return 0;
}

extern "C" int kcpp_model_set_tensor(kcpp_model *m, int idx, const void *src, int64_t nbytes) {
    KTensor *t = tensor_at(m, idx);
    if (!t) return 0;                      // not on this stage
    if ((size_t)nbytes != t->bytes) { g_err = "set_tensor: size mismatch"; return -2; }
    if (!t->rs.empty()) {                  // row split: GGUF rows are contiguous, each slice uploads its own
        const size_t row_bytes = (size_t)tensor_bytes(t->type, t->K, 1);
        for (const RowSlice &r : t->rs) {
            const Lane &ln = m->lanes[r.lane];
            RC(upload(ln.dev, ln.inline_main ? m->stream : ln.s, t->type, t->K, r.hi - r.lo, 1, 0,
                      (const uint8_t *)src + r.lo * row_bytes, r.d));
        }
        RT_CHECK(hipSetDevice(m->device));
        return 0;
    }
    if (t->dec) RC(upload(m->device, m->stream, KT_Q8_0, t->K, t->N, 1, 0, src, t->dec));
    RC(upload(m->device, m->stream, t->type, t->K, t->N, t->slices, t->slice_bytes, src, t->d));
    if (t->pre) {
        RC(kcpp_q6p_build(t->d, t->K, t->N, t->pre, m->stream));
        RT_CHECK(hipStreamSynchronize(m->stream));
    }
    return 0;
}

extern "C" float *kcpp_model_hidden(kcpp_model *m) { return m->x; }
extern "C" int kcpp_model_read_hidden(kcpp_model *m, float *host, int64_t n_floats, int64_t offset) {
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    RT_CHECK(hipMemcpy(host, m->x + offset, (size_t)n_floats * 4, hipMemcpyDeviceToHost));
    return 0;
}
// stream-ordered copy between the residual stream and a caller buffer (device or pinned/pageable
// host; hipMemcpyDefault infers the direction).  dir 0: buf -> stage input, 1: stage output -> buf.
// Pipeline handoff replacing ggml_backend_cuda_cpy_tensor_async (ggml-cuda.cu:2392-2445).
extern "C" int kcpp_model_hidden_io(kcpp_model *m, void *buf, int64_t n_floats, int64_t offset, int dir) {
    RT_CHECK(hipSetDevice(m->device));
    if (n_floats < 0 || offset < 0 || offset + n_floats > (int64_t)m->ub * m->hp.n_embd) { g_err = "hidden_io: range"; return -2; }
    float *x = m->x + offset;
    RT_CHECK(hipMemcpyAsync(dir ? buf : (void *)x, dir ? (const void *)x : buf, (size_t)n_floats * 4, hipMemcpyDefault,
                            m->stream));
    return 0;
}
extern "C" int kcpp_model_sync(kcpp_model *m) {
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    return 0;
}
extern "C" void *kcpp_model_stream(kcpp_model *m) { return m->stream; }
extern "C" int kcpp_model_read_logits(kcpp_model *m, float *host) {
    if (!m->has_output) { g_err = "read_logits: stage has no output head"; return -2; }
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipMemcpyAsync(m->logits_pin, m->logits, (size_t)m->hp.n_vocab * 4, hipMemcpyDeviceToHost, m->stream));
    RT_CHECK(hipStreamSynchronize(m->stream));
    memcpy(host, m->logits_pin, (size_t)m->hp.n_vocab * 4);
    return 0;
}
extern "C" int64_t kcpp_model_weight_bytes(kcpp_model *m) { return m->weight_bytes; }
extern "C" int kcpp_model_set_graphs(kcpp_model *m, int enable) {
    m->use_graphs = enable != 0 && m->lanes.empty();   // split buffers disable graphs (ggml-cuda.cu graph_compute)
    return 0;
}

// rows [lo, hi) of an nrows matrix on device `id` of n under tensor_split (get_row_split / ggml_cuda_op_mul_mat,
// ggml-cuda.cu:625-651,1445-1463): tensor_split is normalized to cumulative starts (ggml_backend_cuda_split_buffer_type,
// all zero: equal shares), the bounds are rounded down to the MMQ tile height (get_row_rounding: 128 rows on CDNA)
// unless they reach nrows, the last device ends at nrows
extern "C" int kcpp_row_split_range(int64_t nrows, int n, const float *tensor_split, int id, int64_t *lo, int64_t *hi) {
    if (n < 1 || n > 16 || id < 0 || id >= n) return -1;
    float start[17];
    float sum = 0.0f;
    bool zero = true;
    for (int i = 0; i < n; ++i) zero &= !tensor_split || tensor_split[i] == 0.0f;
    for (int i = 0; i < n; ++i) { start[i] = sum; sum += zero ? 1.0f : tensor_split[i]; }
    for (int i = 0; i < n; ++i) start[i] /= sum;
    // get_row_rounding: the tile height of every device with a non-empty share
    int64_t rounding = 0;
    for (int i = 0; i < n; ++i)
        if (start[i] < (i + 1 < n ? start[i + 1] : 1.0f)) rounding = 128;
    if (!rounding) rounding = 128;
    int64_t l = 0, h = nrows;
    if (id != 0) {
        l = (int64_t)(nrows * start[id]);
        if (l < nrows) l -= l % rounding;
    }
    if (id != n - 1) {
        h = (int64_t)(nrows * start[id + 1]);
        if (h < nrows) h -= h % rounding;
    }
    *lo = l; *hi = h;
    return 0;
}

// LLAMA_SPLIT_MODE_ROW (koboldcpp --rowsplit, gpttype_adapter.cpp:1892; llm_load_tensors' split_buft for the
// repeating layers' matrices and the output matrix, src/llama.cpp:7038-7057): the stage keeps every non-matrix
// op, the KV cache and the activations on its own device (main_gpu) and the rows of each dense matrix are spread
// over `devices` by tensor_split.  Call after create and before the weights are set; the fused single-token
// kernels (norm / RoPE / KV store inside the mat-vecs) and graph replay are off, as the reference's split
// buffers turn CUDA graphs off.  MoE expert tensors cannot be split (ggml_cuda_op_mul_mat asserts ne02 == 1 for
// split buffers, ggml-cuda.cu:1404): refused.
extern "C" int kcpp_model_set_row_split(kcpp_model *m, int n, const int *devices, const float *tensor_split) {
    if (!m->lanes.empty()) { g_err = "row split already set"; return -2; }
    if (n < 1 || n > 16) { g_err = "row split: 1..16 devices"; return -2; }
    if (m->hp.n_expert > 0) { g_err = "row split: MoE expert tensors cannot be split (ggml-cuda.cu:1404)"; return -3; }
    RT_CHECK(hipSetDevice(m->device));
    int ndev = 0;
    RT_CHECK(hipGetDeviceCount(&ndev));
    for (int i = 0; i < n; ++i)
        if (!devices || devices[i] < 0 || devices[i] >= ndev) { g_err = "row split: bad device index"; return -2; }
    m->lanes.resize(n);
    bool have_inline = false;
    for (int i = 0; i < n; ++i) {
        m->lanes[i].dev = devices[i];
        if (devices[i] == m->device && !have_inline) { m->lanes[i].inline_main = true; have_inline = true; }
    }
    // the split matrices: each layer's q, k, v, o, gate, up, down and the output head; the concatenated q|k|v and
    // gate|up groups of the prefill fusion give way to per-device slices
    std::vector<KTensor *> mats;
    for (auto &L : m->layers) {
        for (int j : {1, 2, 3, 4, 6, 7, 8}) mats.push_back(&L.t[j]);
        if (L.qkv_base) { (void)hipFree(L.qkv_base); L.qkv_base = nullptr; }
        if (L.glu_base) { (void)hipFree(L.glu_base); L.glu_base = nullptr; }
        L.nqkv = 0; L.glu_fused = false;
    }
    if (m->has_output) mats.push_back(&m->output);
    size_t ymax = 0;
    for (KTensor *t : mats) {
        if (t->owned && t->d) (void)hipFree(t->d);
        t->d = nullptr; t->owned = false;
        if (t->pre && t->pre_owned) (void)hipFree(t->pre);       // row slices run q6v3 (no per-slice images)
        t->pre = nullptr; t->pre_owned = false;
        for (int i = 0; i < n; ++i) {
            RowSlice r;
            r.lane = i;
            kcpp_row_split_range(t->N, n, tensor_split, i, &r.lo, &r.hi);
            if (r.hi > r.lo) {
                RT_CHECK(hipSetDevice(devices[i]));
                RT_CHECK(hipMalloc(&r.d, ((size_t)tensor_bytes(t->type, t->K, r.hi - r.lo) + 255) & ~(size_t)255));
                ymax = std::max(ymax, (size_t)(r.hi - r.lo) * (t == &m->output ? 1 : m->ub));
            }
            t->rs.push_back(r);
        }
    }
    for (Lane &ln : m->lanes) {
        if (ln.inline_main) continue;
        RT_CHECK(hipSetDevice(ln.dev));
        RT_CHECK(hipStreamCreateWithFlags(&ln.s, hipStreamNonBlocking));
        RT_CHECK(hipEventCreateWithFlags(&ln.done, hipEventDisableTiming));
        RT_CHECK(hipMalloc(&ln.act, m->act_sz));
        RT_CHECK(hipMalloc((void **)&ln.y, std::max<size_t>(ymax, 1) * 4));
        if (m->gemm_ws_sz) {
            RT_CHECK(hipMalloc(&ln.ws, m->gemm_ws_sz));
            RT_CHECK(hipMemset(ln.ws, 0, m->gemm_ws_sz));        // KT_Q8_0_T tickets
        }
        if (ln.dev != m->device) {             // direct xGMI copies both ways
            (void)hipDeviceEnablePeerAccess(m->device, 0);
            RT_CHECK(hipSetDevice(m->device));
            (void)hipDeviceEnablePeerAccess(ln.dev, 0);
            (void)hipGetLastError();
        }
    }
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
    drop_graphs(m);
    m->use_graphs = false;
    m->fused_decode = false;
    return 0;
}
// the expert ids the last MoE prefill layer of this model (stage) routed its T tokens to, [T][n_expert_used]
// (the host copy moe_prefill groups tokens by): diagnostics for routing-aware parity tests
extern "C" int kcpp_model_moe_ids(kcpp_model *m, int32_t *out, int n) {
    if (!m->moe_ids_h || n < 0 || n > m->ub * std::max(1, m->hp.n_expert_used)) { g_err = "moe ids"; return -1; }
    RT_CHECK(hipStreamSynchronize(m->stream));
    memcpy(out, m->moe_ids_h, (size_t)n * 4);
    return 0;
}
// single-token routing trace (diagnostics): while enabled, every single-token MoE layer copies its top-k ids into
// [layer][n_expert_used]; kcpp_model_moe_trace_read returns the last step's.  Toggling drops the captured graph.
extern "C" int kcpp_model_moe_trace(kcpp_model *m, int enable) {
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    if (enable && !m->moe_trace && m->hp.n_expert > 0) {
        const size_t n = m->layers.size() * (size_t)std::max(1, m->hp.n_expert_used);
        RT_CHECK(hipMalloc(&m->moe_trace, n * 4));
        RT_CHECK(hipMemset(m->moe_trace, 0xFF, n * 4));
    } else if (!enable && m->moe_trace) {
        RT_CHECK(hipFree(m->moe_trace));
        m->moe_trace = nullptr;
    }
    drop_graphs(m);
    return 0;
}
// MoE single-token decode fusions: bit 0 routes inside the two-slot gate|up launch (else k_moe_route), bit 1 runs
// both slots' down projections in one launch (else two chained launches); every combination gives bit-identical ids,
// weights and logits (tests/test_gpu_moe.py).  Drops the captured graph.
extern "C" int kcpp_model_set_fused_route(kcpp_model *m, int on) {
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    m->no_fused_route = !(on & 1);
    m->no_pair_down = !(on & 2);
    drop_graphs(m);
    return 0;
}
extern "C" int64_t kcpp_model_fused_route_count(kcpp_model *m) { return m->n_fused_route + (m->n_pair_down << 32); }
// MoE prefill: grouped expert GEMMs (one launch for every expert's gate|up, one for every down; default) or the
// per-expert loop; returns the previous setting.  kcpp_model_moe_grouped_count: grouped layers run so far.
extern "C" int kcpp_model_set_moe_grouped(kcpp_model *m, int on) {
    const int old = !m->no_moe_grouped;
    m->no_moe_grouped = !on;
    return old;
}
extern "C" int64_t kcpp_model_moe_grouped_count(kcpp_model *m) { return m->n_moe_grouped; }
extern "C" int kcpp_model_moe_trace_read(kcpp_model *m, int32_t *out, int n) {
    if (!m->moe_trace || n < 0 || n > (int)m->layers.size() * std::max(1, m->hp.n_expert_used)) { g_err = "moe trace"; return -1; }
    RT_CHECK(hipStreamSynchronize(m->stream));
    RT_CHECK(hipMemcpy(out, m->moe_trace, (size_t)n * 4, hipMemcpyDeviceToHost));
    return 0;
}
extern "C" int kcpp_model_set_fa_exact(kcpp_model *m, int enable) {
    m->fa_exact = enable != 0;
    drop_graphs(m);
    return 0;
}
extern "C" int kcpp_model_set_kv_types(kcpp_model *m, int tk, int tv) {
    const bool q = tk == KT_Q8_0 || tk == KT_Q4_0;
    if (!((tk == KT_F16 && tv == KT_F16) || (q && (tv == KT_Q8_0 || tv == KT_Q4_0)))) {
        g_err = "kv types: F16/F16 or Q8_0|Q4_0 for both";
        return -1;
    }
    const int64_t E = m->hp.n_embd, H = m->hp.n_head, HKV = m->hp.n_head_kv, D = E / H, EKV = HKV * D;
    if (q && D % 32) { g_err = "quantized kv: head dim must be a multiple of 32"; return -1; }
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipStreamSynchronize(m->stream));
    for (auto &L : m->layers) {
        if (L.kc) RT_CHECK(hipFree(L.kc));
        if (L.vc) RT_CHECK(hipFree(L.vc));
        L.kc = L.vc = nullptr;
        const size_t kb = (size_t)kcpp_kv_cache_bytes(tk, m->hp.n_ctx, EKV), vb = (size_t)kcpp_kv_cache_bytes(tv, m->hp.n_ctx, EKV);
        if (hipMalloc(&L.kc, kb) != hipSuccess || hipMalloc(&L.vc, vb) != hipSuccess) { g_err = "kv alloc"; return -2; }
        RT_CHECK(hipMemset(L.kc, 0, kb));
        RT_CHECK(hipMemset(L.vc, 0, vb));
    }
    m->kv_tk = tk; m->kv_tv = tv;
    drop_graphs(m);
    return 0;
}
extern "C" int kcpp_model_set_fused_decode(kcpp_model *m, int enable) {
    m->fused_decode = enable != 0 && m->lanes.empty();
    drop_graphs(m);
    return 0;
}

static int mm_launch(int type, const void *W, const void *W2, int64_t K, int64_t N, const void *act, int64_t M, float *Y,
                     int64_t ldy, const float *res, int64_t ldr, int mode, void *ws, hipStream_t s) {
    if (M <= 8 && type != KT_Q8_0_T) return kcpp_gemv(type, W, W2, K, N, act, M, Y, ldy, res, ldr, mode, s);
    return kcpp_gemm(type, W, W2, K, N, act, M, Y, ldy, res, ldr, mode, ws, s);
}

// row split (ggml_cuda_op_mul_mat's split branch, ggml-cuda.cu:1403-1700): every lane computes its rows [lo, hi)
// of Y.  A lane other than the inline one waits for the stage stream's ev_in, takes the activation block (and,
// with a residual, its rows of the residual) by peer copies on its own stream, runs the same mat-vec / GEMM on
// its slice into its own rows buffer and copies those rows into Y before its `done` event, which the stage
// stream waits on.  Per row the arithmetic is the unsplit kernel's, so the split changes no row's result
// beyond the GEMM's split-K grouping (which follows the slice's grid).
static int matmul_rows(kcpp_model *m, const KTensor &W, const KTensor *W2, const void *act, int64_t M, float *Y,
                       int64_t ldy, const float *res, int64_t ldr, int mode) {
    const size_t abytes = (size_t)kcpp_act_bytes(W.type, W.K, M);
    // ev_in fences only the producers of act / res: it is recorded before the inline lane's launch, and every other
    // lane is enqueued before it, so the lanes' mat-muls run concurrently with the main device's slice
    bool fenced = false;
    int inl = -1;
    for (size_t i = 0; i < W.rs.size(); ++i) {
        const RowSlice &r = W.rs[i];
        const int64_t n = r.hi - r.lo;
        if (n <= 0) continue;
        const Lane &ln = m->lanes[r.lane];
        if (ln.inline_main) { inl = (int)i; continue; }
        if (!fenced) { RT_CHECK(hipEventRecord(m->ev_in, m->stream)); fenced = true; }
        const void *w2 = W2 ? W2->rs[i].d : nullptr;
        RT_CHECK(hipSetDevice(ln.dev));
        RT_CHECK(hipStreamWaitEvent(ln.s, m->ev_in, 0));
        RT_CHECK(hipMemcpyPeerAsync(ln.act, ln.dev, act, m->device, abytes, ln.s));
        if (res)
            RT_CHECK(hipMemcpy2DAsync(ln.y, n * 4, res + r.lo, ldr * 4, n * 4, M, hipMemcpyDefault, ln.s));
        RC(mm_launch(W.type, r.d, w2, W.K, n, ln.act, M, ln.y, n, res ? ln.y : nullptr, n, mode, ln.ws, ln.s));
        RT_CHECK(hipMemcpy2DAsync(Y + r.lo, ldy * 4, ln.y, n * 4, n * 4, M, hipMemcpyDefault, ln.s));
        RT_CHECK(hipEventRecord(ln.done, ln.s));
        RT_CHECK(hipSetDevice(m->device));
    }
    if (inl >= 0) {
        const RowSlice &r = W.rs[inl];
        RC(mm_launch(W.type, r.d, W2 ? W2->rs[inl].d : nullptr, W.K, r.hi - r.lo, act, M, Y + r.lo, ldy,
                     res ? res + r.lo : nullptr, ldr, mode, m->gemm_ws, m->stream));
    }
    for (size_t i = 0; fenced && i < W.rs.size(); ++i) {
        const RowSlice &r = W.rs[i];
        if (r.hi - r.lo <= 0 || (int)i == inl) continue;
        RT_CHECK(hipStreamWaitEvent(m->stream, m->lanes[r.lane].done, 0));
    }
    return 0;
}

// y[c][n] = W . act  (+res) for M columns: mat-vec for M <= 8, MFMA GEMM above
// the batched GEMM of one weight (M > 8): Q6_K with a prefill image on the int8 kernel (kcpp_gemm's bits), else kcpp_gemm
static int gemm_w(const KTensor &W, const KTensor *W2, const void *act, int64_t M, float *Y, int64_t ldy, const float *res,
                  int64_t ldr, int mode, void *ws, hipStream_t s) {
    if (W.pre && (!W2 || W2->pre)) {
        const int rc = kcpp_gemm_q6p(W.pre, W.d, W2 ? W2->pre : nullptr, W2 ? W2->d : nullptr, W.K, W.N, act, M, Y, ldy,
                                     res, ldr, mode, ws, s);
        if (rc != -3) return rc;
    }
    return kcpp_gemm(W.type, W.d, W2 ? W2->d : nullptr, W.K, W.N, act, M, Y, ldy, res, ldr, mode, ws, s);
}

// the residual GEMM (M > 8) followed by the next rms_norm's Q8_K activation: the norm folded into the GEMM's split-K
// reduce where it splits (kcpp_gemm_rms_norm), the two steps' bits either way
static int gemm_w_norm(const KTensor &W, const void *act, int64_t M, float *Y, int64_t ldy, const float *res, int64_t ldr,
                       void *ws, hipStream_t s, const float *nw, float eps, void *qout) {
    if (W.pre) {
        const int rc = kcpp_gemm_q6p_rms_norm(W.pre, W.d, W.K, W.N, act, M, Y, ldy, res, ldr, ws, s, nw, eps, qout);
        if (rc != -3) return rc;
    }
    return kcpp_gemm_rms_norm(W.type, W.d, W.K, W.N, act, M, Y, ldy, res, ldr, ws, s, nw, eps, qout);
}
// may the residual GEMM of W at T tokens carry the following rms_norm -> Q8_K (gemm_w_norm)?
static bool norm_foldable(const kcpp_model *m, const KTensor &W, int T) {
    return T > 8 && W.rs.empty() && W.type != KT_Q8_0_T && m->lanes.empty() && !m->no_norm_fold;
}

static int matmul(kcpp_model *m, const KTensor &W, const KTensor *W2, const void *act, int64_t M, float *Y, int64_t ldy,
                  const float *res, int64_t ldr, int mode) {
    if (!W.rs.empty()) return matmul_rows(m, W, W2, act, M, Y, ldy, res, ldr, mode);
    if (M <= 8 && W.type != KT_Q8_0_T)
        return kcpp_gemv(W.type, W.d, W2 ? W2->d : nullptr, W.K, W.N, act, M, Y, ldy, res, ldr, mode, m->stream);
    return gemm_w(W, W2, act, M, Y, ldy, res, ldr, mode, m->gemm_ws, m->stream);
}

static int rows_per_wave(int64_t N, int mode) {
    if (mode == 1) return 1;
    return N > 16384 ? 4 : (N > 4096 ? 2 : 1);
}

// MoE FFN for one token (llm_build_moe_ffn, src/llama.cpp:9416-9514), entirely on the device:
// ffn_norm -> router/softmax/top-k on the GPU (moe_ids, moe_w), then per top-k slot j the expert's
// gate|up and down mat-vecs read their expert index from moe_ids[j] (DecArgs.eid) and down writes
// w_j * out into slot j; the combine sums the slots in top-k order and adds the residual.
static int moe_dec(kcpp_model *m, const KLayer &L) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd, F = hp.n_ff;
    const int NU = hp.n_expert_used;
    const KTensor *t = L.t;
    hipStream_t s = m->stream;
    auto is_q81 = [](int ty) { return ty == KT_Q4_1 || ty == KT_Q5_1; };
    // RS gate|up with two slots: both slots' GLU rows in one launch (segment j = slot j, its own expert index), one
    // ramp instead of two; h of slot j at m->h + j F.  The router runs inside that launch where it can (top-2 of <= 8
    // experts, K <= 4096: every workgroup routes on its prologue's normalised row, workgroup 0 stores ids / weights)
    const bool rs_gu = t[6].type == t[7].type &&
                       (t[6].type == KT_Q4_K_RS || t[6].type == KT_Q5_K_RS || t[6].type == KT_Q6_K_RS);
    const bool pair = rs_gu && NU == 2 && m->ub >= 2;
    bool routed = false;
    if (pair && !m->no_fused_route && (t[9].type == KT_F32 || t[9].type == KT_F16) && hp.n_expert <= 8 && E <= 4096) {
        DecArgs a;
        memset(&a, 0, sizeof a);
        a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 2;
        a.W[0] = a.W[1] = (const uint8_t *)t[6].d; a.W2 = (const uint8_t *)t[7].d; a.N[0] = a.N[1] = F;
        a.Y[0] = m->h; a.Y[1] = m->h + F;
        a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[6].slice_bytes;
        a.route_w = t[9].d; a.route_wt = t[9].type; a.route_ne = (int)hp.n_expert;
        a.route_ids = m->moe_ids; a.route_wts = m->moe_w;
        const int rc = kcpp_gemv_dec(t[6].type, &a, 1, 1, rows_per_wave(F, 1), s);
        if (rc != 0 && rc != -3) return rc;
        routed = rc == 0;
        m->n_fused_route += routed;
    }
    if (!routed &&
        kcpp_moe_route_norm(m->x, E, (const float *)t[5].d, hp.eps, t[9].d, t[9].type, E, hp.n_expert, NU, m->moe_ids,
                            m->moe_w, 1, s) != 0) {
        RC(kcpp_rms_norm(m->x, E, (const float *)t[5].d, m->attn, E, nullptr, E, 1, hp.eps, s));
        RC(kcpp_moe_route(m->attn, E, t[9].d, t[9].type, E, hp.n_expert, NU, m->moe_ids, m->moe_w, 1, s));
    }
    if (m->moe_trace)
        RT_CHECK(hipMemcpyAsync(m->moe_trace + (&L - m->layers.data()) * NU, m->moe_ids, (size_t)NU * 4,
                                hipMemcpyDeviceToDevice, s));
    if (is_q81(t[6].type) || is_q81(t[7].type) || is_q81(t[8].type)) {
        // expert types without a fused decode mat-vec (Q4_1 / Q5_1; chosen per layer from the expert tensors, not the
        // model-wide flag: K-quant experts sit in the RS layouts, which the generic expert mat-vec does not read): ffn_norm + activation quantization once, then per
        // slot the generic mat-vec on the expert slice its device-resident id selects (kcpp_gemv_expert)
        const int vg = kcpp_vec_dot_type(t[6].type), vu = kcpp_vec_dot_type(t[7].type), vd = kcpp_vec_dot_type(t[8].type);
        RC(kcpp_rms_norm(m->x, E, (const float *)t[5].d, m->attn, E, nullptr, E, 1, hp.eps, s));
        RC(kcpp_quantize_act(vg, m->attn, E, m->act, E, 1, s));
        if (vu != vg) RC(kcpp_quantize_act(vu, m->attn, E, m->act2, E, 1, s));
        for (int j = 0; j < NU; ++j) {
            const int32_t *id = m->moe_ids + j;
            if (t[6].type == t[7].type) {
                RC(kcpp_gemv_expert(t[6].type, t[6].d, t[7].d, E, F, m->act, m->h, id, (int64_t)t[6].slice_bytes,
                                    hp.n_expert, nullptr, 1, s));
            } else {
                RC(kcpp_gemv_expert(t[6].type, t[6].d, nullptr, E, F, m->act, m->h, id, (int64_t)t[6].slice_bytes,
                                    hp.n_expert, nullptr, 0, s));
                RC(kcpp_gemv_expert(t[7].type, t[7].d, nullptr, E, F, vu != vg ? m->act2 : m->act, m->qkv, id,
                                    (int64_t)t[7].slice_bytes, hp.n_expert, nullptr, 0, s));
                RC(kcpp_silu_mul(m->h, m->h, m->qkv, F, s));
            }
            RC(kcpp_quantize_act(vd, m->h, F, m->act2, F, 1, s));
            RC(kcpp_gemv_expert(t[8].type, t[8].d, nullptr, F, E, m->act2, m->moe_slots + j * E, id,
                                (int64_t)t[8].slice_bytes, hp.n_expert, m->moe_w + j, 0, s));
        }
        return kcpp_moe_combine(m->x, m->moe_slots, E, NU, E, s);
    }
    // RS down projections (MODE 0 store epilogue with DecArgs.pre): k_moe_combine's ((s0 + s1) + ...) + x in the
    // same order, one launch per layer less
    const bool chain = t[8].type == KT_Q4_K_RS || t[8].type == KT_Q5_K_RS || t[8].type == KT_Q6_K_RS;
    if (pair && !routed) {
        DecArgs a;
        memset(&a, 0, sizeof a);
        a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 2;
        a.W[0] = a.W[1] = (const uint8_t *)t[6].d; a.W2 = (const uint8_t *)t[7].d; a.N[0] = a.N[1] = F;
        a.Y[0] = m->h; a.Y[1] = m->h + F;
        a.eid = m->moe_ids; a.eid1 = m->moe_ids + 1; a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[6].slice_bytes;
        RC(kcpp_gemv_dec(t[6].type, &a, 1, 1, rows_per_wave(F, 1), s));
    }
    // RS down projections of both slots in one launch (k_gemv_rs MODE 3: half the waves per slot, met in LDS):
    // ((w0 o0) + (w1 o1)) + x, the two chained launches' result bit for bit
    if (pair && chain && !m->no_pair_down) {
        DecArgs a;
        memset(&a, 0, sizeof a);
        a.K = F; a.x = m->h; a.nseg = 1;
        a.W[0] = a.W[1] = (const uint8_t *)t[8].d; a.N[0] = E; a.Y[0] = m->x; a.res = m->x;
        a.eid = m->moe_ids; a.eid1 = m->moe_ids + 1; a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[8].slice_bytes;
        a.escale = m->moe_w;
        const int rc = kcpp_gemv_dec(t[8].type, &a, 3, 2, rows_per_wave(E, 0), s);
        if (rc == 0) { m->n_pair_down++; return 0; }
        if (rc != -3) return rc;
    }
    for (int j = 0; j < NU; ++j) {
        if (pair) {
        } else if (t[6].type == t[7].type) {
            DecArgs a;
            memset(&a, 0, sizeof a);
            a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 1;
            a.W[0] = (const uint8_t *)t[6].d; a.W2 = (const uint8_t *)t[7].d; a.N[0] = F; a.Y[0] = m->h;
            a.eid = m->moe_ids + j; a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[6].slice_bytes;
            RC(kcpp_gemv_dec(t[6].type, &a, 1, 1, rows_per_wave(F, 1), s));
        } else {
            for (int i = 6; i <= 7; ++i) {
                DecArgs a;
                memset(&a, 0, sizeof a);
                a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 1;
                a.W[0] = (const uint8_t *)t[i].d; a.N[0] = F; a.Y[0] = i == 6 ? m->h : m->qkv;
                a.eid = m->moe_ids + j; a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[i].slice_bytes;
                RC(kcpp_gemv_dec(t[i].type, &a, 0, 1, rows_per_wave(F, 0), s));
            }
            RC(kcpp_silu_mul(m->h, m->h, m->qkv, F, s));
        }
        DecArgs a;
        memset(&a, 0, sizeof a);
        a.K = F; a.x = pair ? m->h + j * F : m->h; a.nseg = 1;
        a.W[0] = (const uint8_t *)t[8].d; a.N[0] = E; a.Y[0] = m->moe_slots + j * E;
        a.eid = m->moe_ids + j; a.n_exp = hp.n_expert; a.ebytes = (int64_t)t[8].slice_bytes; a.escale = m->moe_w + j;
        if (chain) {            // slot sum carried through the down projections, the last one adds the residual
            a.Y[0] = j == NU - 1 ? m->x : m->moe_slots;
            a.pre = j > 0 ? m->moe_slots : nullptr;
            a.res = j == NU - 1 ? m->x : nullptr;
        }
        const int rc = kcpp_gemv_dec(t[8].type, &a, 0, 2, rows_per_wave(E, 0), s);
        if (rc == -8) {
            // n_ff beyond the fused kernels' budget (no RS layout for it: chain is false, slots + combine): quantize the
            // slot's h once, then the generic expert mat-vec (device-resident expert id, times the router weight)
            RC(kcpp_quantize_act(kcpp_vec_dot_type(t[8].type), a.x, F, m->act2, F, 1, s));
            RC(kcpp_gemv_expert(t[8].type, t[8].d, nullptr, F, E, m->act2, m->moe_slots + j * E, m->moe_ids + j,
                                (int64_t)t[8].slice_bytes, hp.n_expert, m->moe_w + j, 0, s));
            continue;
        }
        RC(rc);
    }
    return chain ? 0 : kcpp_moe_combine(m->x, m->moe_slots, E, NU, E, s);
}

// MoE FFN for a ubatch of T tokens: routing on the GPU, one host sync to group the tokens by expert
// (ggml_cuda_mul_mat_id does the same, ggml-cuda.cu:2003-2139), then per expert with tokens: gather
// the normalized rows, gate|up GEMM with silu*up, down GEMM, weighted scatter into the top-k slots.
static bool grouped_type(int t) { return t == KT_Q4_K || t == KT_Q4_K_RS || t == KT_Q5_K || t == KT_Q5_K_RS; }
// the grouped int8 GEMM streams the Q8_K bsums plane of its M-row activation by 16-B DMA: M * (K / 256) * 4 bytes of d
// in front of it must keep it 16-B aligned (kcpp_gemm_grouped returns -3 otherwise, e.g. K 11008 or 6400 with an odd
// routed-row count); such layers take the per-expert path
static bool grouped_act_aligned(int64_t M, int64_t K) { return (M * (K / 256)) % 4 == 0; }

// grouped MoE prefill (after routing): every routed row gathered in expert order, one Q8_K quantization, the gate|up
// GEMMs of all experts in one launch (kcpp_gemm_grouped), the down GEMMs likewise (or per expert for a type the
// grouped kernel lacks, e.g. Q6_K), one scatter -- 5-6 launches per layer instead of 6 per active expert, and grids
// that fill the GPU at ~ubatch*k/n_expert rows per expert.  Per row the arithmetic is the per-expert path's v4
// (unsplit), so gate|up is bitwise that path's and down within its split-K re-association.
static int moe_prefill_grouped(kcpp_model *m, const KLayer &L, int T, const int *cnt, const int *off, bool down_grouped) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd, F = hp.n_ff, UB = m->ub;
    const int NU = hp.n_expert_used, NE = hp.n_expert;
    const KTensor *t = L.t;
    hipStream_t s = m->stream;
    const int64_t R = (int64_t)T * NU;
    if (!m->moe_gx) {
        const int64_t RM = UB * NU;
        if (hipMalloc(&m->moe_gx, RM * E * 4) != hipSuccess || hipMalloc(&m->moe_gh, RM * F * 4) != hipSuccess ||
            hipMalloc(&m->moe_gup, RM * F * 4) != hipSuccess || hipMalloc(&m->moe_geo, RM * E * 4) != hipSuccess ||
            hipMalloc(&m->moe_gact, kcpp_act_bytes(KT_Q4_K, std::max(E, F), RM)) != hipSuccess ||
            hipMalloc(&m->moe_gcnt, 64 * 4) != hipSuccess ||
            hipHostMalloc((void **)&m->moe_gcnt_h, 64 * 4, hipHostMallocDefault) != hipSuccess) {
            g_err = "grouped MoE buffers";
            return -2;
        }
    }
    memcpy(m->moe_gcnt_h, cnt, (size_t)NE * 4);        // the previous layer's copy is done (moe_prefill synchronized)
    RT_CHECK(hipMemcpyAsync(m->moe_gcnt, m->moe_gcnt_h, (size_t)NE * 4, hipMemcpyHostToDevice, s));
    RC(kcpp_moe_gather(m->attn, E, m->moe_rows, (int)R, E, m->moe_gx, s));
    RC(kcpp_quantize_act(kcpp_vec_dot_type(t[6].type), m->moe_gx, E, m->moe_gact, E, R, s));
    RC(kcpp_gemm_grouped(t[6].type, t[6].d, t[7].d, t[6].slice_bytes, E, F, m->moe_gact, R, cnt, m->moe_gcnt, NE,
                         m->moe_gh, m->moe_gup, 1, nullptr, s));
    if (down_grouped && kcpp_vec_dot_type(t[8].type) == KT_Q8_K) {
        void *gws = nullptr;
        if (t[8].type == KT_Q6_K_RS) {          // the f16 fragment image of the padded layout (lazily, once)
            if (!m->moe_gws && hipMalloc(&m->moe_gws, kcpp_gemm_grouped_ws_bytes(KT_Q6_K_RS, F, UB * NU, NE)) != hipSuccess) {
                g_err = "grouped MoE workspace";
                return -2;
            }
            gws = m->moe_gws;
        }
        RC(kcpp_quantize_act(KT_Q8_K, m->moe_gh, F, m->moe_gact, F, R, s));
        RC(kcpp_gemm_grouped(t[8].type, t[8].d, nullptr, t[8].slice_bytes, F, E, m->moe_gact, R, cnt, m->moe_gcnt, NE,
                             m->moe_geo, nullptr, 0, gws, s));
    } else {
        for (int e = 0; e < NE; ++e) {
            const int n = cnt[e];
            if (!n) continue;
            KTensor d = t[8];
            d.d = (uint8_t *)t[8].d + e * t[8].slice_bytes;
            RC(kcpp_quantize_act(kcpp_vec_dot_type(d.type), m->moe_gh + (int64_t)off[e] * F, F, m->act2, F, n, s));
            RC(matmul(m, d, nullptr, m->act2, n, m->moe_geo + (int64_t)off[e] * E, E, nullptr, 0, 0));
        }
    }
    RC(kcpp_moe_scatter(m->moe_slots, E, m->moe_geo, m->moe_rows + UB * NU, m->moe_rw, (int)R, E, s));
    m->n_moe_grouped++;
    return kcpp_moe_combine(m->x, m->moe_slots, (int64_t)T * E, NU, (int64_t)T * E, s);
}

static int moe_prefill(kcpp_model *m, const KLayer &L, int T) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd, F = hp.n_ff, UB = m->ub;
    const int NU = hp.n_expert_used, NE = hp.n_expert;
    const KTensor *t = L.t;
    hipStream_t s = m->stream;
    RC(kcpp_rms_norm(m->x, E, (const float *)t[5].d, m->attn, E, nullptr, E, T, hp.eps, s));
    RC(kcpp_moe_route(m->attn, E, t[9].d, t[9].type, E, NE, NU, m->moe_ids, m->moe_w, T, s));
    RT_CHECK(hipMemcpyAsync(m->moe_ids_h, m->moe_ids, (size_t)T * NU * 4, hipMemcpyDeviceToHost, s));
    RT_CHECK(hipMemcpyAsync(m->moe_w_h, m->moe_w, (size_t)T * NU * 4, hipMemcpyDeviceToHost, s));
    RT_CHECK(hipStreamSynchronize(s));
    int cnt[64] = {0}, off[65];
    for (int i = 0; i < T * NU; ++i) {
        const int e = m->moe_ids_h[i];
        if (e < 0 || e >= NE) { g_err = "MoE router produced an invalid expert id"; return -5; }
        ++cnt[e];
    }
    off[0] = 0;
    for (int e = 0; e < NE; ++e) off[e + 1] = off[e] + cnt[e];
    int fill[64];
    memcpy(fill, off, sizeof fill);
    int32_t *src_rows = m->moe_rows_h, *dst_rows = m->moe_rows_h + UB * NU;
    for (int tk = 0; tk < T; ++tk)
        for (int j = 0; j < NU; ++j) {
            const int e = m->moe_ids_h[tk * NU + j], p = fill[e]++;
            src_rows[p] = tk;
            dst_rows[p] = j * T + tk;                        // slot j, token tk
            m->moe_rw_h[p] = m->moe_w_h[tk * NU + j];
        }
    RT_CHECK(hipMemcpyAsync(m->moe_rows, m->moe_rows_h, (size_t)2 * UB * NU * 4, hipMemcpyHostToDevice, s));
    RT_CHECK(hipMemcpyAsync(m->moe_rw, m->moe_rw_h, (size_t)T * NU * 4, hipMemcpyHostToDevice, s));
    const int64_t RR = (int64_t)T * NU;
    const bool down_grouped = (grouped_type(t[8].type) && grouped_act_aligned(RR, F)) || t[8].type == KT_Q6_K_RS;
    if (!m->no_moe_grouped && t[6].type == t[7].type && grouped_type(t[6].type) && E % 256 == 0 && F % 256 == 0 &&
        NE <= 64 && grouped_act_aligned(RR, E))
        return moe_prefill_grouped(m, L, T, cnt, off, down_grouped);
    float *xg = m->qkv, *eo = m->hglu;
    for (int e = 0; e < NE; ++e) {
        const int n = cnt[e];
        if (!n) continue;
        RC(kcpp_moe_gather(m->attn, E, m->moe_rows + off[e], n, E, xg, s));
        KTensor g = t[6], u = t[7], d = t[8];
        g.d = (uint8_t *)t[6].d + e * t[6].slice_bytes;
        u.d = (uint8_t *)t[7].d + e * t[7].slice_bytes;
        d.d = (uint8_t *)t[8].d + e * t[8].slice_bytes;
        RC(kcpp_quantize_act(kcpp_vec_dot_type(g.type), xg, E, m->act, E, n, s));
        if (g.type == u.type) {
            RC(matmul(m, g, &u, m->act, n, m->h, F, nullptr, 0, 1));           // h = silu(g) * u
        } else {
            RC(matmul(m, g, nullptr, m->act, n, m->h, F, nullptr, 0, 0));
            if (kcpp_vec_dot_type(u.type) != kcpp_vec_dot_type(g.type))
                RC(kcpp_quantize_act(kcpp_vec_dot_type(u.type), xg, E, m->act, E, n, s));
            RC(matmul(m, u, nullptr, m->act, n, eo, F, nullptr, 0, 0));
            RC(kcpp_silu_mul(m->h, m->h, eo, (int64_t)n * F, s));
        }
        RC(kcpp_quantize_act(kcpp_vec_dot_type(d.type), m->h, F, m->act2, F, n, s));
        RC(matmul(m, d, nullptr, m->act2, n, eo, E, nullptr, 0, 0));
        RC(kcpp_moe_scatter(m->moe_slots, E, eo, m->moe_rows + UB * NU + off[e], m->moe_rw + off[e], n, E, s));
    }
    return kcpp_moe_combine(m->x, m->moe_slots, (int64_t)T * E, NU, (int64_t)T * E, s);
}

// single-token layer step, 6-7 launches (gemv_dec.hip fusions); position read from m->pos_dev
static int forward_layers_dec(kcpp_model *m) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd, F = hp.n_ff, H = hp.n_head, HKV = hp.n_head_kv, D = E / H, EKV = HKV * D;
    hipStream_t s = m->stream;
    const float kq_scale = 1.0f / sqrtf((float)D);
    for (int il = m->il0; il < m->il1; ++il) {
        KLayer &L = m->layers[il - m->il0];
        KTensor tl[10];                              // the layer's tensors; KT_Q8_0_T ones by their KT_Q8_0 decode copies
        for (int j = 0; j < 10; ++j) {
            tl[j] = L.t[j];
            if (tl[j].dec) { tl[j].type = KT_Q8_0; tl[j].d = tl[j].dec; }
        }
        const KTensor *t = tl;
        // --- attn_norm + q|k|v + rope + K/V cache store: one launch per quant type present; q|k Q4_K + v Q6_K (the
        // Q4_K_M more-bits layers) in one launch.  (Two launches forked onto a side stream inside the graph
        // replayed slower than in sequence, 453 vs 517 tok/s: removed.)
        DecArgs qa[3];
        int qty[3], nq = 0;
        for (int j = 1; j <= 3;) {
            DecArgs &a = qa[nq];
            memset(&a, 0, sizeof a);
            a.K = E; a.x = m->x; a.nw = (const float *)t[0].d; a.eps = hp.eps;
            a.q16 = m->q16; a.kc = L.kc; a.vc = L.vc; a.ekv = EKV; a.D = (int)D; a.pos = m->pos_dev;
            a.rope_tab = m->rope_tab;
            const int ty = t[j].type;
            while (j <= 3 && t[j].type == ty) {
                a.W[a.nseg] = (const uint8_t *)t[j].d; a.N[a.nseg] = t[j].N; a.role[a.nseg] = j - 1;
                ++a.nseg; ++j;
            }
            qty[nq++] = ty;
        }
        int mixed_rc = -3;
        if (nq == 2 && qty[0] == KT_Q4_K_RS && qty[1] == KT_Q6_K_RS && qa[0].nseg == 2 && qa[1].nseg == 1 &&
            qa[1].role[0] == 2) {
            // q|k Q4_K + v Q6_K (Q4_K_M "more bits" layers): one launch (gemv_rs.hip k_gemv_rs_qkv)
            DecArgs c = qa[0];
            c.W[2] = qa[1].W[0]; c.N[2] = qa[1].N[0]; c.role[2] = 2; c.nseg = 3;
            mixed_rc = kcpp_gemv_rs_qkv_mixed(&c, s);
            if (mixed_rc != -3 && mixed_rc != -5) RC(mixed_rc);
        }
        if (mixed_rc != 0 && nq == 2 && qty[1] == KT_Q8_0 && !m->no_dual_qkv) {
            // q in an RS layout + k|v in Q8_0 (Mixtral's Q5_K_M policy): both launches' workgroups in one grid
            mixed_rc = kcpp_gemv_qkv_dual(&qa[0], qty[0], &qa[1], s);
            if (mixed_rc != -3 && mixed_rc != -5) RC(mixed_rc);
        }
        if (mixed_rc != 0)
            for (int i = 0; i < nq; ++i) RC(kcpp_gemv_dec(qty[i], &qa[i], 2, 1, 2, s));
        // --- attention over the cache (f32 output); wo quantizes it in its own prologue (PRO 2: the Q8_K /
        // Q8_0 conversion overlaps wo's first weight loads instead of ending the attention combine; measured
        // against the combine quantizing and wo copying: 572 vs 575 tok/s, within noise)
        if (m->fa_exact)
            RC(kcpp_flash_attn_exact(m->q16, L.kc, L.vc, m->attn, 1, (int)H, (int)HKV, (int)D, 0, m->pos_dev, kq_scale, s));
        else
            RC(kcpp_flash_attn(m->q16, L.kc, L.vc, m->attn, nullptr, m->fa_ws, 1, (int)H, (int)HKV, (int)D, 0, m->pos_dev,
                               hp.n_ctx, kq_scale, m->dec_short && D == 128 ? 7 : 1, s));
        {   // x += wo . attn
            DecArgs a;
            memset(&a, 0, sizeof a);
            a.K = E; a.nseg = 1;
            a.W[0] = (const uint8_t *)t[4].d; a.N[0] = t[4].N; a.Y[0] = m->x; a.res = m->x;
            a.x = m->attn;
            int rc = kcpp_gemv_dec(t[4].type, &a, 0, 2, rows_per_wave(t[4].N, 0), s);
            if (rc == -3) {
                RC(kcpp_quantize_act(kcpp_vec_dot_type(t[4].type), m->attn, E, m->act, E, 1, s));
                a.x = nullptr; a.act = (const uint8_t *)m->act;
                rc = kcpp_gemv_dec(t[4].type, &a, 0, 0, rows_per_wave(t[4].N, 0), s);
            }
            RC(rc);
        }
        if (hp.n_expert > 0) { RC(moe_dec(m, L)); continue; }
        // --- ffn_norm + gate|up + silu*mul
        if (t[6].type == t[7].type) {
            DecArgs a;
            memset(&a, 0, sizeof a);
            a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 1;
            a.W[0] = (const uint8_t *)t[6].d; a.W2 = (const uint8_t *)t[7].d; a.N[0] = F; a.Y[0] = m->h;
            RC(kcpp_gemv_dec(t[6].type, &a, 1, 1, rows_per_wave(F, 1), s));
        } else {
            for (int j = 6; j <= 7; ++j) {
                DecArgs a;
                memset(&a, 0, sizeof a);
                a.K = E; a.x = m->x; a.nw = (const float *)t[5].d; a.eps = hp.eps; a.nseg = 1;
                a.W[0] = (const uint8_t *)t[j].d; a.N[0] = F; a.Y[0] = j == 6 ? m->h : m->qkv;
                RC(kcpp_gemv_dec(t[j].type, &a, 0, 1, rows_per_wave(F, 0), s));
            }
            RC(kcpp_silu_mul(m->h, m->h, m->qkv, F, s));
        }
        {   // x += down . quant(h)
            DecArgs a;
            memset(&a, 0, sizeof a);
            a.K = F; a.x = m->h; a.nseg = 1;
            a.W[0] = (const uint8_t *)t[8].d; a.N[0] = E; a.Y[0] = m->x; a.res = m->x;
            const int rc = kcpp_gemv_dec(t[8].type, &a, 0, 2, rows_per_wave(E, 0), s);
            if (rc == -8) {   // K-slices beyond the fused kernel's register budget (very large n_ff)
                RC(kcpp_quantize_act(kcpp_vec_dot_type(t[8].type), m->h, F, m->act2, F, 1, s));
                RC(kcpp_gemv(t[8].type, t[8].d, nullptr, F, E, m->act2, 1, m->x, E, m->x, E, 0, s));
            } else if (rc) {
                RC(rc);
            }
        }
    }
    return 0;
}

static int head_dec(kcpp_model *m) {
    DecArgs a;
    memset(&a, 0, sizeof a);
    a.K = m->hp.n_embd; a.x = m->x; a.nw = (const float *)m->output_norm.d; a.eps = m->hp.eps; a.nseg = 1;
    a.W[0] = (const uint8_t *)(m->output.dec ? m->output.dec : m->output.d); a.N[0] = m->hp.n_vocab; a.Y[0] = m->logits;
    return kcpp_gemv_dec(m->output.dec ? KT_Q8_0 : m->output.type, &a, 0, 1, rows_per_wave(m->hp.n_vocab, 0), m->stream);
}

// run layers [il0, il1) on m->x for T tokens (T <= ub).  n_past via pos_dev when graph-replayed.
static int forward_layers(kcpp_model *m, int T, int n_past, bool dev_pos) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd, F = hp.n_ff, H = hp.n_head, HKV = hp.n_head_kv, D = E / H, EKV = HKV * D;
    const int64_t LQ = E + 2 * EKV;
    hipStream_t s = m->stream;
    const float kq_scale = 1.0f / sqrtf((float)D);
    const int32_t *posp = dev_pos ? m->pos_dev : nullptr;
    // a layer's attn_norm Q8_K activation already formed by the previous layer's down GEMM (gemm_w_norm)
    auto qkv_q8k = [](const KTensor *t) {
        return kcpp_vec_dot_type(t[1].type) == KT_Q8_K && kcpp_vec_dot_type(t[2].type) == KT_Q8_K &&
               kcpp_vec_dot_type(t[3].type) == KT_Q8_K;
    };
    bool pre_normed = false;
    for (int il = m->il0; il < m->il1; ++il) {
        KLayer &L = m->layers[il - m->il0];
        const KTensor *t = L.t;
        const bool kq = kcpp_vec_dot_type(t[1].type) == KT_Q8_K;
        bool roped = false;                          // q16 and this step's K/V rows already written
        const bool normed = pre_normed;
        pre_normed = false;
        // attn_norm -> act (Q8_K fused, or f32 then Q8_0)
        if (qkv_q8k(t)) {
            if (!normed) RC(kcpp_rms_norm(m->x, E, (const float *)t[0].d, nullptr, E, m->act, E, T, hp.eps, s));
            if (L.nqkv >= 2) {                       // q|k(|v) rows back to back: one GEMM
                KTensor f = t[1];
                f.N = E + (L.nqkv - 1) * EKV;
                if (L.nqkv == 2 && T > 8 && m->side) {
                    // attn_v (another type: Q6_K on the more-bits layers) on the side stream with its own
                    // workspace, concurrently with the q|k GEMM: its 64-workgroup grid alone leaves CUs idle
                    if (!m->gemm_ws2) {
                        const size_t sz = (size_t)kcpp_gemm_workspace_bytes(t[3].type, E, EKV, m->ub);
                        RT_CHECK(hipMalloc(&m->gemm_ws2, sz));
                    }
                    RT_CHECK(hipEventRecord(m->ev_fork, s));
                    RT_CHECK(hipStreamWaitEvent(m->side, m->ev_fork, 0));
                    RC(gemm_w(t[3], nullptr, m->act, T, m->qkv + E + EKV, LQ, nullptr, 0, 0, m->gemm_ws2, m->side));
                    RC(matmul(m, f, nullptr, m->act, T, m->qkv, LQ, nullptr, 0, 0));
                    RT_CHECK(hipEventRecord(m->ev_join, m->side));
                    RT_CHECK(hipStreamWaitEvent(s, m->ev_join, 0));
                } else {
                    RC(matmul(m, f, nullptr, m->act, T, m->qkv, LQ, nullptr, 0, 0));
                    if (L.nqkv == 2) RC(matmul(m, t[3], nullptr, m->act, T, m->qkv + E + EKV, LQ, nullptr, 0, 0));
                }
            } else {
                RC(matmul(m, t[1], nullptr, m->act, T, m->qkv, LQ, nullptr, 0, 0));
                RC(matmul(m, t[2], nullptr, m->act, T, m->qkv + E, LQ, nullptr, 0, 0));
                RC(matmul(m, t[3], nullptr, m->act, T, m->qkv + E + EKV, LQ, nullptr, 0, 0));
            }
        } else if (m->q80t) {                        // Q8_0 tile layout: norm + TA quantization, one q|k|v launch
            RC(kcpp_rms_norm_q80t(m->x, E, (const float *)t[0].d, m->act, E, T, hp.eps, s));
            if (m->lanes.empty()) {
                const void *Wq[3] = {t[1].d, t[2].d, t[3].d};
                const int64_t Nq[3] = {E, EKV, EKV};
                if (m->kv_tk == KT_F16) {          // rope + the f16 K/V stores in the GEMM's epilogue
                    RC(kcpp_gemm_q80t_qkv_rope(Wq, Nq, E, m->act, T, m->rope_tab, n_past, posp, (int)D, m->q16, L.kc,
                                               L.vc, m->gemm_ws, s));
                    roped = true;
                } else {
                    RC(kcpp_gemm_q80t(Wq, Nq, 3, nullptr, E, m->act, T, m->qkv, LQ, nullptr, 0, 0, nullptr, m->gemm_ws, s));
                }
            } else {
                for (int j = 1; j <= 3; ++j)
                    RC(matmul(m, t[j], nullptr, m->act, T, m->qkv + (j == 1 ? 0 : (j == 2 ? E : E + EKV)), LQ, nullptr, 0, 0));
            }
        } else if (T > 8 && T <= 32 && m->lanes.empty() && t[1].type == KT_Q8_0 && t[2].type == KT_Q8_0 && t[3].type == KT_Q8_0 && E % 128 == 0 &&
                   EKV % 128 == 0) {                 // small-batch Q8_0: one quantization, one q|k|v launch
            RC(kcpp_rms_norm_q80(m->x, E, (const float *)t[0].d, m->act, E, T, hp.eps, s));
            const void *Wq[3] = {t[1].d, t[2].d, t[3].d};
            const int64_t Nq[3] = {E, EKV, EKV};
            RC(kcpp_gemm_q80_segs(Wq, Nq, 3, E, m->act, T, m->qkv, LQ, m->gemm_ws, s));
        } else {
            RC(kcpp_rms_norm(m->x, E, (const float *)t[0].d, m->attn, E, nullptr, E, T, hp.eps, s));
            for (int j = 1; j <= 3; ++j) {
                RC(kcpp_quantize_act(kcpp_vec_dot_type(t[j].type), m->attn, E, m->act, E, T, s));
                const int64_t off = j == 1 ? 0 : (j == 2 ? E : E + EKV);
                RC(matmul(m, t[j], nullptr, m->act, T, m->qkv + off, LQ, nullptr, 0, 0));
            }
        }
        const bool kvq = m->kv_tk != KT_F16;
        if (kvq) {   // quantized cache: f32 rope in place, quantize K/V rows into the cache, Q8_0-dot attention
            RC(kcpp_rope_qk_inplace(m->qkv, LQ, T, (int)H, (int)HKV, (int)D, n_past, posp, m->rope_tab, s));
            RC(kcpp_kv_store_q(m->kv_tk, m->kv_tv, m->qkv, LQ, E, E + EKV, T, EKV, L.kc, L.vc, hp.n_ctx, n_past, posp, s));
        } else if (!roped) {
            RC(kcpp_rope_kv(m->qkv, LQ, nullptr, m->q16, L.kc, L.vc, T, (int)H, (int)HKV, (int)D, n_past, posp, m->rope_tab, s));
        }
        const bool woq = kcpp_vec_dot_type(t[4].type) == KT_Q8_K && !m->fa_exact && !kvq;
        // Q8_0 tile layout, ubatch > 16: attention writes attn_output's KT_Q8_0_TA activation itself (keys split
        // over the grid for short ubatches)
        bool attn_q = false;
        // (row-split lanes too: attention is not split, and wo's lanes read the same activation)
        if (m->q80t && !kvq && !m->fa_exact && t[4].type == KT_Q8_0_T && (T == 1 || (T > 16 && !posp))) {
            const int rc = T == 1 ? kcpp_flash_attn_dec_ta(m->q16, L.kc, L.vc, nullptr, m->act, m->fa_ws, (int)H, (int)HKV,
                                                           (int)D, n_past, posp, hp.n_ctx, kq_scale, s)
                                  : kcpp_flash_attn_prefill_mfma_ex(m->q16, L.kc, L.vc, nullptr, m->act, m->fa_ws, T,
                                                                    (int)H, (int)HKV, (int)D, n_past, kq_scale, s);
            if (rc != 0 && rc != -3) return rc;
            attn_q = rc == 0;
        }
        if (attn_q) {
        } else if (kvq)
            RC(kcpp_flash_attn_q(m->kv_tk, m->kv_tv, m->qkv, LQ, L.kc, L.vc, m->attn, T, (int)H, (int)HKV, (int)D, hp.n_ctx,
                                 n_past, posp, kq_scale, s));
        else if (m->fa_exact)
            RC(kcpp_flash_attn_exact(m->q16, L.kc, L.vc, m->attn, T, (int)H, (int)HKV, (int)D, n_past, posp, kq_scale, s));
        else
            RC(kcpp_flash_attn(m->q16, L.kc, L.vc, m->attn, (woq && T <= 16) ? m->act : nullptr, m->fa_ws, T, (int)H,
                               (int)HKV, (int)D, n_past, posp, hp.n_ctx, kq_scale, 0, s));
        if (!(woq && T <= 16) && !attn_q) RC(kcpp_quantize_act(kcpp_vec_dot_type(t[4].type), m->attn, E, m->act, E, T, s));
        const bool gq = kcpp_vec_dot_type(t[6].type) == KT_Q8_K && kcpp_vec_dot_type(t[7].type) == KT_Q8_K;
        // x += wo . attn; dense Q8_K FFNs: ffn_norm's activation formed with it (in wo's split-K reduce)
        const bool wo_norm = hp.n_expert <= 0 && !m->q80t && gq && norm_foldable(m, t[4], T);
        if (wo_norm)
            RC(gemm_w_norm(t[4], m->act, T, m->x, E, m->x, E, m->gemm_ws, s, (const float *)t[5].d, hp.eps, m->act));
        else
            RC(matmul(m, t[4], nullptr, m->act, T, m->x, E, m->x, E, 0));
        if (hp.n_expert > 0) { RC(T == 1 ? moe_dec(m, L) : moe_prefill(m, L, T)); continue; }   // T == 1: no host sync (graphs)
        if (m->q80t) {
            // ffn_norm -> TA quantization; gate|up with silu(g) u quantized to the TA activation of down in the GEMM's
            // epilogue (one launch); down with the residual
            RC(kcpp_rms_norm_q80t(m->x, E, (const float *)t[5].d, m->act, E, T, hp.eps, s));
            if (m->lanes.empty()) {
                RC(kcpp_gemm_q80t(&t[6].d, &F, 1, t[7].d, E, m->act, T, nullptr, 0, nullptr, 0, 1, m->act2, m->gemm_ws, s));
            } else {
                RC(matmul(m, t[6], &t[7], m->act, T, m->h, F, nullptr, 0, 1));          // h = silu(g) * u
                RC(kcpp_quantize_act(KT_Q8_0_TA, m->h, F, m->act2, F, T, s));
            }
            RC(matmul(m, t[8], nullptr, m->act2, T, m->x, E, m->x, E, 0));               // x += down . h
            continue;
        }
        if (gq) {
            if (!wo_norm) RC(kcpp_rms_norm(m->x, E, (const float *)t[5].d, nullptr, E, m->act, E, T, hp.eps, s));
        } else if (kcpp_vec_dot_type(t[6].type) == KT_Q8_0 && kcpp_vec_dot_type(t[7].type) == KT_Q8_0) {
            RC(kcpp_rms_norm_q80(m->x, E, (const float *)t[5].d, m->act, E, T, hp.eps, s));
        } else {
            RC(kcpp_rms_norm(m->x, E, (const float *)t[5].d, m->attn, E, nullptr, E, T, hp.eps, s));
            RC(kcpp_quantize_act(kcpp_vec_dot_type(t[6].type), m->attn, E, m->act, E, T, s));
        }
        if (L.glu_fused && kcpp_vec_dot_type(t[8].type) == KT_Q8_K) {
            KTensor f = t[6];                          // gate|up rows back to back: one GEMM, then
            f.N = 2 * F;                               // silu(g)*u fused into the Q8_K quantization
            RC(matmul(m, f, nullptr, m->act, T, m->hglu, 2 * F, nullptr, 0, 0));
            RC(kcpp_quantize_act_glu(m->hglu, 2 * F, F, m->act2, F, T, s));
        } else if (T <= 32 && m->lanes.empty() && t[6].type == KT_Q8_0 && t[7].type == KT_Q8_0 && kcpp_vec_dot_type(t[8].type) == KT_Q8_0 &&
                   F % 32 == 0) {
            RC(kcpp_gemm_q80_glu_q80(t[6].d, t[7].d, E, F, m->act, T, m->act2, m->gemm_ws, s));   // Q8_0(silu(g) * u)
        } else {
            if (t[6].type == t[7].type) {
                RC(matmul(m, t[6], &t[7], m->act, T, m->h, F, nullptr, 0, 1));          // h = silu(g) * u
            } else {
                RC(matmul(m, t[6], nullptr, m->act, T, m->h, F, nullptr, 0, 0));
                RC(matmul(m, t[7], nullptr, m->act, T, m->hglu, F, nullptr, 0, 0));
                RC(kcpp_silu_mul(m->h, m->h, m->hglu, (int64_t)T * F, s));
            }
            RC(kcpp_quantize_act(kcpp_vec_dot_type(t[8].type), m->h, F, m->act2, F, T, s));
        }
        // x += down . h; the next layer's attn_norm activation formed with it when that layer takes Q8_K
        const KTensor *tn = il + 1 < m->il1 ? m->layers[il + 1 - m->il0].t : nullptr;
        if (tn && qkv_q8k(tn) && norm_foldable(m, t[8], T)) {
            RC(gemm_w_norm(t[8], m->act2, T, m->x, E, m->x, E, m->gemm_ws, s, (const float *)tn[0].d, hp.eps, m->act));
            pre_normed = true;
        } else {
            RC(matmul(m, t[8], nullptr, m->act2, T, m->x, E, m->x, E, 0));
        }
    }
    return 0;
}

static int head(kcpp_model *m, int T) {
    const kcpp_hparams &hp = m->hp;
    const int64_t E = hp.n_embd;
    const float *last = m->x + (int64_t)(T - 1) * E;
    if (kcpp_vec_dot_type(m->output.type) == KT_Q8_K) {
        RC(kcpp_rms_norm(last, E, (const float *)m->output_norm.d, nullptr, E, m->act, E, 1, hp.eps, m->stream));
    } else {
        RC(kcpp_rms_norm(last, E, (const float *)m->output_norm.d, m->attn, E, nullptr, E, 1, hp.eps, m->stream));
        RC(kcpp_quantize_act(kcpp_vec_dot_type(m->output.type), m->attn, E, m->act, E, 1, m->stream));
    }
    RC(matmul(m, m->output, nullptr, m->act, 1, m->logits, hp.n_vocab, nullptr, 0, 0));
    return 0;
}

// full single-token step with the inputs read from device memory (graph-capturable)
static int decode_step_dev(kcpp_model *m) {
    const kcpp_hparams &hp = m->hp;
    if (m->has_embed)
        RC(kcpp_get_rows(m->tok_embd.type, m->tok_embd.d, hp.n_embd, hp.n_vocab, m->tok_dev, 1, m->x, hp.n_embd,
                         m->stream));
    if (m->fused_decode && m->kv_tk == KT_F16 && !m->q81 && (!m->q80t || m->q80_dec)) {
        RC(forward_layers_dec(m));
        if (m->has_output) RC(head_dec(m));
    } else {
        RC(forward_layers(m, 1, 0, true));
        if (m->has_output) RC(head(m, 1));
    }
    // greedy token on device (tok_dev for the next step); the device position steps to the next token's, so a
    // replay needs no host-to-device copy when tokens follow each other (the graph holds no memcpy node)
    if (m->has_output) RC(launch_argmax(m, true));
    else RC(launch_pos_step(m));
    return 0;
}

// pos_dev <- n_past unless the device already holds it (the previous single-token step advanced it).  The caller
// records n_past + 1 in pos_val only once the step is enqueued (a failed enqueue leaves pos_val = -1).
static int set_pos(kcpp_model *m, int n_past) {
    if (m->pos_val != n_past) {
        m->pos_val = -1;
        m->pin[1] = n_past;
        RT_CHECK(hipMemcpyAsync(m->pos_dev, &m->pin[1], 4, hipMemcpyHostToDevice, m->stream));
    }
    return 0;
}
// one single-token step at n_past (tok_dev already set): graph replay or eager; advances pos_val on success
static int step_one(kcpp_model *m, int n_past) {
    m->pos_val = m->pos_val == n_past ? n_past : -1;
    m->dec_short = n_past + 1 <= m->short_max;
    if (m->use_graphs) {
        RC(ensure_graph(m));
        RC(set_pos(m, n_past));
        const hipError_t e = hipGraphLaunch(m->g_exec[m->dec_short], m->stream);
        if (e != hipSuccess) { m->pos_val = -1; RT_CHECK(e); }
    } else {
        RC(set_pos(m, n_past));
        const int rc = decode_step_dev(m);
        if (rc) { m->pos_val = -1; return rc; }
    }
    m->pos_val = n_past + 1;          // decode_step_dev advanced the device position
    return 0;
}

// single-token graph: embedding of tok_dev, layers at position pos_dev, head, argmax, pos_dev + 1
static int ensure_graph(kcpp_model *m) {
    if (m->g_exec[m->dec_short]) return 0;
    hipGraph_t g;
    RT_CHECK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
    int rc = decode_step_dev(m);
    hipError_t e = hipStreamEndCapture(m->stream, &g);
    if (rc || e != hipSuccess) { g_err = "graph capture failed"; return rc ? rc : -3; }
    RT_CHECK(hipGraphInstantiate(&m->g_exec[m->dec_short], g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    return 0;
}

// the linked single-token step (layer-split engine, expose.cpp): k_link_wait (pull this stage's input from the
// producer stage, device-side), the step, k_link_publish -- one graph replay, no host call between stages
int kcpp_model_set_link(kcpp_model *m, const KLink *L) {
    for (auto &gx : m->g_link)
        if (gx) { (void)hipGraphExecDestroy(gx); gx = nullptr; }
    m->has_link = L != nullptr;
    if (L) m->link = *L;
    return 0;
}

static int ensure_graph_linked(kcpp_model *m) {
    if (m->g_link[m->dec_short]) return 0;
    hipGraph_t g;
    RT_CHECK(hipStreamBeginCapture(m->stream, hipStreamCaptureModeThreadLocal));
    int rc = kcpp_link_wait(m->link, m->stream);
    if (!rc) rc = decode_step_dev(m);
    if (!rc) rc = kcpp_link_publish(m->link, m->stream);
    hipError_t e = hipStreamEndCapture(m->stream, &g);
    if (rc || e != hipSuccess) { g_err = "linked graph capture failed"; return rc ? rc : -3; }
    RT_CHECK(hipGraphInstantiate(&m->g_link[m->dec_short], g, nullptr, nullptr, 0));
    hipGraphDestroy(g);
    return 0;
}

int kcpp_model_step_linked(kcpp_model *m, int n_past) {
    if (!m->has_link || !m->use_graphs) { g_err = "linked step: no link or graphs off"; return -3; }
    if (n_past + 1 > m->hp.n_ctx) { g_err = "context overflow"; return -2; }
    RT_CHECK(hipSetDevice(m->device));
    m->pos_val = m->pos_val == n_past ? n_past : -1;
    m->dec_short = n_past + 1 <= m->short_max;
    RC(ensure_graph_linked(m));
    RC(set_pos(m, n_past));
    const hipError_t e = hipGraphLaunch(m->g_link[m->dec_short], m->stream);
    if (e != hipSuccess) { m->pos_val = -1; RT_CHECK(e); }
    m->pos_val = n_past + 1;
    return 0;
}

extern "C" int kcpp_model_forward_hidden(kcpp_model *m, int T, int n_past) {
    RT_CHECK(hipSetDevice(m->device));
    return forward_layers(m, T, n_past, false);
}

// enqueue one llama_decode of T tokens on the stage's stream (no host synchronisation): the pipeline driver
// (expose.cpp) chains stages with events / RCCL and synchronises once per step
static int decode_enqueue(kcpp_model *m, const int32_t *tokens, int T, int n_past) {
    const kcpp_hparams &hp = m->hp;
    if (T < 1 || n_past + T > hp.n_ctx) { g_err = "context overflow"; return -2; }
    if (m->has_embed && !tokens) { g_err = "decode: stage owns the embedding but tokens == NULL"; return -2; }
    if (T == 1) {
        m->pin[0] = m->has_embed ? tokens[0] : 0;
        if (m->has_embed) RT_CHECK(hipMemcpyAsync(m->tok_dev, &m->pin[0], 4, hipMemcpyHostToDevice, m->stream));
        RC(step_one(m, n_past));
    } else {
        // split into ubatches (llama_decode_internal, src/llama.cpp:17187-17201)
        for (int i = 0; i < T; i += m->ub) {
            const int t = std::min(m->ub, T - i);
            if (m->has_embed) {
                RT_CHECK(hipMemcpyAsync(m->tok_dev, tokens + i, (size_t)t * 4, hipMemcpyHostToDevice, m->stream));
                RC(kcpp_get_rows(m->tok_embd.type, m->tok_embd.d, hp.n_embd, hp.n_vocab, m->tok_dev, t, m->x, hp.n_embd,
                                 m->stream));
            }
            RC(forward_layers(m, t, n_past + i, false));
            if (m->has_output && i + t == T) RC(head(m, t));
        }
    }
    return 0;
}

extern "C" int kcpp_model_decode_async(kcpp_model *m, const int32_t *tokens, int T, int n_past) {
    RT_CHECK(hipSetDevice(m->device));
    return decode_enqueue(m, tokens, T, n_past);
}

extern "C" int kcpp_model_decode(kcpp_model *m, const int32_t *tokens, int T, int n_past, float *logits_host) {
    RT_CHECK(hipSetDevice(m->device));
    RC(decode_enqueue(m, tokens, T, n_past));
    if (m->has_output && logits_host) {
        RT_CHECK(hipMemcpyAsync(logits_host, m->logits, (size_t)m->hp.n_vocab * 4, hipMemcpyDeviceToHost, m->stream));
    }
    RT_CHECK(hipStreamSynchronize(m->stream));
    return 0;
}
extern "C" int kcpp_model_device(kcpp_model *m) { return m->device; }

// greedy argmax over the logits (first index wins ties, like the CPU sampler's top-1):
// stage 1, ARGMAX_BLOCKS workgroups reduce strided slices to (value, index) pairs; stage 2, one
// workgroup reduces those and writes the token to out[0] (and to tok[0] when given: the next
// decode step's embedding input, so a greedy loop never round-trips the token through the host).
#define ARGMAX_BLOCKS 256
__device__ __forceinline__ void amax_merge(float &v, int &i, float v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void amax_block(float &v, int &i) {
    for (int o = 32; o > 0; o >>= 1) amax_merge(v, i, __shfl_xor(v, o, 64), __shfl_xor(i, o, 64));
    __shared__ float sv[4];
    __shared__ int si[4];
    if ((threadIdx.x & 63) == 0) { sv[threadIdx.x >> 6] = v; si[threadIdx.x >> 6] = i; }
    __syncthreads();
    v = sv[0]; i = si[0];
    for (int w = 1; w < 4; ++w) amax_merge(v, i, sv[w], si[w]);
}
__global__ void __launch_bounds__(256) k_argmax_part(const float *__restrict__ x, int n, float2 *part) {
    float v = -INFINITY; int i = 0x7fffffff;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < n; j += ARGMAX_BLOCKS * 256) amax_merge(v, i, x[j], j);
    amax_block(v, i);
    if (threadIdx.x == 0) part[blockIdx.x] = make_float2(v, __int_as_float(i));
}
__global__ void __launch_bounds__(256) k_argmax_final(const float2 *__restrict__ part, int32_t *out, int32_t *tok,
                                                      int32_t *pos) {
    const float2 p = part[threadIdx.x];
    float v = p.x; int i = __float_as_int(p.y);
    amax_block(v, i);
    if (i == 0x7fffffff) i = 0;               // all-NaN logits: no comparison succeeded; keep the token id valid
    if (threadIdx.x == 0) {
        out[0] = i;
        if (tok) tok[0] = i;
        if (pos) { pos[0] += 1; pos[1] += 1; }   // the next single-token step's position and epoch
    }
}
__global__ void k_pos_step(int32_t *pos) { pos[0] += 1; pos[1] += 1; }
static int launch_argmax(kcpp_model *m, bool step_pos) {
    hipLaunchKernelGGL(k_argmax_part, dim3(ARGMAX_BLOCKS), dim3(256), 0, m->stream, m->logits, m->hp.n_vocab,
                       (float2 *)m->argmax_ws);
    hipLaunchKernelGGL(k_argmax_final, dim3(1), dim3(256), 0, m->stream, (const float2 *)m->argmax_ws, m->argmax_dev,
                       m->has_embed ? m->tok_dev : nullptr, step_pos ? m->pos_dev : nullptr);
    RT_CHECK(hipGetLastError());
    return 0;
}
static int launch_pos_step(kcpp_model *m) {
    hipLaunchKernelGGL(k_pos_step, dim3(1), dim3(1), 0, m->stream, m->pos_dev);
    RT_CHECK(hipGetLastError());
    return 0;
}

// pipeline greedy steps without the host (expose.cpp greedy_step): the last stage's argmax on device, and a
// single-token step whose input token (stage 0) is already in tok_dev
extern "C" int kcpp_model_argmax_async(kcpp_model *m) {
    if (!m->has_output) return -1;
    RT_CHECK(hipSetDevice(m->device));
    return launch_argmax(m, false);
}
extern "C" int kcpp_model_step_dev(kcpp_model *m, int n_past) {
    if (n_past + 1 > m->hp.n_ctx) { g_err = "context overflow"; return -2; }
    RT_CHECK(hipSetDevice(m->device));
    return step_one(m, n_past);
}
extern "C" int32_t *kcpp_model_token_dev(kcpp_model *m) { return m->tok_dev; }
extern "C" int32_t *kcpp_model_argmax_dev(kcpp_model *m) { return m->argmax_dev; }

// the token the last single-token step's own argmax left in argmax_dev (decode_step_dev ends every step with it): a
// 4-byte read, no kernel launch
extern "C" int kcpp_model_read_argmax(kcpp_model *m, int32_t *token_out) {
    if (!m->has_output) return -1;
    RT_CHECK(hipSetDevice(m->device));
    RT_CHECK(hipMemcpyAsync(&m->pin[2], m->argmax_dev, 4, hipMemcpyDeviceToHost, m->stream));
    RT_CHECK(hipStreamSynchronize(m->stream));
    *token_out = m->pin[2];
    return 0;
}
extern "C" int kcpp_model_argmax(kcpp_model *m, int32_t *token_out) {
    if (!m->has_output) return -1;
    RT_CHECK(hipSetDevice(m->device));
    RC(launch_argmax(m, false));
    RT_CHECK(hipMemcpyAsync(&m->pin[2], m->argmax_dev, 4, hipMemcpyDeviceToHost, m->stream));
    RT_CHECK(hipStreamSynchronize(m->stream));
    *token_out = m->pin[2];
    return 0;
}

// Greedy decode with the host one step behind the device: enqueue this step (its input is the previous step's device
// argmax, in place), then the 4-byte read of its token into a pinned ring slot, and return the PREVIOUS step's token
// once its read has landed -- the next step is already queued when the host waits, so no per-token bubble (a serving
// loop checks its stop conditions on token k while step k + 1 runs).  *token_out = -1 on the first call after a drain;
// kcpp_model_greedy_drain returns the last step's token and resets the ring.
extern "C" int kcpp_model_decode_greedy_lagged(kcpp_model *m, int n_past, int32_t *token_out) {
    if (!m->has_embed || !m->has_output) { g_err = "decode_greedy needs embedding and output on this stage"; return -2; }
    if (n_past + 1 > m->hp.n_ctx) { g_err = "context overflow"; return -2; }
    RT_CHECK(hipSetDevice(m->device));
    for (hipEvent_t &ev : m->ev_tok)
        if (!ev) RT_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    RC(step_one(m, n_past));
    const int slot = m->lag_k & 1;
    RT_CHECK(hipMemcpyAsync(&m->pin[4 + slot], m->argmax_dev, 4, hipMemcpyDeviceToHost, m->stream));
    RT_CHECK(hipEventRecord(m->ev_tok[slot], m->stream));
    *token_out = -1;
    if (m->lag_k > 0) {
        RT_CHECK(hipEventSynchronize(m->ev_tok[slot ^ 1]));
        *token_out = m->pin[4 + (slot ^ 1)];
    }
    ++m->lag_k;
    return 0;
}
extern "C" int kcpp_model_greedy_drain(kcpp_model *m, int32_t *token_out) {
    RT_CHECK(hipSetDevice(m->device));
    *token_out = -1;
    if (m->lag_k > 0) {
        RT_CHECK(hipEventSynchronize(m->ev_tok[(m->lag_k - 1) & 1]));
        *token_out = m->pin[4 + ((m->lag_k - 1) & 1)];
    }
    m->lag_k = 0;
    return 0;
}

// One greedy step: the input token is the previous argmax (already in tok_dev), the step's own
// argmax is computed inside the same graph replay and returned.  One host sync per token.
extern "C" int kcpp_model_decode_greedy(kcpp_model *m, int n_past, int32_t *token_out) {
    if (!m->has_embed || !m->has_output) { g_err = "decode_greedy needs embedding and output on this stage"; return -2; }
    if (n_past + 1 > m->hp.n_ctx) { g_err = "context overflow"; return -2; }
    RT_CHECK(hipSetDevice(m->device));
    RC(step_one(m, n_past));
    RT_CHECK(hipMemcpyAsync(&m->pin[2], m->argmax_dev, 4, hipMemcpyDeviceToHost, m->stream));
    RT_CHECK(hipStreamSynchronize(m->stream));
    *token_out = m->pin[2];
    return 0;
}
