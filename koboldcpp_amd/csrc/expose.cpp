// expose.cpp -- the koboldcpp C ABI (include/kcpp_expose.h) over the MI355X Llama runtime.
//
// Reference behaviour (gpttype_adapter.cpp / expose.cpp):
//   load_model  -> GGUF (general.architecture "llama"), layer split over the visible GPUs by
//                  tensor_split exactly like llm_load_tensors (src/llama.cpp:7000-7036), weights uploaded
//                  from the mmap'd file in ggml block layout (repacked on the device).
//   generate    -> prompt and memory tokenized (BOS per the vocab) and assembled as gpttype_adapter.cpp:2794-2887
//                  (prompt cut from the front, memory kept), context shifting when enabled (PurgeMissingTokens,
//                  :1504-1571: a removed middle span leaves the KV cache by a K-shift), the KV prefix shared with the previous request reused
//                  ("fast forward", gpttype_adapter.cpp:2929-2945), prefill in ubatches, sampling, streaming
//                  text through new_token()/get_pending_output(), stop on EOS / stop sequences / max_length /
//                  abort; last_process_time / last_eval_time in ms per token (gpttype_adapter.cpp:3513-3526).
// Sampling is host code (as in the reference): repetition penalty over rep_pen_range, logit biases,
// top-k, top-p, min-p, temperature, seeded mt19937; temperature <= 0 or top_k == 1 is greedy on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/kcpp_expose.h"
#include "../../include/kcpp_mi355x.h"
#include "../../include/kcpp_synth.h"
#include "gguf.h"
#include "tokenizer.h"

namespace {

struct Engine {
    gguf::File file;
    Tokenizer tok;
    kcpp_hparams hp{};
    std::vector<int> types;
    std::vector<kcpp_model *> stages;
    std::vector<float *> hidden;            // per stage residual stream (device)
    int ub = 512;
    bool use_contextshift = false;
    std::vector<int> ctx;                   // tokens whose K/V are in the caches
    std::vector<float> logits;
    ~Engine() { for (auto *m : stages) kcpp_model_free(m); }
};

std::unique_ptr<Engine> g_eng;
std::mutex g_out_mtx;
std::vector<std::string> g_generated;       // streamed pieces (new_token / get_stream_count)
std::string g_concat, g_result, g_pending;
std::atomic<bool> g_finished{true}, g_abort{false};
float g_last_eval = 0, g_last_process = 0;
int g_last_count = 0, g_last_seed = 0, g_total_gens = 0;
int g_last_stop = KCPP_STOP_INVALID;
std::vector<int> g_count_ids;

const char *tname(int il, int j) {
    static const char *n[9] = {"attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "ffn_norm", "ffn_gate", "ffn_up", "ffn_down"};
    (void)il;
    return n[j];
}

bool supported_type(int t) {
    return t == KT_F32 || t == KT_F16 || t == KT_Q4_0 || t == KT_Q8_0 || t == KT_Q4_K || t == KT_Q5_K || t == KT_Q6_K;
}

// layer -> device (src/llama.cpp:7010-7036, all layers offloaded)
std::vector<int> split_layers(int n_layer, int n_dev, const float *ts) {
    std::vector<float> sp(n_dev);
    bool zero = true;
    for (int i = 0; i < n_dev; ++i) zero &= ts[i] == 0.0f;
    float acc = 0;
    for (int i = 0; i < n_dev; ++i) { acc += zero ? 1.0f : ts[i]; sp[i] = acc; }
    for (int i = 0; i < n_dev; ++i) sp[i] /= acc;
    const int act = n_layer + 1;
    std::vector<int> dev(n_layer + 1);
    for (int i = 0; i <= n_layer; ++i) {
        const int d = (int)(std::upper_bound(sp.begin(), sp.end(), (float)i / act) - sp.begin());
        dev[i] = std::min(d, n_dev - 1);
    }
    return dev;   // dev[n_layer] = output head's device
}

// run tokens [i0, i0+T) through all stages (ubatch granularity); last stage leaves logits on device
int forward(Engine &e, const int32_t *toks, int T, int n_past) {
    for (int i = 0; i < T; i += e.ub) {
        const int t = std::min(e.ub, T - i);
        for (size_t s = 0; s < e.stages.size(); ++s) {
            if (s > 0) {
                const int rc = kcpp_model_hidden_io(e.stages[s], e.hidden[s - 1], (int64_t)t * e.hp.n_embd, 0, 0);
                if (rc) return rc;
            }
            const int rc = kcpp_model_decode(e.stages[s], s == 0 ? toks + i : nullptr, t, n_past + i, nullptr);
            if (rc) return rc;
        }
    }
    return 0;
}

int sample(Engine &e, const generation_inputs &in, const std::vector<int> &recent, std::mt19937 &rng, bool greedy) {
    kcpp_model *last = e.stages.back();
    if (greedy && in.rep_pen <= 1.0f) {
        int32_t t = 0;
        kcpp_model_argmax(last, &t);
        return t;
    }
    // host sampling over the logits of the last position (the reference samples on the host too)
    e.logits.resize(e.hp.n_vocab);
    int32_t dummy;
    (void)dummy;
    {
        // re-run nothing: copy the head output of the last decode
        if (kcpp_model_read_logits(last, e.logits.data())) return e.tok.eos();
    }
    std::vector<float> &l = e.logits;
    for (int k = 0; k < KCPP_LOGIT_BIAS_MAX; ++k) {
        const logit_bias &b = in.logit_biases[k];
        if (b.token_id > 0 && b.token_id < (int)l.size() && b.bias != 0.0f) l[b.token_id] += b.bias;
    }
    if (in.rep_pen > 1.0f) {
        const int range = in.rep_pen_range > 0 ? in.rep_pen_range : (int)recent.size();
        for (int k = std::max(0, (int)recent.size() - range); k < (int)recent.size(); ++k) {
            float &v = l[recent[k]];
            v = v > 0 ? v / in.rep_pen : v * in.rep_pen;
        }
    }
    if (greedy) return (int)(std::max_element(l.begin(), l.end()) - l.begin());
    std::vector<int> idx(l.size());
    for (size_t k = 0; k < idx.size(); ++k) idx[k] = (int)k;
    const int topk = in.top_k > 0 ? std::min<int>(in.top_k, (int)idx.size()) : (int)idx.size();
    std::partial_sort(idx.begin(), idx.begin() + topk, idx.end(), [&](int a, int b) { return l[a] > l[b]; });
    idx.resize(topk);
    const float temp = in.temperature > 0 ? in.temperature : 1.0f;
    std::vector<double> p(idx.size());
    const double mx = l[idx[0]];
    double sum = 0;
    for (size_t k = 0; k < idx.size(); ++k) { p[k] = std::exp((l[idx[k]] - mx) / temp); sum += p[k]; }
    for (auto &v : p) v /= sum;
    size_t keep = p.size();
    if (in.top_p > 0 && in.top_p < 1) {
        double c = 0;
        for (size_t k = 0; k < p.size(); ++k) { c += p[k]; if (c >= in.top_p) { keep = k + 1; break; } }
    }
    if (in.min_p > 0) {
        size_t k2 = 0;
        while (k2 < keep && p[k2] >= in.min_p * p[0]) ++k2;
        keep = std::max<size_t>(1, k2);
    }
    double tot = 0;
    for (size_t k = 0; k < keep; ++k) tot += p[k];
    std::uniform_real_distribution<double> u(0.0, tot);
    double r = u(rng);
    for (size_t k = 0; k < keep; ++k) { r -= p[k]; if (r <= 0) return idx[k]; }
    return idx[keep - 1];
}


// ---- context shifting (restatement of model_adapter.cpp:337-430 and gpttype_adapter.cpp:1504-1571)
bool arr_start_with(const std::vector<int> &t, const std::vector<int> &q) {
    if (t.size() < q.size()) return false;
    for (size_t i = 0; i < q.size(); ++i)
        if (t[i] != q[i]) return false;
    return true;
}
int arr_find_index_of(const std::vector<int> &t, const std::vector<int> &q) {
    const int ss = (int)q.size(), tas = (int)t.size();
    if (tas < ss) return -1;
    for (int i = 0; i < tas; ++i) {
        bool fail = false;
        for (int k = 0; k < ss; ++k)
            if (i + k >= tas || t[i + k] != q[k]) { fail = true; break; }
        if (!fail) return i;
    }
    return -1;
}
// longest common contiguous run, first maximum in (i, j) order as the reference's full-table scan finds it;
// two rolling rows instead of the (m+1) x (n+1) table
std::vector<int> longest_common_subseq(const std::vector<int> &x, const std::vector<int> &y) {
    const int m = (int)x.size(), n = (int)y.size();
    std::vector<int> prev(n + 1, 0), cur(n + 1, 0);
    int best = 0, best_i = 0;
    for (int i = 1; i <= m; ++i) {
        cur[0] = 0;
        for (int j = 1; j <= n; ++j) {
            cur[j] = x[i - 1] == y[j - 1] ? prev[j - 1] + 1 : 0;
            if (cur[j] > best) { best = cur[j]; best_i = i; }
        }
        std::swap(prev, cur);
    }
    return std::vector<int>(x.begin() + (best_i - best), x.begin() + best_i);
}
// PurgeMissingTokens: when the new prompt is the old context with a middle span removed (the front end
// trimmed it to fit), erase that span from the KV cache (rows move down, K re-rotated) instead of
// re-processing everything after it.  Returns the number of erased positions.
int purge_missing_tokens(Engine &e, std::vector<int> &cur, const std::vector<int> &inp, int genamt, int nctx) {
    const int ShortfallThreshold = 200 + std::min(nctx / 30, 140);
    const int SlackAllowance = 60 + std::min(nctx / 60, 70);
    const int new_len = (int)inp.size();
    if (new_len == 0) return 0;
    int trimstart = 0;
    bool purgeneeded = true;
    for (int i = 0; i < (int)cur.size(); ++i) {
        if (cur[i] == inp[i]) trimstart += 1;
        else break;
        if (i + 2 >= new_len) { purgeneeded = false; break; }
    }
    if (!purgeneeded || new_len < 6 || cur.size() < 6 || new_len - trimstart < ShortfallThreshold) return 0;
    const int LCSTokThreshold = std::max(std::min((new_len - trimstart) - (genamt + SlackAllowance), (int)(nctx * 0.45)),
                                         ShortfallThreshold - SlackAllowance);
    const std::vector<int> cur_wo(cur.begin() + trimstart, cur.end()), new_wo(inp.begin() + trimstart, inp.end());
    const std::vector<int> shared = longest_common_subseq(cur_wo, new_wo);
    if ((int)shared.size() <= LCSTokThreshold || !arr_start_with(new_wo, shared)) return 0;
    const int found = arr_find_index_of(cur, shared);
    if (found < 0 || found <= trimstart) return 0;
    const int diff = found - trimstart;
    for (kcpp_model *m : e.stages)
        if (kcpp_model_kv_shift(m, trimstart, diff, (int)cur.size())) {
            fprintf(stderr, "[kcpp] context shift failed: %s\n", kcpp_last_error());
            cur.resize(trimstart);                 // KV beyond trimstart is no longer trusted: recompute it
            return 0;
        }
    // as the reference: the moved tail excludes the last token (it is re-evaluated by the fast forward)
    for (size_t i = trimstart + diff; i + 1 < cur.size(); ++i) cur[i - diff] = cur[i];
    cur.resize(cur.size() - diff);
    fprintf(stderr, "[kcpp] Context Shifting: Erased %d tokens at position %d\n", diff, trimstart + 1);
    return diff;
}

}  // namespace

extern "C" {

bool load_model(const load_model_inputs inputs) {
    auto e = std::make_unique<Engine>();
    std::string err;
    if (!inputs.model_filename || !e->file.open(inputs.model_filename, err)) {
        fprintf(stderr, "[kcpp] load_model: %s\n", err.c_str());
        return false;
    }
    gguf::File &f = e->file;
    const std::string arch = f.get_s("general.architecture", "");
    if (arch != "llama") { fprintf(stderr, "[kcpp] load_model: architecture '%s' not supported\n", arch.c_str()); return false; }
    if (!e->tok.init(f, err)) { fprintf(stderr, "[kcpp] load_model: %s\n", err.c_str()); return false; }
    const gguf::Tensor *emb = f.tensor("token_embd.weight");
    if (!emb) { fprintf(stderr, "[kcpp] load_model: no token_embd.weight\n"); return false; }
    kcpp_hparams &hp = e->hp;
    hp.n_embd = (int)f.get_i("llama.embedding_length", emb->ne[0]);
    hp.n_vocab = (int)emb->ne[1];
    hp.n_layer = (int)f.get_i("llama.block_count", 0);
    hp.n_ff = (int)f.get_i("llama.feed_forward_length", 0);
    hp.n_head = (int)f.get_i("llama.attention.head_count", 0);
    hp.n_head_kv = (int)f.get_i("llama.attention.head_count_kv", hp.n_head);
    hp.eps = (float)f.get_f("llama.attention.layer_norm_rms_epsilon", 1e-5);
    const bool user_rope = inputs.rope_freq_base > 0 && (inputs.rope_freq_base != 10000.0f || inputs.rope_freq_scale != 1.0f);
    hp.rope_base = user_rope ? inputs.rope_freq_base : (float)f.get_f("llama.rope.freq_base", 10000.0);
    hp.rope_freq_scale = user_rope && inputs.rope_freq_scale > 0 ? inputs.rope_freq_scale : 1.0f;
    hp.n_ctx = inputs.max_context_length > 0 ? inputs.max_context_length + 8 : 2048 + 8;
    if (hp.n_layer <= 0 || hp.n_head <= 0 || hp.n_embd / hp.n_head != 128) {
        fprintf(stderr, "[kcpp] load_model: need head_dim 128 (got n_embd %d / n_head %d)\n", hp.n_embd, hp.n_head);
        return false;
    }
    // mixture of experts (llm_load_hparams / llm_load_tensors, src/llama.cpp:5444-5445, 7176-7215)
    hp.n_expert = (int)f.get_i("llama.expert_count", 0);
    hp.n_expert_used = (int)f.get_i("llama.expert_used_count", 0);
    if (hp.n_expert > 0 && (hp.n_expert_used < 1 || hp.n_expert_used > hp.n_expert || hp.n_expert > 64)) {
        fprintf(stderr, "[kcpp] load_model: unsupported expert_count %d / expert_used_count %d\n", hp.n_expert,
                hp.n_expert_used);
        return false;
    }
    const int LW = hp.n_expert > 0 ? 10 : 9;
    // canonical tensor order: tok_embd, output_norm, output, layers x LW (+ ffn_gate_inp for MoE);
    // MoE gate/up/down are the 3-D *_exps tensors, or the older per-expert tensors concatenated
    struct Src { const gguf::Tensor *t = nullptr; int type = 0; int64_t bytes = 0; const uint8_t *data = nullptr; };
    std::vector<Src> ts(3 + LW * hp.n_layer);
    std::vector<std::vector<uint8_t>> merged;       // concatenated split experts (kept until upload)
    merged.reserve(3 * hp.n_layer);
    auto rbytes = [](const gguf::Tensor *t) {
        return t->ne[0] / ks_block_elems(t->type) * ks_block_bytes(t->type) * t->ne[1] * t->ne[2] * t->ne[3];
    };
    auto set = [&](int k, const gguf::Tensor *t) {
        if (t) { ts[k].t = t; ts[k].type = t->type; ts[k].bytes = rbytes(t); ts[k].data = t->data; }
    };
    set(0, emb);
    set(1, f.tensor("output_norm.weight"));
    set(2, f.tensor("output.weight"));
    if (!ts[2].t) set(2, emb);                     // tied embeddings
    static const char *exps[3] = {"ffn_gate_exps", "ffn_up_exps", "ffn_down_exps"};
    static const char *exp1[3] = {"ffn_gate", "ffn_up", "ffn_down"};
    for (int il = 0; il < hp.n_layer; ++il) {
        const std::string b = "blk." + std::to_string(il) + ".";
        for (int j = 0; j < 9; ++j) {
            const int k = 3 + LW * il + j;
            if (hp.n_expert == 0 || j < 6) { set(k, f.tensor(b + tname(il, j) + ".weight")); continue; }
            set(k, f.tensor(b + exps[j - 6] + ".weight"));
            if (ts[k].t) {
                if (ts[k].t->ne[2] != hp.n_expert) { fprintf(stderr, "[kcpp] load_model: %s: expert dim\n", ts[k].t->name.c_str()); return false; }
                continue;
            }
            std::vector<uint8_t> buf;                // blk.N.ffn_gate.E.weight, E = 0..n_expert-1
            for (int x = 0; x < hp.n_expert; ++x) {
                const gguf::Tensor *t = f.tensor(b + exp1[j - 6] + "." + std::to_string(x) + ".weight");
                if (!t || (x > 0 && t->type != ts[k].type)) { ts[k] = Src(); break; }
                if (x == 0) set(k, t);
                const int64_t nb = rbytes(t);
                buf.insert(buf.end(), t->data, t->data + nb);
            }
            if (ts[k].t) {
                merged.push_back(std::move(buf));
                ts[k].data = merged.back().data();
                ts[k].bytes = (int64_t)merged.back().size();
            }
        }
        if (LW == 10) set(3 + LW * il + 9, f.tensor(b + "ffn_gate_inp.weight"));
    }
    e->types.resize(ts.size());
    for (size_t k = 0; k < ts.size(); ++k) {
        if (!ts[k].t) { fprintf(stderr, "[kcpp] load_model: missing tensor #%zu\n", k); return false; }
        if (!supported_type(ts[k].type)) {
            fprintf(stderr, "[kcpp] load_model: tensor %s has unsupported type %d\n", ts[k].t->name.c_str(), ts[k].type);
            return false;
        }
        e->types[k] = ts[k].type;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) { fprintf(stderr, "[kcpp] load_model: no GPU\n"); return false; }
    const std::vector<int> ldev = split_layers(hp.n_layer, std::min(ndev, KCPP_TENSOR_SPLIT_MAX), inputs.tensor_split);
    e->ub = inputs.blasbatchsize > 0 ? std::min(inputs.blasbatchsize, 512) : 512;
    e->use_contextshift = inputs.use_contextshift;
    int il = 0;
    while (il < hp.n_layer || e->stages.empty()) {
        const int d = il < hp.n_layer ? ldev[il] : ldev[hp.n_layer];
        int il1 = il;
        while (il1 < hp.n_layer && ldev[il1] == d) ++il1;
        const bool last = il1 == hp.n_layer;
        if (last && ldev[hp.n_layer] != d) {
            fprintf(stderr, "[kcpp] load_model: output head must share the last layers' device\n");
            return false;
        }
        kcpp_model *m = kcpp_model_create(&hp, e->types.data(), d, il, il1, e->stages.empty(), last, e->ub);
        if (!m) { fprintf(stderr, "[kcpp] load_model: %s\n", kcpp_last_error()); return false; }
        e->stages.push_back(m);
        e->hidden.push_back(kcpp_model_hidden(m));
        if (e->stages.size() > 1) {
            hipSetDevice(d);
            hipDeviceEnablePeerAccess(ldev[std::max(0, il - 1)], 0);   // xGMI peer copies for the handoff
            (void)hipGetLastError();
        }
        il = il1;
        if (last) break;
    }
    for (size_t k = 0; k < ts.size(); ++k) {
        for (kcpp_model *m : e->stages)
            if (kcpp_model_set_tensor(m, (int)k, ts[k].data, ts[k].bytes)) {
                fprintf(stderr, "[kcpp] load_model: upload %s: %s\n", ts[k].t->name.c_str(), kcpp_last_error());
                return false;
            }
    }
    g_eng = std::move(e);
    return true;
}

generation_outputs generate(const generation_inputs in) {
    generation_outputs out;
    out.status = 0;
    out.stopreason = KCPP_STOP_INVALID;
    out.text = "";
    Engine *e = g_eng.get();
    if (!e) return out;
    {
        std::lock_guard<std::mutex> lk(g_out_mtx);
        g_generated.clear();
        g_concat.clear();
    }
    g_finished = false;
    g_abort = false;
    const int max_ctx = std::min(in.max_context_length > 0 ? in.max_context_length : e->hp.n_ctx - 8, e->hp.n_ctx - 8);
    const int max_len = std::max(1, std::min(in.max_length > 0 ? in.max_length : 64, max_ctx - 1));
    // prompt assembly as gpttype_adapter.cpp:2794-2887: the prompt is cut from the front (BOS kept first) to
    // leave room for max_length, the memory is kept whole (cut from its front only if it alone does not fit)
    // and the prompt makes room for it
    std::vector<int> toks = e->tok.encode(in.prompt ? in.prompt : "", true);
    const std::vector<int> bosv = e->tok.encode("", true);
    if ((int)toks.size() + max_len > max_ctx) {
        toks.erase(toks.begin(), toks.begin() + ((int)toks.size() - max_ctx + max_len));
        if (!bosv.empty() && !toks.empty()) toks[0] = bosv[0];
    }
    if (in.memory && in.memory[0]) {
        std::vector<int> mem = e->tok.encode(in.memory, true);
        if (!bosv.empty() && !toks.empty() && toks[0] == bosv[0]) toks.erase(toks.begin());
        if ((int)mem.size() + max_len + 4 > max_ctx) {
            mem.erase(mem.begin(), mem.begin() + ((int)mem.size() - max_ctx + max_len + 4));
            if (!bosv.empty() && !mem.empty()) mem[0] = bosv[0];
        }
        const int total = (int)(mem.size() + toks.size()) + max_len;
        if (total > max_ctx) {
            const int excess = total - max_ctx;
            if ((int)toks.size() >= excess) toks.erase(toks.begin(), toks.begin() + excess);
            else toks.clear();
        }
        toks.insert(toks.begin(), mem.begin(), mem.end());
    }
    if (toks.empty()) toks.push_back(e->tok.bos());
    if (e->use_contextshift) purge_missing_tokens(*e, e->ctx, toks, max_len, max_ctx);
    // fast forward over the shared prefix (recompute at least the last prompt token for its logits)
    size_t keep = 0;
    while (keep < toks.size() && keep < e->ctx.size() && e->ctx[keep] == toks[keep]) ++keep;
    if (keep == toks.size()) --keep;
    e->ctx.assign(toks.begin(), toks.begin() + keep);
    const auto t0 = std::chrono::steady_clock::now();
    if (forward(*e, toks.data() + keep, (int)(toks.size() - keep), (int)keep)) {
        fprintf(stderr, "[kcpp] generate: prefill failed: %s\n", kcpp_last_error());
        g_finished = true;
        return out;
    }
    e->ctx.insert(e->ctx.end(), toks.begin() + keep, toks.end());
    const auto t1 = std::chrono::steady_clock::now();
    std::mt19937 rng((uint32_t)(in.seed <= 0 ? (int)std::random_device{}() : in.seed));
    g_last_seed = in.seed;
    const bool greedy = in.temperature <= 0.0f || in.top_k == 1;
    std::vector<std::string> stops;
    for (int k = 0; k < KCPP_STOP_TOKEN_MAX; ++k)
        if (in.stop_sequence[k] && in.stop_sequence[k][0]) stops.emplace_back(in.stop_sequence[k]);
    int n_gen = 0, stop = KCPP_STOP_OUT_OF_TOKENS;
    for (; n_gen < max_len; ++n_gen) {
        if (g_abort) { stop = KCPP_STOP_CUSTOM_STOPPER; break; }
        const int t = sample(*e, in, e->ctx, rng, greedy);
        if (t == e->tok.eos() && !in.bypass_eos_token) { stop = KCPP_STOP_EOS_TOKEN_HIT; break; }
        const std::string piece = e->tok.piece(t);
        bool hit = false;
        {
            std::lock_guard<std::mutex> lk(g_out_mtx);
            g_generated.push_back(piece);
            g_concat += piece;
            for (const std::string &s : stops) {
                const size_t p = g_concat.find(s);
                if (p != std::string::npos) { g_concat.resize(p); hit = true; break; }
            }
        }
        if (hit) { stop = KCPP_STOP_CUSTOM_STOPPER; ++n_gen; break; }
        if ((int)e->ctx.size() >= e->hp.n_ctx - 1) break;
        const int32_t tt = t;
        if (forward(*e, &tt, 1, (int)e->ctx.size())) { fprintf(stderr, "[kcpp] generate: decode failed\n"); break; }
        e->ctx.push_back(t);
    }
    const auto t2 = std::chrono::steady_clock::now();
    const double tp = std::chrono::duration<double, std::milli>(t1 - t0).count();
    const double tg = std::chrono::duration<double, std::milli>(t2 - t1).count();
    const int np = (int)(toks.size() - keep);
    g_last_process = (float)(tp / std::max(1, np));
    g_last_eval = (float)(tg / std::max(1, n_gen));
    g_last_count = n_gen;
    g_last_stop = stop;
    g_total_gens += 1;
    {
        std::lock_guard<std::mutex> lk(g_out_mtx);
        g_result = g_concat;
    }
    out.status = 1;
    out.stopreason = stop;
    out.text = g_result.c_str();
    g_finished = true;
    return out;
}

const char *new_token(int idx) {
    std::lock_guard<std::mutex> lk(g_out_mtx);
    if (idx < 0 || idx >= (int)g_generated.size()) return nullptr;
    return g_generated[idx].c_str();
}
int get_stream_count(void) { std::lock_guard<std::mutex> lk(g_out_mtx); return (int)g_generated.size(); }
bool has_finished(void) { return g_finished; }
float get_last_eval_time(void) { return g_last_eval; }
float get_last_process_time(void) { return g_last_process; }
int get_last_token_count(void) { return g_last_count; }
int get_last_seed(void) { return g_last_seed; }
int get_total_gens(void) { return g_total_gens; }
int get_total_img_gens(void) { return 0; }
int get_last_stop_reason(void) { return g_last_stop; }
const char *get_pending_output(void) {
    std::lock_guard<std::mutex> lk(g_out_mtx);
    g_pending = g_concat;
    return g_pending.c_str();
}
bool abort_generate(void) { g_abort = true; return true; }
token_count_outputs token_count(const char *input, bool addbos) {
    token_count_outputs o;
    o.count = 0;
    o.ids = nullptr;
    if (!g_eng || !input) return o;
    g_count_ids = g_eng->tok.encode(input, addbos);
    o.count = (int)g_count_ids.size();
    o.ids = g_count_ids.data();
    return o;
}
bool sd_load_model(const sd_load_model_inputs) { return false; }
sd_generation_outputs sd_generate(const sd_generation_inputs) { sd_generation_outputs o; o.status = 0; o.data = ""; return o; }
bool whisper_load_model(const whisper_load_model_inputs) { return false; }
whisper_generation_outputs whisper_generate(const whisper_generation_inputs) {
    whisper_generation_outputs o; o.status = 0; o.text = ""; return o;
}

}  // extern "C"
