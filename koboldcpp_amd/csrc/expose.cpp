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
// Sampling is host code (as in the reference): the full SampleLogits chain restated in sampler.h (logit biases,
// DRY, rep_pen, top-k/a/p, min-p, tfs, typical, temperature / dynatemp / smoothing, mirostat, XTC) over
// the user's sampler_order and a seeded mt19937; when that chain reduces to argmax (greedy, no biases /
// penalties / bans) the token comes from the on-device argmax instead of a logits copy.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <ctime>
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
#include "kcpp_internal.h"
#include "sampler.h"
#include "tokenizer.h"

namespace {

// RCCL (librccl, loaded at run time so a one-GPU deployment does not need it): the entry points the stage
// handoff uses, with ncclComm_t / ncclDataType_t / ncclResult_t as their ABI types (rccl.h)
struct Rccl {
    typedef int (*InitAllFn)(void **comms, int ndev, const int *devlist);
    typedef int (*SendFn)(const void *buf, size_t count, int dtype, int peer, void *comm, hipStream_t stream);
    typedef int (*RecvFn)(void *buf, size_t count, int dtype, int peer, void *comm, hipStream_t stream);
    typedef int (*GroupFn)(void);
    typedef int (*DestroyFn)(void *comm);
    InitAllFn init_all = nullptr;
    SendFn send = nullptr;
    RecvFn recv = nullptr;
    GroupFn group_start = nullptr, group_end = nullptr;
    DestroyFn destroy = nullptr;
    bool load() {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return false;
        init_all = (InitAllFn)dlsym(h, "ncclCommInitAll");
        send = (SendFn)dlsym(h, "ncclSend");
        recv = (RecvFn)dlsym(h, "ncclRecv");
        group_start = (GroupFn)dlsym(h, "ncclGroupStart");
        group_end = (GroupFn)dlsym(h, "ncclGroupEnd");
        destroy = (DestroyFn)dlsym(h, "ncclCommDestroy");
        return init_all && send && recv && group_start && group_end && destroy;
    }
};
constexpr int kNcclFloat32 = 7;   // ncclFloat32 (rccl.h)

struct Engine {
    gguf::File file;
    Tokenizer tok;
    kcpp_hparams hp{};
    std::vector<int> types;
    std::vector<kcpp_model *> stages;
    std::vector<float *> hidden;            // per stage residual stream (device)
    std::vector<int> devs;                  // per stage device
    // stage handoff (replaces ggml_backend_sched_compute_splits' per-split input copies and events,
    // ggml-backend.cpp:2108-2201): RCCL send/recv between the stage streams when every stage has its own GPU,
    // otherwise a device copy ordered by events; never a host synchronisation between stages
    Rccl rccl;
    std::vector<void *> comms;              // rank s = stage s
    std::vector<hipEvent_t> ev_done, ev_read;
    // greedy single-token steps: the hand-off inside each stage's graph (link.hip: the consumer's first kernel pulls the
    // producer's row once its flag is up, the producer's last kernel raises it) -- no event, copy or host call between
    // stages; prefill ubatches keep the RCCL / event-ordered copies above
    bool linked = false;
    std::vector<void *> link_blk;           // per stage: 256 B of flag words on the stage's device
    int ub = 512;
    bool use_contextshift = false;
    std::vector<int> ctx;                   // tokens whose K/V are in the caches
    std::vector<float> logits;
    // the last stage's argmax_dev holds the greedy token of the current logits AND stage 0's token input holds the
    // same token: true after a single-token step (its graph ends in the argmax) once the token is home
    bool dev_tok = false;
    ~Engine() {
        for (size_t s = 0; s < stages.size(); ++s) {
            hipSetDevice(devs[s]);
            if (s < ev_done.size() && ev_done[s]) hipEventDestroy(ev_done[s]);
            if (s < ev_read.size() && ev_read[s]) hipEventDestroy(ev_read[s]);
        }
        for (void *c : comms) if (c && rccl.destroy) rccl.destroy(c);
        for (auto *m : stages) kcpp_model_free(m);
        for (size_t s = 0; s < link_blk.size(); ++s)
            if (link_blk[s]) { hipSetDevice(devs[s]); hipFree(link_blk[s]); }
    }
};

std::unique_ptr<Engine> g_eng;
std::mutex g_out_mtx;
std::vector<std::string> g_generated;       // streamed pieces (new_token / get_stream_count)
std::string g_concat, g_result, g_pending;
std::atomic<bool> g_finished{true}, g_abort{false};
float g_last_eval = 0, g_last_process = 0;
int g_last_count = 0, g_last_seed = 0, g_total_gens = 0;
float g_mirostat_mu = 0.0f;
int g_last_stop = KCPP_STOP_INVALID;
std::vector<int> g_count_ids;

const char *tname(int il, int j) {
    static const char *n[9] = {"attn_norm", "attn_q", "attn_k", "attn_v", "attn_output", "ffn_norm", "ffn_gate", "ffn_up", "ffn_down"};
    (void)il;
    return n[j];
}

bool supported_type(int t) {
    return t == KT_F32 || t == KT_F16 || t == KT_Q4_0 || t == KT_Q4_1 || t == KT_Q5_0 || t == KT_Q5_1 || t == KT_Q8_0 || t == KT_Q2_K || t == KT_Q3_K || t == KT_Q4_K || t == KT_Q5_K ||
           t == KT_IQ4_NL || t == KT_IQ4_XS || t == KT_IQ2_XXS || t == KT_IQ2_XS || t == KT_IQ2_S || t == KT_IQ3_XXS || t == KT_IQ3_S || t == KT_IQ1_S || t == KT_IQ1_M ||
           t == KT_Q6_K;
}

}  // namespace

// CalcGradientAIRopeFreqBase (gpttype_adapter.cpp:1598-1640): the RoPE base for a context beyond the trained one,
// float arithmetic as the reference's (log10f / powf); solar = GGUFArch::ARCH_SOLAR (context x 8, positive offset)
extern "C" float kcpp_gradient_ai_rope_base(float original_rope_base, int n_ctx_train, int n_ctx_desired, int solar) {
    if (n_ctx_desired <= n_ctx_train || n_ctx_desired <= 2048) return original_rope_base;
    const float ctx_multiplier = solar ? 8.0f : 1.0f;
    const float chi_ctx_train_value = (n_ctx_train * ctx_multiplier) / 6.28318;
    const float chi_ctx_value = (n_ctx_desired * ctx_multiplier) / 6.28318;
    const float gradient_ai_rope_freq_base_value = powf(original_rope_base, log10f(chi_ctx_value) / log10f(chi_ctx_train_value));
    if (!solar) return gradient_ai_rope_freq_base_value;
    const float extended_rope_positive_offset_value =
        1 + ((log10f(chi_ctx_value) - log10f(chi_ctx_train_value)) /
             ((log10f(chi_ctx_value) * log10f(chi_ctx_train_value)) - (log10f(chi_ctx_value) + log10f(chi_ctx_train_value))));
    return gradient_ai_rope_freq_base_value * extended_rope_positive_offset_value;
}

namespace {

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

// The pipeline schedule is written against the stage operations below: HipOps drives the engine's stage streams
// (RCCL send/recv or event-ordered peer copies) in the product, TraceOps records the enqueue order for the CPU test
// hook kcpp_pipeline_trace (tests/test_pipeline.py).  Neither forward() nor greedy_step() synchronises the host.
struct PipeOps {
    virtual ~PipeOps() = default;
    virtual size_t n_stages() const = 0;
    virtual int ubatch() const = 0;
    virtual int decode(size_t s, const int32_t *toks, int t, int n_past) = 0;   // enqueue t tokens (stage 0: the ids)
    virtual int step_dev(size_t s, int n_past) = 0;       // one token whose input is already on the device
    virtual int handoff(size_t s, int t) = 0;             // stage s-1's residual stream (t tokens) -> stage s
    virtual int argmax_dev() = 0;                         // last stage: greedy token of its last logits, on device
    virtual int token_home() = 0;                         // that token -> stage 0's input token (device copy)
    bool in_greedy = false;                               // inside greedy_step
};

// run tokens [i0, i0+T) through all stages, ubatch by ubatch, everything enqueued: stage s works on ubatch u while
// stage s+1 works on ubatch u-1 (the pipeline the reference gets from n_copies = 4, ggml-backend.cpp:1372); the
// caller's logits read on the last stage is the only host synchronisation
int forward(PipeOps &o, const int32_t *toks, int T, int n_past) {
    const int ub = o.ubatch();
    for (int i = 0; i < T; i += ub) {
        const int t = std::min(ub, T - i);
        for (size_t s = 0; s < o.n_stages(); ++s) {
            if (s > 0) {
                const int rc = o.handoff(s, t);
                if (rc) return rc;
            }
            const int rc = o.decode(s, s == 0 ? toks + i : nullptr, t, n_past + i);
            if (rc) return rc;
        }
    }
    return 0;
}

// one greedy token through all stages without the host: stage 0 embeds the token the last stage's argmax left
// (moved home by token_home), each later stage takes its predecessor's hand-off, the last stage's step computes
// the next greedy token on device, which goes home for the next step.  (HipOps with linked stages: the hand-offs
// and the token's way home happen inside the stage steps, link.hip.)
int greedy_step(PipeOps &o, int n_past) {
    o.in_greedy = true;
    int rc = 0;
    for (size_t s = 0; s < o.n_stages() && !rc; ++s) {
        if (s > 0) rc = o.handoff(s, 1);
        if (!rc) rc = o.step_dev(s, n_past);
    }
    if (!rc) rc = o.token_home();
    o.in_greedy = false;
    return rc;
}

struct HipOps : PipeOps {
    Engine &e;
    explicit HipOps(Engine &en) : e(en) {}
    size_t n_stages() const override { return e.stages.size(); }
    int ubatch() const override { return e.ub; }
    int decode(size_t s, const int32_t *toks, int t, int n_past) override {
        return kcpp_model_decode_async(e.stages[s], toks, t, n_past);
    }
    int step_dev(size_t s, int n_past) override {
        return e.linked ? kcpp_model_step_linked(e.stages[s], n_past) : kcpp_model_step_dev(e.stages[s], n_past);
    }
    int argmax_dev() override { return kcpp_model_argmax_async(e.stages.back()); }
    // stage s-1's residual stream (t tokens) -> stage s's input, on the two stages' streams
    int handoff(size_t s, int t) override {
        if (in_greedy && e.linked) return 0;                       // pulled by stage s's own graph (link.hip)
        const size_t count = (size_t)t * e.hp.n_embd;
        hipStream_t src = (hipStream_t)kcpp_model_stream(e.stages[s - 1]), dst = (hipStream_t)kcpp_model_stream(e.stages[s]);
        if (!e.comms.empty()) {
            if (e.rccl.group_start()) return -20;
            const int r1 = e.rccl.send(e.hidden[s - 1], count, kNcclFloat32, (int)s, e.comms[s - 1], src);
            const int r2 = e.rccl.recv(e.hidden[s], count, kNcclFloat32, (int)s - 1, e.comms[s], dst);
            if (e.rccl.group_end() || r1 || r2) return -21;
            return 0;
        }
        // dst waits for the producer, copies, and the producer's next write waits for the copy to have read
        if (hipSetDevice(e.devs[s - 1]) || hipEventRecord(e.ev_done[s - 1], src)) return -22;
        if (hipSetDevice(e.devs[s]) || hipStreamWaitEvent(dst, e.ev_done[s - 1], 0)) return -22;
        const hipError_t ce = e.devs[s] == e.devs[s - 1]
                                  ? hipMemcpyAsync(e.hidden[s], e.hidden[s - 1], count * 4, hipMemcpyDeviceToDevice, dst)
                                  : hipMemcpyPeerAsync(e.hidden[s], e.devs[s], e.hidden[s - 1], e.devs[s - 1], count * 4, dst);
        if (ce != hipSuccess || hipEventRecord(e.ev_read[s], dst)) return -23;
        if (hipSetDevice(e.devs[s - 1]) || hipStreamWaitEvent(src, e.ev_read[s], 0)) return -22;
        return 0;
    }
    // the last stage's argmax (4 bytes) into stage 0's token input: stage 0's stream waits for the last stage's
    // step, then a peer copy over xGMI (one stage: the argmax kernel already wrote the token input)
    int token_home() override {
        const size_t L = e.stages.size() - 1;
        if (L == 0 || (in_greedy && e.linked)) return 0;           // linked: stage 0's graph pulls the token
        
        hipStream_t last = (hipStream_t)kcpp_model_stream(e.stages[L]), first = (hipStream_t)kcpp_model_stream(e.stages[0]);
        if (hipSetDevice(e.devs[L]) || hipEventRecord(e.ev_done[L], last)) return -24;
        if (hipSetDevice(e.devs[0]) || hipStreamWaitEvent(first, e.ev_done[L], 0)) return -24;
        const hipError_t ce = e.devs[0] == e.devs[L]
                                  ? hipMemcpyAsync(kcpp_model_token_dev(e.stages[0]), kcpp_model_argmax_dev(e.stages[L]), 4,
                                                   hipMemcpyDeviceToDevice, first)
                                  : hipMemcpyPeerAsync(kcpp_model_token_dev(e.stages[0]), e.devs[0],
                                                       kcpp_model_argmax_dev(e.stages[L]), e.devs[L], 4, first);
        return ce == hipSuccess ? 0 : -25;
    }
};

// records the schedule: "d<s>:<t>@<n_past>" decode, "h<s>:<t>" hand-off into stage s, "s<s>@<n_past>" device-token
// step, "a" last-stage argmax, "k" token home
struct TraceOps : PipeOps {
    size_t S;
    int ub;
    std::string log;
    TraceOps(size_t s, int u) : S(s), ub(u) {}
    size_t n_stages() const override { return S; }
    int ubatch() const override { return ub; }
    void put(const std::string &x) { log += (log.empty() ? "" : " ") + x; }
    int decode(size_t s, const int32_t *toks, int t, int n_past) override {
        if ((s == 0) != (toks != nullptr)) return -1;              // ids only into the embedding stage
        put("d" + std::to_string(s) + ":" + std::to_string(t) + "@" + std::to_string(n_past));
        return 0;
    }
    int step_dev(size_t s, int n_past) override { put("s" + std::to_string(s) + "@" + std::to_string(n_past)); return 0; }
    int handoff(size_t s, int t) override { put("h" + std::to_string(s) + ":" + std::to_string(t)); return 0; }
    int argmax_dev() override { put("a"); return 0; }
    int token_home() override { put("k"); return 0; }
};

int forward(Engine &e, const int32_t *toks, int T, int n_past) {
    HipOps o(e);
    return forward(o, toks, T, n_past);
}

// the linked single-token hand-off (link.hip) when every stage replays graphs and each pair of neighbouring stages
// (and the last and the first) can reach each other's memory; KCPP_HANDOFF=copy / rccl keep the single-token hops on
// the event-ordered copies / RCCL
static void init_links(Engine &e) {
    const size_t S = e.stages.size();
    const char *mode = getenv("KCPP_HANDOFF");
    if (S < 2 || (mode && (!strcmp(mode, "copy") || !strcmp(mode, "rccl")))) return;
    auto reach = [&](int a, int b) {            // device a's kernels may access device b's memory
        if (a == b) return true;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, a, b) != hipSuccess || !ok) return false;
        hipSetDevice(a);
        const hipError_t r = hipDeviceEnablePeerAccess(b, 0);
        (void)hipGetLastError();
        return r == hipSuccess || r == hipErrorPeerAccessAlreadyEnabled;
    };
    for (size_t s = 0; s < S; ++s) {
        const size_t p = (s + S - 1) % S, c = (s + 1) % S;
        if (!reach(e.devs[s], e.devs[p]) || !reach(e.devs[s], e.devs[c])) return;
    }
    // flag blocks in fine-grained device memory: a peer GPU's flag stores are visible to the polling kernel without a
    // kernel boundary (coarse-grained lines may sit in the owner's L2 until one); stages sharing one GPU could do with
    // coarse-grained memory, but one rule keeps the multi-GPU path the one the tests exercise
    e.link_blk.assign(S, nullptr);
    for (size_t s = 0; s < S; ++s) {
        hipSetDevice(e.devs[s]);
        if (hipExtMallocWithFlags(&e.link_blk[s], 256, hipDeviceMallocFinegrained) != hipSuccess) {
            (void)hipGetLastError();
            e.link_blk[s] = nullptr;
            return;                               // no fine-grained memory: the event-ordered hand-offs
        }
        if (hipMemset(e.link_blk[s], 0, 256) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return;
    }
    // words of stage s's block: [0] step counter, [16] ready_in, [32] copied_out, [48] error (a wait that gave up)
    auto word = [&](size_t s, int i) { return (unsigned *)e.link_blk[s] + i; };
    for (size_t s = 0; s < S; ++s) {
        const size_t p = (s + S - 1) % S, c = (s + 1) % S;
        KLink L{};
        L.stepctr = word(s, 0);
        L.ready_in = word(s, 16);
        L.copied_out = word(s, 32);
        L.ready_out = word(c, 16);
        L.copied_report = word(p, 32);
        if (s == 0) {
            L.src_tok = kcpp_model_argmax_dev(e.stages[S - 1]);
            L.dst_tok = kcpp_model_token_dev(e.stages[0]);
            L.in_lag = 1;
        } else {
            L.src_x = e.hidden[s - 1];
            L.dst_x = e.hidden[s];
            L.n = e.hp.n_embd;
        }
        L.out_lag = s == S - 1 ? 0 : 1;
        L.err = word(s, 48);
        if (kcpp_model_set_link(e.stages[s], &L)) return;
    }
    e.linked = true;
}

// after a sync: did any linked wait give up (k_link_wait's bounded poll)?  Reported once, cleared.
static bool link_errors(Engine &e) {
    if (!e.linked) return false;
    bool bad = false;
    for (size_t s = 0; s < e.link_blk.size(); ++s) {
        unsigned w = 0;
        hipSetDevice(e.devs[s]);
        if (hipMemcpy(&w, (unsigned *)e.link_blk[s] + 48, 4, hipMemcpyDeviceToHost) != hipSuccess || w) {
            fprintf(stderr, "[kcpp] linked hand-off: stage %zu gave up waiting at step %u\n", s, w);
            const unsigned z = 0;
            (void)hipMemcpy((unsigned *)e.link_blk[s] + 48, &z, 4, hipMemcpyHostToDevice);
            bad = true;
        }
    }
    return bad;
}

// events for the copy handoff, and an RCCL clique when every stage sits on its own device (RCCL refuses two
// ranks on one GPU); KCPP_HANDOFF=copy forces the event-ordered copies
bool init_handoff(Engine &e) {
    const size_t S = e.stages.size();
    e.ev_done.assign(S, nullptr);
    e.ev_read.assign(S, nullptr);
    for (size_t s = 0; s < S; ++s) {
        hipSetDevice(e.devs[s]);
        if (hipEventCreateWithFlags(&e.ev_done[s], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.ev_read[s], hipEventDisableTiming) != hipSuccess)
            return false;
    }
    if (S < 2) return true;
    init_links(e);
    std::vector<int> sorted = e.devs;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char *mode = getenv("KCPP_HANDOFF");
    if (!distinct || (mode && !strcmp(mode, "copy")) || !e.rccl.load()) return true;
    e.comms.assign(S, nullptr);
    if (e.rccl.init_all(e.comms.data(), (int)S, e.devs.data()) != 0) {
        fprintf(stderr, "[kcpp] load_model: ncclCommInitAll failed, stage handoff by peer copies\n");
        e.comms.clear();
    }
    return true;
}

// the stages of a model over ndev (possibly virtual) devices, nreal of them real: layer split exactly as
// llm_load_tensors (src/llama.cpp:7000-7036), or one row-split stage (LLAMA_SPLIT_MODE_ROW) on the main device
bool build_stages(Engine &e, int ndev, int nreal, const float *tensor_split, bool rowsplit, int main_gpu) {
    const kcpp_hparams &hp = e.hp;
    const std::vector<int> ldev = split_layers(hp.n_layer, std::min(ndev, KCPP_TENSOR_SPLIT_MAX), tensor_split);
    int il = 0;
    // stages of consecutive layers per device; the output head on its own device (upper_bound of
    // (act - 1) / act, src/llama.cpp:7030-7033) -- a head-only stage when that is not the last layers' device
    auto add_stage = [&](int d, int i0, int i1, bool out) {
        const int gpu = d % nreal;
        kcpp_model *m = kcpp_model_create(&hp, e.types.data(), gpu, i0, i1, e.stages.empty(), out, e.ub);
        if (!m) { fprintf(stderr, "[kcpp] load_model: %s\n", kcpp_last_error()); return false; }
        e.stages.push_back(m);
        e.hidden.push_back(kcpp_model_hidden(m));
        e.devs.push_back(gpu);
        if (e.stages.size() > 1 && e.devs[e.devs.size() - 2] != gpu) {
            hipSetDevice(gpu);
            hipDeviceEnablePeerAccess(e.devs[e.devs.size() - 2], 0);   // xGMI peer copies for the handoff
            (void)hipGetLastError();
        }
        return true;
    };
    if (rowsplit && std::min(ndev, KCPP_TENSOR_SPLIT_MAX) > 1) {
        // LLAMA_SPLIT_MODE_ROW (gpttype_adapter.cpp:1892): one stage on the main device (cublas_info,
        // gpttype_adapter.cpp:1708) owning every layer; the matrices' rows spread over the devices by tensor_split
        const int nd = std::min(ndev, KCPP_TENSOR_SPLIT_MAX);
        const int main_dev = std::min(main_gpu <= 0 ? 0 : main_gpu, nd - 1) % nreal;
        std::vector<int> devs(nd);
        for (int i = 0; i < nd; ++i) devs[i] = i % nreal;
        kcpp_model *m = kcpp_model_create(&hp, e.types.data(), main_dev, 0, hp.n_layer, 1, 1, e.ub);
        if (!m) { fprintf(stderr, "[kcpp] load_model: %s\n", kcpp_last_error()); return false; }
        e.stages.push_back(m);
        e.hidden.push_back(kcpp_model_hidden(m));
        e.devs.push_back(main_dev);
        if (kcpp_model_set_row_split(m, nd, devs.data(), tensor_split)) {
            fprintf(stderr, "[kcpp] load_model: row split: %s\n", kcpp_last_error());
            return false;
        }
        il = hp.n_layer;
    }
    while (il < hp.n_layer) {
        const int d = ldev[il];
        int il1 = il;
        while (il1 < hp.n_layer && ldev[il1] == d) ++il1;
        const bool last = il1 == hp.n_layer;
        if (!add_stage(d, il, il1, last && ldev[hp.n_layer] == d)) return false;
        if (last && ldev[hp.n_layer] != d && !add_stage(ldev[hp.n_layer], hp.n_layer, hp.n_layer, true)) return false;
        il = il1;
    }
    return true;
}

// per-generate sampler state: the reference's parameter clamps (gpttype_adapter.cpp:2576-2584, 2625-2735),
// sampler order (:2957-2976), DRY restart sequences (:2650-2700), single-character token bans (:2518-2568)
struct SamplerSetup {
    ksamp::Params P;
    std::vector<ksamp::LogitBias> biases;
    ksamp::RestartSeqs restarts;
    std::vector<int> banned;
    std::vector<std::string> phrases;      // antislop: banned multi-token phrases (lower case)
    int delay = 0;                         // delayed_generated_tokens_limit: tokens held back before streaming
    int n_ctx = 0;
    bool suppress_eos = false;
};

std::string lower(std::string s) {
    for (char &c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

// GetOverlappingTokenSequences, gpttype_adapter.cpp:348-408
void overlapping_sequences(const Engine &e, const std::string &str, ksamp::RestartSeqs &seqs, int max_tail) {
    bool ext = !str.empty();
    for (unsigned char c : str) ext &= c > 127;
    for (int v = 0; v < e.hp.n_vocab; ++v) {
        const std::string word = e.tok.piece(v);
        if (word.find(str) != std::string::npos) {
            auto its = seqs.equal_range(v);
            bool empty = false;
            for (auto it = its.first; it != its.second; ++it) empty |= it->second.empty();
            if (!empty) seqs.emplace(v, std::vector<int>());
            continue;
        }
        const size_t wl = word.size(), sl = str.size();
        size_t pos = (size_t)-1;
        while ((pos = word.find(str[0], pos + 1)) != std::string::npos) {
            bool match = true;
            size_t i;
            for (i = 1; i < sl && i + pos < wl; ++i)
                if (word[pos + i] != str[i]) { match = false; break; }
            if (match && !ext) {
                std::vector<int> tail = e.tok.encode(str.substr(i), false);
                if (max_tail >= 0 && (int)tail.size() > max_tail) tail.resize(max_tail);
                auto its = seqs.equal_range(v);
                bool found = false;
                for (auto it = its.first; it != its.second; ++it) found |= it->second == tail;
                if (!found) seqs.emplace(v, tail);
            }
        }
    }
}

SamplerSetup make_sampler(const Engine &e, const generation_inputs &in, int n_ctx) {
    SamplerSetup S;
    ksamp::Params &P = S.P;
    S.n_ctx = n_ctx;
    const int nv = e.hp.n_vocab;
    for (int k = 0; k < KCPP_LOGIT_BIAS_MAX; ++k) {
        const logit_bias &b = in.logit_biases[k];
        if (b.token_id >= 0 && b.token_id < nv && b.bias != 0) S.biases.push_back({b.token_id, b.bias});
    }
    P.top_k = (float)in.top_k; P.top_a = in.top_a; P.top_p = in.top_p; P.min_p = in.min_p; P.typical_p = in.typical_p;
    P.tfs = in.tfs; P.temp = in.temperature; P.rep_pen = in.rep_pen; P.rep_pen_slope = in.rep_pen_slope;
    P.presence_penalty = in.presence_penalty; P.mirostat = in.mirostat; P.mirostat_eta = in.mirostat_eta;
    P.mirostat_tau = in.mirostat_tau; P.dry_multiplier = in.dry_multiplier; P.dry_base = in.dry_base;
    P.dry_allowed_length = in.dry_allowed_length; P.dry_penalty_last_n = in.dry_penalty_last_n;
    P.xtc_threshold = in.xtc_threshold; P.xtc_probability = in.xtc_probability; P.dynatemp_range = in.dynatemp_range;
    P.dynatemp_exponent = in.dynatemp_exponent; P.smoothing_factor = in.smoothing_factor;
    P.rep_pen_range = std::max(1, in.rep_pen_range);
    if (P.rep_pen_slope > 1 || P.rep_pen_slope <= 0) P.rep_pen_slope = 1;
    if (P.top_k < 1) P.top_k = (float)nv;
    if (in.sampler_len <= 0)
        P.order = {ksamp::S_REP_PEN, ksamp::S_TOP_K, ksamp::S_TOP_A, ksamp::S_TFS, ksamp::S_TYP, ksamp::S_TOP_P, ksamp::S_TEMP};
    else
        for (int i = 0; i < std::min(in.sampler_len, KCPP_SAMPLER_MAX); ++i) P.order.push_back(in.sampler_order[i]);
    if (P.dry_multiplier > 0) {
        for (int x = 0; x < KCPP_DRY_SEQ_BREAK_MAX; ++x) {
            if (!in.dry_sequence_breakers[x] || !in.dry_sequence_breakers[x][0]) continue;
            std::string w = in.dry_sequence_breakers[x];
            if (w.size() > 40) w.resize(40);
            overlapping_sequences(e, w, S.restarts, 20);
        }
    }
    // token bans and antislop phrases (gpttype_adapter.cpp:2514-2545): a single-character entry that is one token bans
    // every vocabulary entry containing it; anything longer is a phrase, caught after sampling by the delayed-output
    // rewind in generate(); the output is held back by the longest phrase's token count + 3
    std::vector<std::string> single;
    for (int x = 0; x < KCPP_BAN_TOKEN_MAX; ++x) {
        if (!in.banned_tokens[x] || !in.banned_tokens[x][0]) continue;
        const std::string w = lower(in.banned_tokens[x]);
        const int tokcount = (int)e.tok.encode(w, false).size();
        if (tokcount == 0) continue;
        if (tokcount == 1 && w.length() < 2) single.push_back(w);
        else {
            S.delay = std::max(S.delay, tokcount + 3);
            S.phrases.push_back(w);
        }
    }
    if (!single.empty())
        for (int v = 0; v < nv; ++v) {
            const std::string w = lower(e.tok.piece(v));
            for (const std::string &b : single)
                if (w.find(b) != std::string::npos) { S.banned.push_back(v); break; }
        }
    S.suppress_eos = !in.allow_eos_token && !in.bypass_eos_token;
    return S;
}

// true when the reference chain reduces to argmax of the raw logits, so the on-device argmax is the same token
bool chain_is_argmax(const SamplerSetup &S) {
    const ksamp::Params &P = S.P;
    if (!S.biases.empty() || !S.banned.empty() || P.mirostat == 1 || P.mirostat == 2) return false;
    if (P.dry_multiplier > 0 && P.dry_base > 0) return false;
    if (P.rep_pen != 1.0f || P.presence_penalty != 0) return false;
    if (P.typical_p < 1.0f) return false;               // locally-typical sampling may drop the argmax
    if (P.xtc_probability > 0 && P.xtc_threshold <= 0.5f) return false;
    // greedy: temperature <= 0 (top-1 inside sample_temperature) or top_k == 1 anywhere in the order
    bool has_temp = false, has_topk = false;
    for (int s : P.order) { has_temp |= s == ksamp::S_TEMP; has_topk |= s == ksamp::S_TOP_K; }
    return (has_topk && (int)P.top_k == 1) || (has_temp && P.temp <= 0 && P.dynatemp_range <= 0);
}

// one sampled token from the last stage's logits (gpttype_adapter.cpp:3182-3232); < 0 on a device error.
// slop: the antislop bans recorded for this position (set to the lowest logit like the token bans, :3219-3225)
// on_dev: the token is the device argmax (the next step can take it from the device, greedy_step)
int sample(Engine &e, const SamplerSetup &S, const std::vector<int> &last_n, std::mt19937 &rng, float *mu,
           const std::vector<int> *slop, bool *on_dev) {
    kcpp_model *last = e.stages.back();
    const int eos = e.tok.eos(), eot = e.tok.eot();
    *on_dev = false;
    if (chain_is_argmax(S) && !slop) {
        int32_t t = 0;
        // after a single-token step the step's own argmax is already on the device: read it; after a prefill, run it
        if (e.dev_tok ? kcpp_model_read_argmax(last, &t) : kcpp_model_argmax(last, &t)) return -1;
        if (!(S.suppress_eos && (t == eos || (t == eot && eot != -1)))) {
            *on_dev = true;
            return t;
        }
    }
    e.logits.resize(e.hp.n_vocab);
    if (kcpp_model_read_logits(last, e.logits.data())) return -1;
    float *l = e.logits.data();
    const float low = ksamp::lowest_logit(l, e.logits.size());
    // EOS and EOT both set to the lowest logit (gpttype_adapter.cpp:3198-3209)
    if (S.suppress_eos && eos >= 0 && eos < e.hp.n_vocab) l[eos] = low;
    if (S.suppress_eos && eot >= 0 && eot < e.hp.n_vocab) l[eot] = low;
    for (int b : S.banned) l[b] = low;
    if (slop)
        for (int b : *slop)
            if (b >= 0 && b < e.hp.n_vocab) l[b] = low;
    return ksamp::sample_logits(l, S.n_ctx, e.hp.n_vocab, S.P, S.biases, S.restarts, e.ctx, last_n, rng, mu);
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
    // RoPE (gpttype_adapter.cpp:1677-1700, 1926-1950): a user --ropeconfig (rope_freq_scale > 0) wins; a model that
    // sets its own RoPE (freq_base not 10000 / 500000, a linear scale, or YaRN) keeps its values; otherwise the base
    // is auto-scaled for the requested context by the GradientAI rule (CalcGradientAIRopeFreqBase)
    const float base_train = (float)f.get_f("llama.rope.freq_base", 10000.0);
    float ropescale = (float)f.get_f("llama.rope.scaling.factor", 0.0);
    if (ropescale == 0.0f) ropescale = (float)f.get_f("llama.rope.scale_linear", 0.0);
    const float scale_train = ropescale == 0.0f ? 1.0f : 1.0f / ropescale;
    // YaRN is refused only where the model's own RoPE values would be used: a user --ropeconfig replaces them and the
    // reference then never reads the model's YaRN settings (gpttype_adapter.cpp:1681-1687, 1926-1930)
    if (f.get_s("llama.rope.scaling.type", "") == "yarn" && !(inputs.rope_freq_scale > 0.0f)) {
        fprintf(stderr, "[kcpp] load_model: YaRN rope scaling is not supported (pass --ropeconfig to override)\n");
        return false;
    }
    const int n_ctx_train = (int)f.get_i("llama.context_length", 2048);     // FileFormatExtraMeta default
    // ARCH_SOLAR (model_adapter.cpp:309): llama, freq_base 10000, 435 or 611 tensors
    const bool solar = base_train == 10000.0f && (f.tensors.size() == 435 || f.tensors.size() == 611);
    if (inputs.rope_freq_scale > 0.0f) {
        hp.rope_base = inputs.rope_freq_base;
        hp.rope_freq_scale = inputs.rope_freq_scale;
    } else if ((base_train != 10000.0f && base_train != 500000.0f) || scale_train != 1.0f) {
        hp.rope_base = base_train;
        hp.rope_freq_scale = scale_train;
    } else {
        hp.rope_base = kcpp_gradient_ai_rope_base(base_train, n_ctx_train, inputs.max_context_length, solar);
        hp.rope_freq_scale = 1.0f;
    }
    hp.n_ctx = inputs.max_context_length > 0 ? inputs.max_context_length + 8 : 2048 + 8;
    if (hp.n_layer <= 0 || hp.n_head <= 0 || (hp.n_embd / hp.n_head != 128 && hp.n_embd / hp.n_head != 64)) {
        fprintf(stderr, "[kcpp] load_model: need head_dim 128 or 64 (got n_embd %d / n_head %d)\n", hp.n_embd, hp.n_head);
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
    // n_gpu_layers (src/llama.cpp:6977-7036: layers [0, n_layer - n_gpu_layers) stay on the CPU backend): this backend
    // has no CPU compute path, so a partial offload is refused instead of silently becoming a full one; negative
    // (koboldcpp's auto) and >= n_layer offload everything (the output head, which the reference keeps on the CPU
    // for n_gpu_layers == n_layer, runs here on the last GPU)
    if (inputs.gpulayers >= 0 && inputs.gpulayers < hp.n_layer) {
        fprintf(stderr, "[kcpp] load_model: gpulayers %d < %d layers: partial offload (CPU layers) is not supported by "
                        "this backend; use gpulayers >= %d (or -1)\n", inputs.gpulayers, hp.n_layer, hp.n_layer);
        return false;
    }
    // rope_freqs.weight (Llama-3.1 / 3.2: src/llama.cpp:7171, one tensor shared by every layer's rope,
    // build_rope_factors :10269), n_rot / 2 F32 frequency factors
    std::vector<float> rope_ff;
    if (const gguf::Tensor *rf = f.tensor("rope_freqs.weight")) {
        const int nff = (hp.n_embd / hp.n_head) / 2;
        if (rf->type != KT_F32 || rf->ne[0] != nff || rf->ne[1] * rf->ne[2] * rf->ne[3] != 1) {
            fprintf(stderr, "[kcpp] load_model: rope_freqs.weight: expected %d F32 values\n", nff);
            return false;
        }
        rope_ff.assign((const float *)rf->data, (const float *)rf->data + nff);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) { fprintf(stderr, "[kcpp] load_model: no GPU\n"); return false; }
    // test hook: KCPP_VIRTUAL_DEVICES=n splits the layers as if n GPUs were visible, stage i on GPU i % ndev
    const int nreal = ndev;
    if (getenv("KCPP_VIRTUAL_DEVICES")) ndev = std::max(1, atoi(getenv("KCPP_VIRTUAL_DEVICES")));
    e->ub = inputs.blasbatchsize > 0 ? std::min(inputs.blasbatchsize, 512) : 512;
    e->use_contextshift = inputs.use_contextshift;
    if (!build_stages(*e, ndev, nreal, inputs.tensor_split, inputs.use_rowsplit, inputs.cublas_info)) return false;
    if (!init_handoff(*e)) { fprintf(stderr, "[kcpp] load_model: handoff events\n"); return false; }
    // KV cache types (gpttype_adapter.cpp:1958-1959: quant_k/v > 1 -> Q4_0, == 1 -> Q8_0, else F16).  Quantized
    // caches imply flash attention and no context shift (koboldcpp.py's --quantkv handling); this runtime's
    // attention is always the flash form.  K and V must both be F16 or both quantized.
    const auto kvtype = [](int q) { return q > 1 ? KT_Q4_0 : (q == 1 ? KT_Q8_0 : KT_F16); };
    const int tk = kvtype(inputs.quant_k), tv = kvtype(inputs.quant_v);
    if (tk != KT_F16 || tv != KT_F16) {
        for (kcpp_model *m : e->stages)
            if (kcpp_model_set_kv_types(m, tk, tv)) {
                fprintf(stderr, "[kcpp] load_model: quant_k %d / quant_v %d: %s\n", inputs.quant_k, inputs.quant_v,
                        kcpp_last_error());
                return false;
            }
        e->use_contextshift = false;
    }
    if (!rope_ff.empty())
        for (kcpp_model *m : e->stages)
            if (kcpp_model_set_rope_freqs(m, rope_ff.data(), (int)rope_ff.size())) {
                fprintf(stderr, "[kcpp] load_model: rope_freqs: %s\n", kcpp_last_error());
                return false;
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
            const int cut = std::min((int)mem.size(), (int)mem.size() - max_ctx + max_len + 4);   // clamped (the
            mem.erase(mem.begin(), mem.begin() + cut);                       // reference pre-resizes, :2840-2845)
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
    e->dev_tok = false;
    if (forward(*e, toks.data() + keep, (int)(toks.size() - keep), (int)keep)) {
        fprintf(stderr, "[kcpp] generate: prefill failed: %s\n", kcpp_last_error());
        g_finished = true;
        return out;
    }
    e->ctx.insert(e->ctx.end(), toks.begin() + keep, toks.end());
    // forward() only enqueues: the prompt's time ends when the last stage's stream has drained (the reference's
    // llama_decode returns after the graph ran, gpttype_adapter.cpp:3064, 3160-3164)
    if (kcpp_model_sync(e->stages.back())) {
        fprintf(stderr, "[kcpp] generate: prefill failed: %s\n", kcpp_last_error());
        g_finished = true;
        return out;
    }
    const auto t1 = std::chrono::steady_clock::now();
    // seed as gpttype_adapter.cpp:2736-2740 (time-based when <= 0 or 0xFFFFFFFF)
    uint32_t seed = (uint32_t)in.seed;
    if (in.seed <= 0 || seed == 0xFFFFFFFFu) seed = (uint32_t)time(nullptr) % 1000000u;
    std::mt19937 rng(seed);
    g_last_seed = (int)seed;
    // SampleLogits' n_ctx is kcpp_data->n_ctx, which generate() sets to the request's max_context_length
    // (gpttype_adapter.cpp:2646, passed as nctx at :3227)
    const SamplerSetup S = make_sampler(*e, in, in.max_context_length > 0 ? in.max_context_length : max_ctx);
    // SampleLogits' function-static mirostat_mu (:1369) is initialised by the first call that enters the
    // mirostat branch, with that call's tau
    static bool mu_init = false;
    if (!mu_init && (S.P.mirostat == 1 || S.P.mirostat == 2)) { g_mirostat_mu = 2.0f * S.P.mirostat_tau; mu_init = true; }
    // last_n_tokens: repeat_last_n zeros, then every context token in order (:2892-2895, 3236-3243, 3420-3425)
    std::vector<int> last_n(S.P.rep_pen_range, 0);
    for (int t : e->ctx) {
        if (!last_n.empty()) last_n.erase(last_n.begin());
        last_n.push_back(t);
    }
    std::vector<std::string> stops;
    std::vector<int> special_stops;          // a stop string that is one special token without text (:2497-2510)
    for (int k = 0; k < KCPP_STOP_TOKEN_MAX; ++k)
        if (in.stop_sequence[k] && in.stop_sequence[k][0]) {
            stops.emplace_back(in.stop_sequence[k]);
            const std::vector<int> st = e->tok.encode(in.stop_sequence[k], false);
            if (st.size() == 1 && e->tok.piece(st[0]).empty()) special_stops.push_back(st[0]);
        }
    // generated text streams through a delay line of S.delay tokens (delayed_generated_tokens,
    // gpttype_adapter.cpp:3251-3267); stop strings are matched on the streamed text only
    std::deque<std::string> delayed;
    std::map<int, std::vector<int>> slop;    // antislop bans: position -> token ids banned there (:3219, 3325-3331)
    bool hit = false;
    auto emit = [&](const std::string &piece) {
        std::lock_guard<std::mutex> lk(g_out_mtx);
        g_generated.push_back(piece);
        g_concat += piece;
        for (const std::string &st : stops) {
            const size_t p = g_concat.find(st);
            if (p != std::string::npos) { g_concat.resize(p); hit = true; break; }
        }
    };
    int n_gen = 0, stop = KCPP_STOP_OUT_OF_TOKENS;
    double tm_sample = 0, tm_step = 0;     // host time in sample() / in the step's enqueue (KCPP_GEN_TIMING diagnostics)
    for (; n_gen < max_len; ++n_gen) {
        if (g_abort) { stop = KCPP_STOP_CUSTOM_STOPPER; break; }
        const auto sb = slop.find((int)e->ctx.size());
        bool on_dev = false;
        const auto ts0 = std::chrono::steady_clock::now();
        const int t = sample(*e, S, last_n, rng, &g_mirostat_mu, sb == slop.end() ? nullptr : &sb->second, &on_dev);
        tm_sample += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
        if (t < 0) { fprintf(stderr, "[kcpp] generate: sampling failed: %s\n", kcpp_last_error()); break; }
        if (!last_n.empty()) last_n.erase(last_n.begin());     // (:3238: an antislop rewind may have emptied it)
        last_n.push_back(t);
        const bool eos_tok = t == e->tok.eos() || (t == e->tok.eot() && t != -1);
        const bool special_stop = std::find(special_stops.begin(), special_stops.end(), t) != special_stops.end();
        // rendered text (:3253-3257): special tokens as text with render_special, else EOS / EOT / special stops silent
        std::string piece = e->tok.piece(t, in.render_special);
        if (!in.render_special && (eos_tok || special_stop)) piece.clear();
        delayed.push_back(piece);
        while ((int)delayed.size() > S.delay && !delayed.empty()) {
            emit(delayed.front());
            delayed.pop_front();
        }
        // antislop (:3293-3341): a banned phrase in the held-back text rewinds the context to just before the
        // shortest tail of tokens that contains it, and bans that tail's first token at that position
        bool rewound = false;
        if (!S.phrases.empty()) {
            std::string scan;
            for (const std::string &d : delayed) scan += d;
            scan = lower(scan);
            for (const std::string &ph : S.phrases) {
                if (scan.find(ph) == std::string::npos) continue;
                std::string check;
                int rewind = 0;
                for (int i = (int)delayed.size() - 1; i >= 0; --i) {
                    check = delayed[i] + check;
                    ++rewind;
                    if (lower(check).find(ph) != std::string::npos) break;
                }
                const int cur = (int)e->ctx.size() + 1;            // current_context_tokens: the context + t
                if (rewind > 0 && cur - rewind > 0) {
                    const int last_tok = cur - rewind < (int)e->ctx.size() ? e->ctx[cur - rewind] : t;
                    delayed.resize(delayed.size() - rewind);
                    // ContextRewind (:424-480): last_n shrinks, the context drops `rewind` tokens, and the new last
                    // context token is evaluated again (its cache row and every later one are rewritten)
                    if (rewind >= (int)last_n.size()) last_n.clear();
                    else last_n.resize(last_n.size() - rewind);
                    e->ctx.resize(std::max(0, cur - rewind));
                    const int32_t back = e->ctx.back();
                    e->ctx.pop_back();
                    e->dev_tok = false;
                    if (forward(*e, &back, 1, (int)e->ctx.size())) {
                        fprintf(stderr, "[kcpp] generate: decode failed\n");
                        hit = true;
                    }
                    e->ctx.push_back(back);
                    slop[(int)e->ctx.size()].push_back(last_tok);
                    rewound = true;
                    break;
                }
            }
        }
        // EOS (when allowed) or a special stop token ends the generation (:3344-3375), as does a stop string
        if (!in.bypass_eos_token && in.allow_eos_token && eos_tok) { stop = KCPP_STOP_EOS_TOKEN_HIT; ++n_gen; break; }
        if (special_stop) { stop = KCPP_STOP_EOS_TOKEN_HIT; ++n_gen; break; }
        if (hit) { stop = KCPP_STOP_CUSTOM_STOPPER; ++n_gen; break; }
        if (rewound) continue;
        if ((int)e->ctx.size() >= e->hp.n_ctx - 1) { ++n_gen; break; }
        const int32_t tt = t;
        int frc;
        const auto tf0 = std::chrono::steady_clock::now();
        if (on_dev) {
            // the greedy token is the device argmax: the step takes it from the device (no host-to-device copy, no
            // second argmax launch -- the bench's decode_greedy loop, koboldcpp --benchmark's settings hit this)
            HipOps o(*e);
            frc = (!e->dev_tok && o.token_home()) ? -1 : greedy_step(o, (int)e->ctx.size());
            e->dev_tok = frc == 0;
        } else {
            frc = forward(*e, &tt, 1, (int)e->ctx.size());
            e->dev_tok = frc == 0 && e->stages.size() == 1;     // one stage: its argmax also wrote the token input
        }
        tm_step += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
        if (frc) { fprintf(stderr, "[kcpp] generate: decode failed\n"); break; }
        e->ctx.push_back(t);
    }
    if (link_errors(*e)) fprintf(stderr, "[kcpp] generate: a linked hand-off timed out; the tokens after it are invalid\n");
    if (getenv("KCPP_GEN_TIMING"))
        fprintf(stderr, "[kcpp] generate timing: %d tokens, sample %.3f ms/token, step enqueue %.3f ms/token\n", n_gen,
                tm_sample / std::max(1, n_gen), tm_step / std::max(1, n_gen));
    while (!delayed.empty()) {               // flush what the delay line still holds (:3497-3505)
        if (!hit) emit(delayed.front());
        delayed.pop_front();
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

// GGUF header / tensor-table validation alone (the first step of load_model): 0 when the file parses, else -1 with
// the reason in err (tests/test_gguf_loader.py)
// the BPE pre-tokenizer alone (tests): byte end offsets of the words of text under pre-tokenizer type `pre` (the
// GGUF tokenizer.ggml.pre value); returns the word count (at most cap offsets written)
int kcpp_pretokenize(const char *pre, const char *text, int64_t *ends, int cap) {
    if (!pre || !text) return -1;
    const std::vector<size_t> e = Tokenizer::pretokenize_offsets(std::string(pre), std::string(text));
    for (size_t i = 0; i < e.size() && (int)i < cap; ++i) ends[i] = (int64_t)e[i];
    return (int)e.size();
}

// the GGUF's tokenizer alone (tests, host only): token ids of text (generate()'s tokenization: special tokens
// parsed, BOS per the vocabulary when add_bos); returns the count (at most cap written), -1 on a load error
int kcpp_tokenize_probe(const char *gguf_path, const char *text, int add_bos, int32_t *out, int cap) {
    gguf::File f;
    std::string err;
    Tokenizer tk;
    if (!gguf_path || !text || !f.open(gguf_path, err) || !tk.init(f, err)) {
        if (!err.empty()) fprintf(stderr, "[kcpp] tokenize_probe: %s\n", err.c_str());
        return -1;
    }
    const std::vector<int> ids = tk.encode(std::string(text), add_bos != 0);
    for (size_t i = 0; i < ids.size() && (int)i < cap; ++i) out[i] = ids[i];
    return (int)ids.size();
}

// the GGUF's tokenizer alone (tests, host only): every vocabulary id's streamed text (generate()'s piece rendering)
// concatenated into out (at most cap bytes), ends[i] = end offset of id i's piece (at most n_ends written);
// returns the vocabulary size, -1 on a load error
int kcpp_pieces_probe(const char *gguf_path, char *out, int64_t cap, int64_t *ends, int n_ends) {
    gguf::File f;
    std::string err;
    Tokenizer tk;
    if (!gguf_path || !f.open(gguf_path, err) || !tk.init(f, err)) return -1;
    int64_t o = 0;
    for (int i = 0; i < tk.n_vocab(); ++i) {
        const std::string p = tk.piece(i);
        if (out && o + (int64_t)p.size() <= cap) memcpy(out + o, p.data(), p.size());
        o += (int64_t)p.size();
        if (ends && i < n_ends) ends[i] = o;
    }
    return tk.n_vocab();
}

// bench.py --gpus N (N > 1): the drop-in engine over n_dev GPUs -- load_model's stages (build_stages), hand-off
// (init_handoff: RCCL clique over distinct GPUs), forward() -- with synthetic weights instead of a GGUF.  Prefill of
// n_prompt ids in ubatches of ub (timed to the last stage's drain), then n_warm + n_steps greedy tokens by
// greedy_step: argmax on the last stage, the token moved home to stage 0 on device, no host synchronisation inside
// a step (generate() reads each token on the host: its samplers and stop checks run there, as the reference's).
// out = {prefill_s, decode_s (the n_steps timed tokens), n_past at the end, 1 when the hand-off is RCCL}.
int kcpp_engine_bench(const kcpp_hparams *hp, const int *types, int n_types, int n_dev, const float *tensor_split,
                      uint64_t seed, int n_prompt, int ub, int n_warm, int n_steps, double *out) {
    if (!hp || !types || !out || n_dev < 1 || n_prompt < 1 || n_prompt + n_warm + n_steps + 1 > hp->n_ctx) return -2;
    int nreal = 0;                          // KCPP_VIRTUAL_DEVICES (tests): several stages per GPU, stage i on GPU i % nreal
    if (hipGetDeviceCount(&nreal) != hipSuccess || nreal < 1 || (nreal < n_dev && !getenv("KCPP_VIRTUAL_DEVICES"))) {
        fprintf(stderr, "[kcpp] engine_bench: %d GPUs requested, %d visible\n", n_dev, nreal);
        return -1;
    }
    nreal = std::min(nreal, n_dev);
    auto e = std::make_unique<Engine>();
    e->hp = *hp;
    e->types.assign(types, types + n_types);
    e->ub = std::max(1, std::min(ub, 512));
    float ts[KCPP_TENSOR_SPLIT_MAX] = {0};
    for (int i = 0; i < n_dev && i < KCPP_TENSOR_SPLIT_MAX; ++i) ts[i] = tensor_split ? tensor_split[i] : 1.0f;
    if (!build_stages(*e, n_dev, nreal, ts, false, 0) || !init_handoff(*e)) return -3;
    for (kcpp_model *m : e->stages)
        if (kcpp_model_synth_weights(m, seed)) return -4;
    std::vector<int32_t> prompt(n_prompt);
    for (int i = 0; i < n_prompt; ++i) prompt[i] = 16 + (i % 2);          // the " 1" pattern of bench.py
    kcpp_model *last = e->stages.back();
    HipOps o(*e);
    auto sync_all = [&]() {
        for (kcpp_model *m : e->stages)
            if (kcpp_model_sync(m)) return -1;
        return 0;
    };
    // warm-up: a short prefill (first touch, graph capture on every stage)
    if (forward(o, prompt.data(), std::min(64, n_prompt), 0) || kcpp_model_sync(last)) return -5;
    const auto t0 = std::chrono::steady_clock::now();
    if (forward(o, prompt.data(), n_prompt, 0) || kcpp_model_sync(last)) return -5;
    const auto t1 = std::chrono::steady_clock::now();
    int n_past = n_prompt;
    std::chrono::steady_clock::time_point t2 = t1;
    // greedy tokens without the host: the prefill's token goes home on device, then every step's token too
    if (o.argmax_dev() || o.token_home()) return -6;
    std::chrono::steady_clock::time_point te = t1;
    for (int i = 0; i < n_warm + n_steps; ++i) {
        if (i == n_warm) {
            if (sync_all()) return -6;
            t2 = std::chrono::steady_clock::now();
        }
        if (greedy_step(o, n_past)) return -6;
        ++n_past;
    }
    te = std::chrono::steady_clock::now();                             // host: every step enqueued
    if (sync_all()) return -6;                                         // the last token computed and home
    if (link_errors(*e)) return -7;
    const auto t3 = std::chrono::steady_clock::now();
    if (getenv("KCPP_ENGINE_HOST_TIMING"))
        fprintf(stderr, "[kcpp] engine_bench: %zu stages, host enqueue %.1f us/token, wall %.1f us/token\n",
                e->stages.size(), std::chrono::duration<double>(te - t2).count() * 1e6 / n_steps,
                std::chrono::duration<double>(t3 - t2).count() * 1e6 / n_steps);
    out[0] = std::chrono::duration<double>(t1 - t0).count();
    out[1] = std::chrono::duration<double>(t3 - t2).count();
    out[2] = n_past;
    out[3] = e->comms.empty() ? 0.0 : 1.0;
    return 0;
}

// bench / test hook (not part of koboldcpp's ABI): replace the loaded model's weights by the runtime's synthetic weights
// (kcpp_model_synth_weights on every stage).  bench.py's generate() leg loads a full-size GGUF whose tensor data is a
// sparse-file hole (no checkpoints exist offline) and synthesizes the weights on the device; the context is dropped.
int kcpp_expose_synth_weights(uint64_t seed) {
    Engine *e = g_eng.get();
    if (!e) return -1;
    for (kcpp_model *m : e->stages)
        if (kcpp_model_synth_weights(m, seed)) return -2;
    e->ctx.clear();
    return 0;
}

// test hook (tests/test_pipeline.py): load_model's layer placement (split_layers): out[i] = device of layer i for
// i < n_layer, out[n_layer] = the output head's device
int kcpp_split_layers(int n_layer, int n_dev, const float *tensor_split, int *out) {
    if (n_layer < 1 || n_dev < 1 || n_dev > KCPP_TENSOR_SPLIT_MAX || !tensor_split || !out) return -1;
    const std::vector<int> d = split_layers(n_layer, n_dev, tensor_split);
    for (int i = 0; i <= n_layer; ++i) out[i] = d[i];
    return 0;
}

// test hook (tests/test_pipeline.py): the enqueue order of the pipeline schedule for n_stages stages -- a prefill of
// T tokens at n_past in ubatches of ub, the last stage's argmax and its way home, then `steps` greedy steps -- as
// TraceOps records it (space-separated into out).  Returns the length written, -1 on bad arguments.
int kcpp_pipeline_trace(int n_stages, int ub, int T, int n_past, int steps, char *out, int cap) {
    if (n_stages < 1 || ub < 1 || T < 1 || !out || cap < 1) return -1;
    TraceOps o((size_t)n_stages, ub);
    std::vector<int32_t> toks((size_t)T, 1);
    if (forward(o, toks.data(), T, n_past) || o.argmax_dev() || o.token_home()) return -1;
    for (int i = 0; i < steps; ++i)
        if (greedy_step(o, n_past + T + i)) return -1;
    snprintf(out, (size_t)cap, "%s", o.log.c_str());
    return (int)std::min<size_t>(o.log.size(), (size_t)cap - 1);
}

int kcpp_tokenizer_special_ids(const char *gguf_path, int32_t *out) {
    gguf::File f;
    std::string err;
    Tokenizer tk;
    if (!gguf_path || !out || !f.open(gguf_path, err) || !tk.init(f, err)) return -1;
    out[0] = tk.bos(); out[1] = tk.eos(); out[2] = tk.eot();
    return 0;
}

int kcpp_gguf_check(const char *path, char *err, int err_len) {
    gguf::File f;
    std::string e;
    const bool ok = path && f.open(path, e);
    if (err && err_len > 0) snprintf(err, (size_t)err_len, "%s", ok ? "" : e.c_str());
    return ok ? 0 : -1;
}

// test hook (tests/test_sampler.py): the restated SampleLogits chain on caller logits.  fp = {top_k, top_a, top_p,
// min_p, typical_p, tfs, temp, rep_pen, rep_pen_slope, presence_penalty, mirostat_tau, mirostat_eta, dry_multiplier,
// dry_base, xtc_threshold, xtc_probability, dynatemp_range, dynatemp_exponent, smoothing_factor}; ip = {rep_pen_range,
// mirostat, dry_allowed_length, dry_penalty_last_n}; restarts: n_restart (head, tail length, tail...) records.
// Writes up to cap candidates (id, p) left after the chain (before the draw; mirostat: after its own top-k) and
// returns the drawn token, or -1 on bad arguments.
int kcpp_sampler_probe(const float *logits, int n_vocab, int n_ctx, const float *fp, const int *ip, const int *order,
                       int n_order, const int *ctx_toks, int n_ctx_toks, const int *last_n, int n_last,
                       const int *restarts, int n_restart_ints, unsigned seed, float *mu, int *out_ids, float *out_p,
                       int cap, int *out_n) {
    if (!logits || n_vocab <= 0 || !fp || !ip) return -1;
    ksamp::Params P;
    P.top_k = fp[0]; P.top_a = fp[1]; P.top_p = fp[2]; P.min_p = fp[3]; P.typical_p = fp[4]; P.tfs = fp[5]; P.temp = fp[6];
    P.rep_pen = fp[7]; P.rep_pen_slope = fp[8]; P.presence_penalty = fp[9]; P.mirostat_tau = fp[10]; P.mirostat_eta = fp[11];
    P.dry_multiplier = fp[12]; P.dry_base = fp[13]; P.xtc_threshold = fp[14]; P.xtc_probability = fp[15];
    P.dynatemp_range = fp[16]; P.dynatemp_exponent = fp[17]; P.smoothing_factor = fp[18];
    P.rep_pen_range = ip[0]; P.mirostat = ip[1]; P.dry_allowed_length = ip[2]; P.dry_penalty_last_n = ip[3];
    for (int i = 0; i < n_order; ++i) P.order.push_back(order[i]);
    ksamp::RestartSeqs rs;
    for (int i = 0; i + 1 < n_restart_ints;) {
        const int head = restarts[i], len = restarts[i + 1];
        if (len < 0 || i + 2 + len > n_restart_ints) return -1;
        rs.emplace(head, std::vector<int>(restarts + i + 2, restarts + i + 2 + len));
        i += 2 + len;
    }
    const std::vector<int> ctxv(ctx_toks, ctx_toks + n_ctx_toks), lastv(last_n, last_n + n_last);
    std::mt19937 rng(seed);
    std::vector<ksamp::TokData> cand;
    int tok;
    ksamp::Cands c;
    if (P.mirostat == 1 || P.mirostat == 2) {
        std::mt19937 rng2(seed);
        float mu2 = *mu;
        tok = ksamp::sample_logits(logits, n_ctx, n_vocab, P, {}, rs, ctxv, lastv, rng2, &mu2);
        *mu = mu2;
        c = ksamp::Cands{nullptr, 0, false};
    } else {
        c = ksamp::apply_chain(cand, logits, n_ctx, n_vocab, P, {}, rs, ctxv, lastv, rng, false);
        ksamp::Cands c2 = c;
        std::vector<ksamp::TokData> keep(c.data, c.data + c.size);
        ksamp::Cands ck{keep.data(), keep.size(), c.sorted};
        tok = ksamp::draw(&ck, rng);
        (void)c2;
        ksamp::softmax(&c);             // the probabilities the draw used
    }
    const int n = (int)std::min<size_t>(c.size, (size_t)std::max(cap, 0));
    for (int i = 0; i < n; ++i) { out_ids[i] = c.data[i].id; out_p[i] = c.data[i].p; }
    if (out_n) *out_n = (int)c.size;
    return tok;
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
