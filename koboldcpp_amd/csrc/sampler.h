// sampler.h -- koboldcpp's host-side sampler chain, restated (gpttype_adapter.cpp:483-1434).
//
// The reference samples on the host from the last position's logits: logit biases, (grammar), DRY,
// a top-5000 prefilter, then either mirostat v1/v2 or the user's sampler_order over
// {top_k, top_a, top_p + min_p, tfs, typical, temperature (dynatemp / smoothing), rep_pen}, XTC last,
// and one draw from std::discrete_distribution over mt19937.  Every function below follows the
// reference function named in its comment, including its sort / tie / min_keep behaviour, so that a
// given seed draws the same token from the same logits (same libstdc++ distributions).
// Grammar-constrained sampling is outside SURVEY.md 8 and is not provided.
#pragma once

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <numeric>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

namespace ksamp {

struct TokData {          // llama_token_data
    int id;
    float logit;
    float p;
};
struct Cands {            // llama_token_data_array: data + size + sorted
    TokData *data;
    size_t size;
    bool sorted;
};

enum { S_TOP_K = 0, S_TOP_A = 1, S_TOP_P = 2, S_TFS = 3, S_TYP = 4, S_TEMP = 5, S_REP_PEN = 6 };   // expose.h:12-22

// restart sequences: head token -> tails (gpttype_adapter.cpp:114)
using RestartSeqs = std::unordered_multimap<int, std::vector<int>>;

struct Params {
    float top_k = 0, top_a = 0, top_p = 1, min_p = 0, typical_p = 1, tfs = 1, temp = 1;
    int rep_pen_range = 1;         // last_n_size (repeat_last_n, >= 1)
    float rep_pen = 1, rep_pen_slope = 1, presence_penalty = 0;
    int mirostat = 0;
    float mirostat_tau = 5, mirostat_eta = 0.1f;
    float dry_multiplier = 0, dry_base = 0;
    int dry_allowed_length = 0, dry_penalty_last_n = 0;
    float xtc_threshold = 0, xtc_probability = 0;
    float dynatemp_range = 0, dynatemp_exponent = 1, smoothing_factor = 0;
    std::vector<int> order;        // sampler_order
};

// sample_softmax, gpttype_adapter.cpp:483-506
inline void softmax(Cands *c) {
    if (!c->sorted) {
        std::sort(c->data, c->data + c->size, [](const TokData &a, const TokData &b) { return a.logit > b.logit; });
        c->sorted = true;
    }
    const float mx = c->data[0].logit;
    float cum = 0.0f;
    for (size_t i = 0; i < c->size; ++i) {
        const float p = expf(c->data[i].logit - mx);
        c->data[i].p = p;
        cum += p;
    }
    for (size_t i = 0; i < c->size; ++i) c->data[i].p /= cum;
}

// sample_top_k, gpttype_adapter.cpp:508-583 (partial sort for k <= 128, 128-bucket histogram above)
inline void top_k(Cands *c, int k) {
    if (k <= 0) k = (int)c->size;
    k = std::max(k, 1);
    k = std::min(k, (int)c->size);
    if (!c->sorted) {
        auto comp = [](const TokData &a, const TokData &b) { return a.logit > b.logit; };
        if (k <= 128) {
            std::partial_sort(c->data, c->data + k, c->data + c->size, comp);
        } else {
            constexpr int nb = 128;
            constexpr float lo = -10.0f, hi = 10.0f;
            constexpr float scale = nb / (hi - lo);
            constexpr float inter = -lo * scale;
            std::vector<int> bidx(c->size), histo(nb, 0);
            for (int i = 0; i < (int)c->size; ++i) {
                int ib = int(scale * c->data[i].logit + inter);
                ib = std::max(0, std::min(nb - 1, ib));
                bidx[i] = ib;
                ++histo[ib];
            }
            int nhave = 0, ib = nb - 1;
            for (; ib >= 0; --ib) {
                nhave += histo[ib];
                if (nhave >= k) break;
            }
            std::vector<TokData> tmp(nhave);
            TokData *ptr = tmp.data();
            std::vector<TokData *> bptr;
            bptr.reserve(nb - ib);
            for (int j = nb - 1; j >= ib; --j) { bptr.push_back(ptr); ptr += histo[j]; }
            for (int i = 0; i < (int)c->size; ++i) {
                const int j = bidx[i];
                if (j >= ib) *bptr[nb - 1 - j]++ = c->data[i];
            }
            ptr = tmp.data();
            int ndone = 0;
            for (int j = nb - 1; j > ib; --j) {
                std::sort(ptr, ptr + histo[j], comp);
                ptr += histo[j];
                ndone += histo[j];
            }
            std::partial_sort(ptr, ptr + k - ndone, ptr + histo[ib], comp);
            std::memcpy(c->data, tmp.data(), k * sizeof(TokData));
        }
        c->sorted = true;
    }
    c->size = k;
}

// sample_token, gpttype_adapter.cpp:585-612
inline int draw(Cands *c, std::mt19937 &rng) {
    softmax(c);
    std::vector<float> probs;
    probs.reserve(c->size);
    for (size_t i = 0; i < c->size; ++i) probs.push_back(c->data[i].p);
    std::discrete_distribution<> dist(probs.begin(), probs.end());
    return c->data[dist(rng)].id;
}

// sample_token_mirostat, gpttype_adapter.cpp:614-643
inline int mirostat_v1(int n_vocab, Cands *c, std::mt19937 &rng, float tau, float eta, int m, float *mu) {
    const float N = float(n_vocab);
    softmax(c);
    float sum_ti_bi = 0.0f, sum_ti_sq = 0.0f;
    for (size_t i = 0; i < size_t(m - 1) && i < c->size - 1; ++i) {
        const float t_i = logf(float(i + 2) / float(i + 1));
        const float b_i = logf(c->data[i].p / c->data[i + 1].p);
        sum_ti_bi += t_i * b_i;
        sum_ti_sq += t_i * t_i;
    }
    const float s_hat = sum_ti_bi / sum_ti_sq;
    const float eps_hat = s_hat - 1;
    const float k = powf((eps_hat * powf(2, *mu)) / (1 - powf(N, -eps_hat)), 1 / s_hat);
    top_k(c, int(k));
    const int X = draw(c, rng);
    size_t xi = 0;
    while (xi < c->size && c->data[xi].id != X) ++xi;
    const float e = -log2f(c->data[xi].p) - tau;
    *mu = *mu - eta * e;
    return X;
}

// sample_token_mirostat_v2, gpttype_adapter.cpp:645-671
inline int mirostat_v2(Cands *c, std::mt19937 &rng, float tau, float eta, float *mu) {
    softmax(c);
    size_t n = 0;
    while (n < c->size && !(-log2f(c->data[n].p) > *mu)) ++n;
    c->size = n == 0 ? 1 : n;
    softmax(c);
    const int X = draw(c, rng);
    size_t xi = 0;
    while (xi < c->size && c->data[xi].id != X) ++xi;
    const float e = -log2f(c->data[xi].p) - tau;
    *mu = *mu - eta * e;
    return X;
}

// sample_top_a, gpttype_adapter.cpp:675-701
inline void top_a(Cands *c, float a, size_t min_keep) {
    if (a <= 0.0f || c->size <= 1) return;
    softmax(c);
    const float mp = c->data[0].p, thr = a * mp * mp;
    size_t last = c->size;
    for (size_t i = 0; i < c->size; ++i)
        if (c->data[i].p < thr && i >= min_keep) { last = i; break; }
    c->size = last;
}

// sample_xtc, gpttype_adapter.cpp:703-742
inline void xtc(Cands *c, float threshold, float probability, std::mt19937 &rng) {
    if (threshold > 0.5f || probability <= 0.0f || c->size <= 1) return;
    std::uniform_real_distribution<float> dist(0.0f, 1.0f);
    if (dist(rng) >= probability) return;
    softmax(c);
    size_t last = c->size;
    for (size_t i = 0; i < c->size; ++i)
        if (c->data[i].p < threshold) { last = i; break; }
    if (last > 1) {
        for (size_t i = 0; i < last - 1; ++i) c->data[i].logit -= 999.0f;
        c->sorted = false;
    }
}

// sample_dry, gpttype_adapter.cpp:744-948 (restart-sequence limit, reverse Z-algorithm, per-token max repeat)
inline void dry(int n_ctx, int range, float mult, float base, int allowed, const RestartSeqs &restarts,
                const std::vector<int> &ctx_tokens, Cands *c) {
    if (mult <= 0.0f || base <= 0.0f) return;
    if (range <= 0 || range > n_ctx) range = n_ctx;
    const int nrep = std::min(std::min((int)ctx_tokens.size(), range), n_ctx);
    if (nrep <= allowed) return;
    const int *last_tokens = ctx_tokens.data() + ctx_tokens.size() - nrep;
    std::vector<int> rc(nrep, 0);
    int rep_limit = nrep;
    for (size_t i = 0; i < (size_t)nrep; ++i) {
        const size_t ix = nrep - 1 - i;
        auto its = restarts.equal_range(last_tokens[ix]);
        if (its.first == restarts.end()) continue;
        int longest = -1;
        for (auto it = its.first; it != its.second; ++it) {
            const int sl = (int)it->second.size();
            if (sl > longest && sl <= (int)i) {
                bool match = true;
                for (size_t o = 0; o < (size_t)sl; ++o)
                    if (it->second[o] != last_tokens[ix + 1 + o]) { match = false; break; }
                if (match) longest = sl;
            }
        }
        if (longest >= 0) { rep_limit = (int)i - longest; break; }
    }
    if (rep_limit <= allowed) return;
    {
        const int last = nrep - 1;
        int rt = 0, lt = 0;
        for (int k = 1; k < nrep; ++k) {
            if (k > rt) {
                int n = 0;
                while (n + k < nrep && last_tokens[last - n] == last_tokens[last - (n + k)]) ++n;
                rc[last - k] = std::min(n, rep_limit);
                if (n > 0) { lt = k; rt = k + n - 1; }
            } else {
                const int p = k - lt, right = rt - k + 1;
                if (rc[last - p] < right) {
                    rc[last - k] = std::min(rc[last - p], rep_limit);
                } else {
                    int i = rt + 1;
                    while (i < nrep && last_tokens[last - i] == last_tokens[last - (i - k)]) i += 1;
                    rc[last - k] = std::min(i - k, rep_limit);
                    lt = k;
                    rt = i - 1;
                }
            }
        }
    }
    std::unordered_map<int, int> maxrep;
    for (size_t i = 0; i + 1 < (size_t)nrep; ++i) {
        const int len = rc[i];
        if (len >= allowed) {
            const int tok = last_tokens[i + 1];
            auto it = maxrep.find(tok);
            if (it == maxrep.end() || it->second < len) maxrep[tok] = len;
        }
    }
    const float FLOAT_MAX_LOG = 88.7228391f;
    int max_exp = 0;
    if (base > 1.000001f) max_exp = (int)(FLOAT_MAX_LOG / std::log(base));
    size_t count = 0;
    for (const auto &kv : maxrep) {
        int e = kv.second - allowed;
        if (max_exp > 0 && e > max_exp) e = max_exp;
        const float penalty = mult * pow(base, e);                // pow(float, int) is double, as in the reference
        c->data[kv.first].logit -= penalty;                        // candidates are still id-indexed here
        ++count;
    }
    if (count > 0) c->sorted = false;
}

// sample_rep_pen, gpttype_adapter.cpp:950-1007 (near half at full penalty, far half at the sloped penalty)
inline void rep_pen(int n_ctx, int range, float pen, float slope, float presence, const std::vector<int> &last_n, Cands *c) {
    const int nrep = std::min(std::min((int)last_n.size(), range), n_ctx);
    const int *lt = last_n.data() + last_n.size() - nrep;
    if (nrep == 0 || (pen == 1.0f && presence == 0)) return;
    std::unordered_map<int, int> near, far;
    for (size_t i = 0; i < (size_t)nrep; ++i) {
        if ((i * 2) >= (size_t)nrep) near[lt[i]]++;
        else far[lt[i]]++;
    }
    float reduced = pen;
    if (reduced > 1.0f) reduced = 1.0f + ((pen - 1.0f) * slope);
    for (size_t i = 0; i < c->size; ++i) {
        const bool in_near = near.count(c->data[i].id) != 0, in_far = far.count(c->data[i].id) != 0;
        if (!in_near && !in_far) continue;
        const float penalty = in_near ? pen : reduced;
        if (c->data[i].logit <= 0) c->data[i].logit *= penalty;
        else c->data[i].logit /= penalty;
        c->data[i].logit -= presence;
    }
    c->sorted = false;
}

// sample_top_p, gpttype_adapter.cpp:1009-1033
inline void top_p(Cands *c, float p, size_t min_keep) {
    if (p >= 1.0f) return;
    softmax(c);
    float cum = 0.0f;
    size_t last = c->size;
    for (size_t i = 0; i < c->size; ++i) {
        cum += c->data[i].p;
        if (cum >= p && i + 1 >= min_keep) { last = i + 1; break; }
    }
    c->size = last;
}

// sample_min_p, gpttype_adapter.cpp:1035-1088 (unsorted fast path, sorted fallback)
inline void min_p(Cands *c, float p, size_t min_keep) {
    if (p <= 0.0f || !c->size) return;
    bool applied = false;
    if (!c->sorted) {
        std::vector<TokData> kept;
        float mx = -FLT_MAX;
        for (size_t i = 0; i < c->size; ++i) mx = std::max(mx, c->data[i].logit);
        const float min_logit = mx + logf(p);
        for (size_t i = 0; i < c->size; ++i)
            if (c->data[i].logit >= min_logit) kept.push_back(c->data[i]);
        if (kept.size() >= min_keep) {
            std::memcpy(c->data, kept.data(), kept.size() * sizeof(TokData));
            c->size = kept.size();
            applied = true;
        }
    }
    if (!applied) {
        if (!c->sorted) {
            std::sort(c->data, c->data + c->size, [](const TokData &a, const TokData &b) { return a.logit > b.logit; });
            c->sorted = true;
        }
        const float min_logit = c->data[0].logit + logf(p);
        size_t i = 1;
        for (; i < c->size; ++i)
            if (c->data[i].logit < min_logit && i >= min_keep) break;
        c->size = i;
    }
}

// sample_tail_free, gpttype_adapter.cpp:1090-1142
inline void tail_free(Cands *c, float z, size_t min_keep) {
    if (z >= 1.0f || c->size <= 2) return;
    softmax(c);
    std::vector<float> d1(c->size - 1), d2(c->size - 2);
    for (size_t i = 0; i < d1.size(); ++i) d1[i] = c->data[i].p - c->data[i + 1].p;
    for (size_t i = 0; i < d2.size(); ++i) d2[i] = std::abs(d1[i] - d1[i + 1]);
    const float s = std::accumulate(d2.begin(), d2.end(), 0.0f);
    if (s > 1e-6f) for (float &v : d2) v /= s;
    else for (float &v : d2) v = 1.0f / d2.size();
    float cum = 0.0f;
    size_t last = c->size;
    for (size_t i = 0; i < d2.size(); ++i) {
        cum += d2[i];
        if (cum > z && i >= min_keep) { last = i; break; }
    }
    c->size = last;
}

// sampler_typical, gpttype_adapter.cpp:1144-1203
inline void typical(Cands *c, float p, size_t min_keep) {
    if (p >= 1.0f) return;
    softmax(c);
    float ent = 0.0f;
    for (size_t i = 0; i < c->size; ++i)
        if (c->data[i].p > 0) ent += -c->data[i].p * logf(c->data[i].p);
    std::vector<float> sh;
    for (size_t i = 0; i < c->size; ++i) sh.push_back(fabsf(-logf(c->data[i].p) - ent));
    std::vector<size_t> idx(c->size);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return sh[a] < sh[b]; });
    float cum = 0.0f;
    size_t last = idx.size();
    for (size_t i = 0; i < idx.size(); ++i) {
        cum += c->data[idx[i]].p;
        if (cum > p && i >= min_keep - 1) { last = i + 1; break; }
    }
    std::vector<TokData> nw;
    for (size_t i = 0; i < last; ++i) nw.push_back(c->data[idx[i]]);
    std::copy(nw.begin(), nw.end(), c->data);
    c->size = nw.size();
    c->sorted = false;
}

inline void smooth(Cands *c, float f) {      // quadratic smoothing (shared by temperature and entropy)
    softmax(c);
    const float h = c->data[0].logit;
    for (size_t i = 0; i < c->size; ++i) {
        const float s = c->data[i].logit - h;
        c->data[i].logit = -f * s * s + h;
    }
    softmax(c);
}

// sample_entropy (dynamic temperature), gpttype_adapter.cpp:1205-1263
inline void entropy(Cands *c, float tmin, float tmax, float expo, float smoothing) {
    if (c->size <= 1) return;
    const float max_ent = -logf(1.0f / c->size);
    softmax(c);
    float ent = 0.0f;
    for (size_t i = 0; i < c->size; ++i)
        if (c->data[i].p > 0.0f) ent -= c->data[i].p * logf(c->data[i].p);
    const float dyn = tmin + (tmax - tmin) * powf(ent / max_ent, expo);
    for (size_t i = 0; i < c->size; ++i) c->data[i].logit /= dyn;
    const double mx = c->data[0].logit;
    double cum = 0.0;
    for (size_t i = 0; i < c->size; ++i) {
        const double p = exp(c->data[i].logit - mx);
        c->data[i].p = (float)p;
        cum += p;
    }
    for (size_t i = 0; i < c->size; ++i) c->data[i].p /= cum;
    if (smoothing > 0 && c->size > 1) smooth(c, smoothing);
}

// sample_temperature, gpttype_adapter.cpp:1265-1296 (temp <= 0: 1/256 then top-1)
inline void temperature(Cands *c, float temp, float smoothing) {
    bool greedy = false;
    if (temp <= 0) { temp = 0.00390625f; smoothing = 0; greedy = true; }
    for (size_t i = 0; i < c->size; ++i) c->data[i].logit /= temp;
    if (smoothing > 0 && c->size > 1) smooth(c, smoothing);
    if (greedy) top_k(c, 1);
}

// SampleLogits, gpttype_adapter.cpp:1338-1434 (grammar omitted).  `logits` already carries the EOS /
// banned-token suppression the caller applies (gpttype_adapter.cpp:3200-3224).  mirostat_mu is the
// function-static of the reference (initialised once per process to 2 * tau).
struct LogitBias { int token_id; float bias; };

// the candidate chain of SampleLogits up to (not including) the final draw: biases, DRY, top-5000, then the
// user's sampler order and XTC.  `cand` holds the candidates; returns the array view.  (mirostat: not here)
inline Cands apply_chain(std::vector<TokData> &cand, const float *logits, int n_ctx, int n_vocab, const Params &P,
                         const std::vector<LogitBias> &biases, const RestartSeqs &restarts,
                         const std::vector<int> &ctx_tokens, const std::vector<int> &last_n, std::mt19937 &rng,
                         bool stop_before_order) {
    cand.clear();
    cand.reserve(n_vocab);
    for (int t = 0; t < n_vocab; ++t) cand.push_back(TokData{t, logits[t], 0.0f});
    for (const LogitBias &b : biases) cand[b.token_id].logit += b.bias;
    Cands c{cand.data(), cand.size(), false};
    dry(n_ctx, P.dry_penalty_last_n, P.dry_multiplier, P.dry_base, P.dry_allowed_length, restarts, ctx_tokens, &c);
    top_k(&c, 5000);
    if (stop_before_order) return c;
    for (int s : P.order) {
        switch (s) {
        case S_TOP_K: top_k(&c, (int)P.top_k); break;
        case S_TOP_A: top_a(&c, P.top_a, 1); break;
        case S_TOP_P: top_p(&c, P.top_p, 1); min_p(&c, P.min_p, 1); break;
        case S_TFS: tail_free(&c, P.tfs, 1); break;
        case S_TYP: typical(&c, P.typical_p, 1); break;
        case S_TEMP:
            if (P.dynatemp_range > 0) {
                const float lo = std::max(0.0f, P.temp - P.dynatemp_range), hi = std::max(0.0f, P.temp + P.dynatemp_range);
                entropy(&c, lo, hi, std::max(0.0f, P.dynatemp_exponent), P.smoothing_factor);
            } else {
                temperature(&c, P.temp, P.smoothing_factor);
            }
            break;
        case S_REP_PEN: rep_pen(n_ctx, P.rep_pen_range, P.rep_pen, P.rep_pen_slope, P.presence_penalty, last_n, &c); break;
        default: break;
        }
    }
    xtc(&c, P.xtc_threshold, P.xtc_probability, rng);
    return c;
}

// SampleLogits, gpttype_adapter.cpp:1338-1434 (grammar omitted).  `logits` already carries the EOS /
// banned-token suppression the caller applies (gpttype_adapter.cpp:3200-3224).  mirostat_mu is the
// function-static of the reference (initialised once per process to 2 * tau).
inline int sample_logits(const float *logits, int n_ctx, int n_vocab, const Params &P, const std::vector<LogitBias> &biases,
                         const RestartSeqs &restarts, const std::vector<int> &ctx_tokens, const std::vector<int> &last_n,
                         std::mt19937 &rng, float *mirostat_mu) {
    std::vector<TokData> cand;
    const bool miro = P.mirostat == 1 || P.mirostat == 2;
    Cands c = apply_chain(cand, logits, n_ctx, n_vocab, P, biases, restarts, ctx_tokens, last_n, rng, miro);
    if (miro) {
        rep_pen(n_ctx, P.rep_pen_range, P.rep_pen, P.rep_pen_slope, P.presence_penalty, last_n, &c);
        temperature(&c, P.temp, P.smoothing_factor);
        if (P.mirostat == 1) return mirostat_v1(n_vocab, &c, rng, P.mirostat_tau, P.mirostat_eta, 100, mirostat_mu);
        return mirostat_v2(&c, rng, P.mirostat_tau, P.mirostat_eta, mirostat_mu);
    }
    return draw(&c, rng);
}

// LowestLogit, gpttype_adapter.cpp:294-303
inline float lowest_logit(const float *l, size_t n) {
    if (n == 0) return 0.0f;
    const float v = *std::min_element(l, l + n);
    return v < 0 ? (v - 8) : 0;
}

}  // namespace ksamp
