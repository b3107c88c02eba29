// ref_sampler.cpp -- TEST INFRASTRUCTURE ONLY (tests/test_sampler_ref.py).  Never linked into the product.
//
// Runs the reference's own SampleLogits (gpttype_adapter.cpp:1338-1434) on caller logits: this harness includes
// /root/reference/gpttype_adapter.cpp as one translation unit, exactly as the reference's Makefile compiles it
// (Makefile:557-560), sets the file-scope state SampleLogits reads (last_n_tokens / current_context_tokens for
// sample_rep_pen and sample_dry, dry_sequence_breakers; no logit biases, no grammar) and prints the drawn token.
// Symbols of the reference's other translation units that the sampler never reaches stay unresolved at link time
// (oracle/Makefile ref_sampler): nothing else of the reference runs.
//
// stdin: one or more cases, each
//   int32 n_vocab, n_ctx, n_order, n_ctx_toks, n_last, n_restart_ints; uint32 seed; float mu (unused: mirostat
//   starts at SampleLogits' own static 2 tau, so a mirostat case must be the first of its process);
//   float fp[19]; int32 ip[4]; int32 order[n_order], ctx[n_ctx_toks], last_n[n_last], restarts[n_restart_ints];
//   float logits[n_vocab]
// (fp / ip / restart records as kcpp_sampler_probe, koboldcpp_amd/csrc/expose.cpp).  stdout: one line per case,
// "token".
#include "gpttype_adapter.cpp"

#include <cstdio>
#include <cstring>

static bool rd(void *p, size_t n) { return fread(p, 1, n, stdin) == n; }

int main(int argc, char **argv) {
    // "rope" mode: lines "original_base n_ctx_train n_ctx_desired solar" -> the reference's
    // CalcGradientAIRopeFreqBase (gpttype_adapter.cpp:1598) of them, printed exactly (%.9g)
    if (argc > 1 && !strcmp(argv[1], "rope")) {
        float base;
        int train, want, solar;
        while (scanf("%f %d %d %d", &base, &train, &want, &solar) == 4)
            printf("%.9g\n", CalcGradientAIRopeFreqBase(base, train, want, solar ? GGUFArch::ARCH_SOLAR : GGUFArch::ARCH_DEFAULT));
        return 0;
    }
    for (;;) {
        int32_t h[6];
        uint32_t seed;
        float mu, fp[19];
        int32_t ip[4];
        if (!rd(h, sizeof h)) break;
        if (!rd(&seed, 4) || !rd(&mu, 4) || !rd(fp, sizeof fp) || !rd(ip, sizeof ip)) return 2;
        const int n_vocab = h[0], n_ctx = h[1];
        std::vector<int32_t> order(h[2]), ctx(h[3]), last(h[4]), rs(h[5]);
        std::vector<float> lg(n_vocab);
        if (!rd(order.data(), 4 * order.size()) || !rd(ctx.data(), 4 * ctx.size()) || !rd(last.data(), 4 * last.size()) ||
            !rd(rs.data(), 4 * rs.size()) || !rd(lg.data(), 4 * lg.size()))
            return 2;
        current_context_tokens.assign(ctx.begin(), ctx.end());
        last_n_tokens.assign(last.begin(), last.end());
        dry_sequence_breakers.clear();
        for (size_t i = 0; i + 1 < rs.size();) {
            const int head = rs[i], len = rs[i + 1];
            dry_sequence_breakers.emplace(head, std::vector<gpt_vocab::id>(rs.begin() + i + 2, rs.begin() + i + 2 + len));
            i += 2 + (size_t)len;
        }
        logit_biases.clear();
        std::vector<samplers> so;
        for (int v : order) so.push_back((samplers)v);
        std::mt19937 rng(seed);
        const int tok = SampleLogits(lg.data(), n_ctx, n_vocab, ip[0], fp[7], fp[8], fp[9], fp[0], fp[1], fp[2], fp[3],
                                     fp[4], fp[5], fp[6], rng, ip[1], fp[10], fp[11], fp[12], fp[13], ip[2], ip[3], fp[14],
                                     fp[15], so, nullptr, fp[16], fp[17], fp[18]);
        printf("%d\n", tok);
        fflush(stdout);
    }
    return 0;
}
