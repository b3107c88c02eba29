// ref_vocab.cpp -- TEST INFRASTRUCTURE ONLY: drives the reference's own tokenizer (src/llama-vocab.cpp,
// src/unicode.cpp, src/unicode-data.cpp, compiled from /root/reference by oracle/Makefile `ref_vocab`) on a
// vocabulary given as a text file, so tests can pin the runtime tokenizer (koboldcpp_amd/csrc/tokenizer.h) to the
// reference's llama_tokenize_internal.  Never linked into the product.
//
// The vocabulary fields are set the way llm_load_vocab (src/llama.cpp:6200-6740) sets them from a GGUF: model
// type and pre-tokenizer flags (:6326-6466), token texts / scores / attributes (:6489-6520), byte-level merges
// (:6240-6260), the special-token cache sorted by text length (:6716-6733).  llama.cpp itself (the model loader) is
// not compiled, so this file also defines llama_log_internal as a log sink.
//
// usage: ref_vocab VOCAB TEXTS OUT
//   VOCAB: "bpe <pre-name>" | "spm"; then n; n lines "<hex text> <score> <type>" (GGUF token_type: 1 normal,
//          2 unknown, 3 control, 4 user-defined, 6 byte); then m; m lines "<hex left> <hex right>" (BPE merges);
//          then "bos eos unk add_bos" ids
//   TEXTS: n; n lines of hex text;  OUT: one line of token ids per text (add_special false, parse_special true),
//   then one line per vocabulary id: its piece (llama_token_to_piece_impl, special = false) in hex, "-" if empty
#include "llama-vocab.h"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>

void llama_log_internal(ggml_log_level, const char *, ...) {}

static std::string unhex(const std::string &h) {
    if (h == "-") return "";
    std::string s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s.push_back((char)std::stoi(h.substr(i, 2), nullptr, 16));
    return s;
}

// src/llama.cpp:6338-6441: pre-tokenizer name -> type and the flags that go with it
static void set_pre(llama_vocab &v, const std::string &p) {
    v.tokenizer_add_space_prefix = false;
    v.tokenizer_clean_spaces = true;
    if (p == "default") v.type_pre = LLAMA_VOCAB_PRE_TYPE_DEFAULT;
    else if (p == "llama3" || p == "llama-v3" || p == "llama-bpe") {
        v.type_pre = LLAMA_VOCAB_PRE_TYPE_LLAMA3; v.tokenizer_ignore_merges = true; v.tokenizer_add_bos = true;
    } else if (p == "deepseek-llm") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_DEEPSEEK_LLM; v.tokenizer_clean_spaces = false; }
    else if (p == "deepseek-coder") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_DEEPSEEK_CODER; v.tokenizer_clean_spaces = false; }
    else if (p == "falcon") v.type_pre = LLAMA_VOCAB_PRE_TYPE_FALCON;
    else if (p == "mpt") v.type_pre = LLAMA_VOCAB_PRE_TYPE_MPT;
    else if (p == "starcoder") v.type_pre = LLAMA_VOCAB_PRE_TYPE_STARCODER;
    else if (p == "gpt-2" || p == "phi-2" || p.rfind("jina-", 0) == 0) v.type_pre = LLAMA_VOCAB_PRE_TYPE_GPT2;
    else if (p == "refact") v.type_pre = LLAMA_VOCAB_PRE_TYPE_REFACT;
    else if (p == "command-r") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_COMMAND_R; v.tokenizer_clean_spaces = false; }
    else if (p == "qwen2") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_QWEN2; v.tokenizer_clean_spaces = false; }
    else if (p == "stablelm2") v.type_pre = LLAMA_VOCAB_PRE_TYPE_STABLELM2;
    else if (p == "olmo") v.type_pre = LLAMA_VOCAB_PRE_TYPE_OLMO;
    else if (p == "dbrx") v.type_pre = LLAMA_VOCAB_PRE_TYPE_DBRX;
    else if (p == "smaug-bpe") v.type_pre = LLAMA_VOCAB_PRE_TYPE_SMAUG;
    else if (p == "poro-chat") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_PORO; v.tokenizer_clean_spaces = false; }
    else if (p == "chatglm-bpe") v.type_pre = LLAMA_VOCAB_PRE_TYPE_CHATGLM4;
    else if (p == "viking") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_VIKING; v.tokenizer_clean_spaces = false; }
    else if (p == "jais") v.type_pre = LLAMA_VOCAB_PRE_TYPE_JAIS;
    else if (p == "tekken") {
        v.type_pre = LLAMA_VOCAB_PRE_TYPE_TEKKEN; v.tokenizer_clean_spaces = false; v.tokenizer_ignore_merges = true;
        v.tokenizer_add_bos = true;
    } else if (p == "smollm") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_SMOLLM; v.tokenizer_clean_spaces = false; }
    else if (p == "codeshell") v.type_pre = LLAMA_VOCAB_PRE_TYPE_CODESHELL;
    else if (p == "bloom") v.type_pre = LLAMA_VOCAB_PRE_TYPE_BLOOM;
    else if (p == "gpt3-finnish") v.type_pre = LLAMA_VOCAB_PRE_TYPE_GPT3_FINNISH;
    else if (p == "exaone") v.type_pre = LLAMA_VOCAB_PRE_TYPE_EXAONE;
    else if (p == "chameleon") { v.type_pre = LLAMA_VOCAB_PRE_TYPE_CHAMELEON; v.tokenizer_add_bos = true; v.tokenizer_clean_spaces = false; }
    else throw std::runtime_error("unknown pre-tokenizer " + p);
}

int main(int argc, char **argv) {
    if (argc != 4) { fprintf(stderr, "usage: ref_vocab VOCAB TEXTS OUT\n"); return 2; }
    std::ifstream fv(argv[1]);
    llama_vocab v;
    std::string kind;
    fv >> kind;
    if (kind == "bpe") {
        std::string pre;
        fv >> pre;
        v.type = LLAMA_VOCAB_TYPE_BPE;
        set_pre(v, pre);
    } else {
        v.type = LLAMA_VOCAB_TYPE_SPM;                     // :6442-6447
        v.type_pre = LLAMA_VOCAB_PRE_TYPE_DEFAULT;
        v.tokenizer_add_space_prefix = true;
        v.tokenizer_clean_spaces = false;
        v.tokenizer_add_bos = true;
    }
    size_t n;
    fv >> n;
    v.n_vocab = (uint32_t)n;
    v.id_to_token.resize(n);
    for (size_t i = 0; i < n; ++i) {
        std::string h;
        float score;
        int tt;
        fv >> h >> score >> tt;
        auto &td = v.id_to_token[i];
        td.text = unhex(h);
        td.score = score;
        // llama_token_type -> attribute (src/llama.cpp:6506-6516)
        td.attr = tt == 1 ? LLAMA_TOKEN_ATTR_NORMAL : tt == 2 ? LLAMA_TOKEN_ATTR_UNKNOWN : tt == 3 ? LLAMA_TOKEN_ATTR_CONTROL
                : tt == 4 ? LLAMA_TOKEN_ATTR_USER_DEFINED : tt == 6 ? LLAMA_TOKEN_ATTR_BYTE : LLAMA_TOKEN_ATTR_UNDEFINED;
        v.token_to_id[td.text] = (llama_token)i;
        v.max_token_len = std::max(v.max_token_len, (int)td.text.size());
    }
    size_t m;
    fv >> m;
    for (size_t i = 0; i < m; ++i) {
        std::string a, b;
        fv >> a >> b;
        v.bpe_ranks.emplace(std::make_pair(unhex(a), unhex(b)), (int)i);
    }
    int bos, eos, unk, add_bos;
    fv >> bos >> eos >> unk >> add_bos;
    v.special_bos_id = bos; v.special_eos_id = eos; v.special_unk_id = unk;
    if (add_bos >= 0) v.tokenizer_add_bos = add_bos != 0;
    if (v.type == LLAMA_VOCAB_TYPE_SPM) {
        // linefeed: the <0x0A> byte token (:6582-6588)
        auto it = v.token_to_id.find("<0x0A>");
        v.linefeed_id = it != v.token_to_id.end() ? it->second : unk;
    }
    // special-token cache: control / user-defined / unknown tokens, longest text first (:6716-6733)
    for (size_t i = 0; i < n; ++i)
        if (v.id_to_token[i].attr & (LLAMA_TOKEN_ATTR_CONTROL | LLAMA_TOKEN_ATTR_USER_DEFINED | LLAMA_TOKEN_ATTR_UNKNOWN))
            v.cache_special_tokens.push_back((llama_token)i);
    std::sort(v.cache_special_tokens.begin(), v.cache_special_tokens.end(), [&](llama_token a, llama_token b) {
        return v.id_to_token[a].text.size() > v.id_to_token[b].text.size();
    });
    v.init_tokenizer();
    std::ifstream ft(argv[2]);
    std::ofstream fo(argv[3]);
    size_t nt;
    ft >> nt;
    for (size_t i = 0; i < nt; ++i) {
        std::string h;
        ft >> h;
        const auto ids = llama_tokenize_internal(v, unhex(h), false, true);
        for (size_t k = 0; k < ids.size(); ++k) fo << (k ? " " : "") << ids[k];
        fo << "\n";
    }
    // then every token's piece as koboldcpp streams it (llama_token_to_piece_impl, special = false), in hex
    static const char hx[] = "0123456789abcdef";
    for (size_t i = 0; i < n; ++i) {
        char buf[1024];
        const int32_t len = llama_token_to_piece_impl(v, (llama_token)i, buf, sizeof buf, 0, false);
        std::string h;
        for (int32_t k = 0; k < len; ++k) { h += hx[(unsigned char)buf[k] >> 4]; h += hx[(unsigned char)buf[k] & 15]; }
        fo << (h.empty() ? "-" : h) << "\n";
    }
    return 0;
}
