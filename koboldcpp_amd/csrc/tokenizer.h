// tokenizer.h -- GGUF-vocabulary tokenizers for the drop-in generate() path.
//   "llama" (SentencePiece BPE, llm_tokenizer_spm semantics, src/llama-vocab.cpp): "▁" for spaces, optional
//     space prefix, greedy highest-score bigram merges over UTF-8 characters, <0xXX> byte fallback.
//   "gpt2" (byte-level BPE): GPT-2 byte->unicode map, merges by rank (whole pre-token words found in the
//     vocabulary taken as is for the llama3 / tekken pre-tokenizers: tokenizer_ignore_merges, src/llama-vocab.cpp:777).
//     The pre-tokenizer of every type llm_load_vocab accepts (src/llama.cpp:6338-6441) is its list of split passes
//     (llm_tokenizer_bpe's regex_exprs, src/llama-vocab.cpp:597-712), applied in order, each splitting every current
//     piece into its matches and the text between them (unicode_regex_split, src/unicode.cpp:663-830):
//       - the passes the reference runs with hand-written matchers are restated on code points with the Unicode
//         classes of unicode_ranges.h: llama3 (unicode_regex_split_custom_llama3, :355-492), gpt2
//         (unicode_regex_split_custom_gpt2, :248-352), and qwen2's expression (llama3's with single digits);
//       - every other pass runs on the C++ <regex> engines as the reference does: expressions that use \p{L} /
//         \p{N} / \p{P} on a "collapsed" text (ASCII kept, other code points replaced by one byte per class:
//         whitespace 0x0B, number 0xD1, letter 0xD2, punctuation 0xD3, anything else 0xD0) with each class
//         rewritten as a bracket of its byte and its ASCII members; the others on the code points as wchar_t with
//         non-ASCII whitespace replaced by 0x0B.
//     Pinned to the reference tokenizer itself (oracle/_ref/ref_vocab, tests/test_tokenizer_ref.py).  Invalid UTF-8
//     bytes become U+FFFD (the reference throws).
// Special tokens (token types UNKNOWN / CONTROL / USER_DEFINED) are split out of the text first, longest first,
// as tokenizer_st_partition with parse_special (src/llama-vocab.cpp:1544; koboldcpp's common_tokenize(..., true)).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <queue>
#include <regex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gguf.h"
#include "unicode_ranges.h"

#include <algorithm>
#include <cstring>

// deepseek-llm's letter and punctuation classes (src/llama-vocab.cpp:613-614), as universal character names
static const char *const kDeepseekLetters =
    "\\s?[A-Za-z\u00b5\u00c0-\u00d6\u00d8-\u00f6\u00f8-\u01ba\u01bc-\u01bf\u01c4-\u0293\u0295-\u02af\u0370-\u0373\u0376\u0377\u037b-\u037d\u037f\u0386\u0388-\u038a\u038c\u038e-\u03a1\u03a3-\u03f5\u03f7-\u0481\u048a-\u052f\u0531-\u0556\u10a0-\u10c5\u13a0-\u13f5\u13f8-\u13fd\u1c90-\u1cba\u1cbd-\u1cbf\u1d00-\u1d2b\u1d6b-\u1d77\u1d79-\u1d9a\u1e00-\u1f15\u1f18-\u1f1d\u1f20-\u1f45\u1f48-\u1f4d\u1f50-\u1f57\u1f59\u1f5b\u1f5d\u1f5f-\u1f7d\u1f80-\u1fb4\u1fb6-\u1fbc\u1fbe\u1fc2-\u1fc4\u1fc6-\u1fcc\u1fd0-\u1fd3\u1fd6-\u1fdb\u1fe0-\u1fec\u1ff2-\u1ff4\u1ff6-\u1ffc\u2102\u2107\u210a-\u2113\u2115\u2119-\u211d\u2124\u2126\u2128\u212a-\u212d\u212f-\u2134\u2139\u213c-\u213f\u2145-\u2149\u214e\u2183\u2184\u2c00-\u2c7b\u2c7e-\u2ce4\u2ceb-\u2cee\u2cf2\u2cf3\ua640-\ua66d\ua680-\ua69b\ua722-\ua76f\ua771-\ua787\ua78b-\ua78e\uab70-\uabbf\ufb00-\ufb06\ufb13-\ufb17\uff21-\uff3a\uff41-\uff5a\U00010400-\U0001044f\U000104b0-\U000104d3\U000104d8-\U000104fb\U00010c80-\U00010cb2\U00010cc0-\U00010cf2\U000118a0-\U000118df\U0001e900-\U0001e943]+";
static const char *const kDeepseekPunct = "\\s?[!-/:-~\uff01-\uff0f\uff1a-\uff5e\u2018-\u201f\u3000-\u3002]+";

class Tokenizer {
public:
    bool init(const gguf::File &f, std::string &err) {
        model_ = f.get_s("tokenizer.ggml.model", "llama");
        const gguf::Value *toks = f.get("tokenizer.ggml.tokens");
        if (!toks || toks->astr.empty()) { err = "GGUF has no tokenizer.ggml.tokens"; return false; }
        vocab_ = toks->astr;
        for (size_t i = 0; i < vocab_.size(); ++i) id_.emplace(vocab_[i], (int)i);
        if (const gguf::Value *sc = f.get("tokenizer.ggml.scores")) scores_.assign(sc->anum.begin(), sc->anum.end());
        scores_.resize(vocab_.size(), 0.0f);
        if (const gguf::Value *tt = f.get("tokenizer.ggml.token_type")) ttype_.assign(tt->anum.begin(), tt->anum.end());
        ttype_.resize(vocab_.size(), 1);
        bos_ = (int)f.get_i("tokenizer.ggml.bos_token_id", 1);
        eos_ = (int)f.get_i("tokenizer.ggml.eos_token_id", 2);
        add_bos_ = f.get_i("tokenizer.ggml.add_bos_token", 1) != 0;
        add_space_prefix_ = f.get_i("tokenizer.ggml.add_space_prefix", model_ == "llama" ? 1 : 0) != 0;
        if (model_ == "gpt2") {
            const gguf::Value *m = f.get("tokenizer.ggml.merges");
            if (!m) { err = "BPE vocab without merges"; return false; }
            for (size_t i = 0; i < m->astr.size(); ++i) rank_.emplace(m->astr[i], (int)i);
            build_byte_map();
            const std::string pre = f.get_s("tokenizer.ggml.pre", "default");
            pre_ = pre_type(pre);
            passes_ = make_passes(pre);
            ignore_merges_ = pre_ == PRE_LLAMA3 || pre == "tekken";
        } else if (model_ != "llama") {
            err = "unsupported tokenizer model " + model_;
            return false;
        }
        // EOT (llm_load_vocab, src/llama.cpp:6606, 6642-6661): tokenizer.ggml.eot_token_id, else the first token whose
        // text is one of the known end-of-turn markers (the reference walks an unordered_map; here the lowest id wins)
        eot_ = (int)f.get_i("tokenizer.ggml.eot_token_id", -1);
        if (eot_ < 0 || eot_ >= (int)vocab_.size()) {
            eot_ = -1;
            static const char *marks[] = {"<|eot_id|>", "<|im_end|>", "<|end|>", "<end_of_turn>", "<|endoftext|>", "<EOT>"};
            for (size_t i = 0; i < vocab_.size() && eot_ < 0; ++i)
                for (const char *mk : marks)
                    if (vocab_[i] == mk) { eot_ = (int)i; break; }
        }
        for (size_t i = 0; i < vocab_.size(); ++i)     // cache_special_tokens (src/llama.cpp:6720-6733)
            if ((ttype_[i] == 2 || ttype_[i] == 3 || ttype_[i] == 4) && !vocab_[i].empty()) special_.push_back((int)i);
        std::stable_sort(special_.begin(), special_.end(),
                         [&](int a, int b) { return vocab_[a].size() > vocab_[b].size(); });
        return true;
    }
    enum Pre { PRE_LLAMA3 = 0, PRE_QWEN2 = 1, PRE_GPT2 = 2, PRE_STL = 3 };
    static Pre pre_type(const std::string &p) {
        if (p == "llama3" || p == "llama-v3" || p == "llama-bpe" || p == "dbrx" || p == "smaug-bpe" || p == "chatglm-bpe")
            return PRE_LLAMA3;
        if (p == "qwen2" || p == "stablelm2") return PRE_QWEN2;
        return PRE_GPT2;
    }
    // one split pass: a hand-written matcher (kind PRE_LLAMA3 / PRE_QWEN2 / PRE_GPT2) or a <regex> expression
    // (PRE_STL: `wide` = run on the code points, else on the collapsed text with the class-rewritten expression)
    struct Pass {
        Pre kind;
        bool wide = false;
        std::shared_ptr<std::regex> rx;
        std::shared_ptr<std::wregex> wrx;
    };
    static Pass custom(Pre k) { Pass p; p.kind = k; return p; }
    static Pass stl(const std::string &expr) {
        Pass p;
        p.kind = PRE_STL;
        const bool cats = expr.find("\\p{L}") != std::string::npos || expr.find("\\p{N}") != std::string::npos ||
                          expr.find("\\p{P}") != std::string::npos;
        if (cats) {
            p.rx = std::make_shared<std::regex>(collapse_expr(expr));
        } else {
            p.wide = true;
            std::vector<uint32_t> cp;
            std::vector<size_t> bend;
            decode_utf8(expr, cp, bend);
            p.wrx = std::make_shared<std::wregex>(std::wstring(cp.begin(), cp.end()));
        }
        return p;
    }
    // the pass lists of llm_tokenizer_bpe (src/llama-vocab.cpp:597-712) by GGUF pre name (src/llama.cpp:6338-6441);
    // the gpt2 / llama3 expressions are the reference's hand-matched ones
    static std::vector<Pass> make_passes(const std::string &p) {
        const Pass gpt2 = custom(PRE_GPT2);
        const std::string finnish = " ?[^(\\s|.,!?\u2026\u3002\uff0c\u3001\u0964\u06d4\u060c)]+";
        const std::string cjk = "[\u4e00-\u9fa5\u0800-\u4e00\uac00-\ud7ff]+";
        if (pre_type(p) == PRE_LLAMA3) return {custom(PRE_LLAMA3)};
        if (pre_type(p) == PRE_QWEN2) return {custom(PRE_QWEN2)};
        if (p == "gpt-2" || p == "phi-2" || p.rfind("jina-", 0) == 0 || p == "mpt" || p == "olmo" || p == "jais") return {gpt2};
        if (p == "deepseek-llm")
            return {stl("[\r\n]"), stl(kDeepseekLetters), stl(kDeepseekPunct), stl("\\s+$"),
                    stl(cjk), stl("\\p{N}+")};
        if (p == "deepseek-coder")
            return {stl("[\r\n]"), stl("\\s?\\p{L}+"), stl("\\s?\\p{P}+"), stl(cjk), stl("\\p{N}")};
        if (p == "falcon") return {stl("[\\p{P}\\$\\+<=>\\^~\\|`]+"), gpt2, stl("[0-9][0-9][0-9]")};
        if (p == "starcoder" || p == "refact" || p == "command-r" || p == "smollm" || p == "codeshell" || p == "exaone")
            return {stl("\\p{N}"), gpt2};
        if (p == "bloom" || p == "poro-chat" || p == "gpt3-finnish") return {stl(finnish)};
        if (p == "viking") return {stl(finnish), stl("\\p{N}")};
        if (p == "tekken")
            return {stl("[^\\r\\n\\p{L}\\p{N}]?((?=[\\p{L}])([^a-z]))*((?=[\\p{L}])([^A-Z]))+|[^\\r\\n\\p{L}\\p{N}]?"
                        "((?=[\\p{L}])([^a-z]))+((?=[\\p{L}])([^A-Z]))*|\\p{N}| ?[^\\s\\p{L}\\p{N}]+[\\r\\n/]*|\\s*[\\r\\n]+|"
                        "\\s+(?!\\S)|\\s+")};
        if (p == "chameleon")
            return {stl("<sentinel:[0-9]+>"), stl("(IMGIMG)((A|B|C|D|E|F|G|H|I){1,4})Z"), stl("([\\t\\n]|    |  )"),
                    stl("\\p{N}"), stl("[\\p{P}!-/:-@\\[-`{-~]"), gpt2};
        // "default" and any other name (the reference rejects unknown names; its default list)
        return {stl("[\\p{P}\\$\\+<=>\\^~\\|]+"), gpt2, stl("\\p{N}+"), stl("[0-9][0-9][0-9]")};
    }
    int bos() const { return bos_; }
    int eos() const { return eos_; }
    int eot() const { return eot_; }
    int n_vocab() const { return (int)vocab_.size(); }

    std::vector<int> encode(const std::string &text, bool add_bos) const {
        std::vector<int> out;
        if (add_bos && add_bos_) out.push_back(bos_);
        if (text.empty()) return out;
        // fragments: raw text (id -1, byte range) and special tokens, in order
        struct Frag { int id; size_t off, len; };
        std::vector<Frag> fr{{-1, 0, text.size()}};
        for (int sid : special_) {
            const std::string &st = vocab_[sid];
            std::vector<Frag> nx;
            for (const Frag &g : fr) {
                if (g.id >= 0) { nx.push_back(g); continue; }
                size_t pos = g.off;
                const size_t end = g.off + g.len;
                while (true) {
                    const size_t m = text.find(st, pos);
                    if (m == std::string::npos || m + st.size() > end) break;
                    if (m > pos) nx.push_back({-1, pos, m - pos});
                    nx.push_back({sid, m, st.size()});
                    pos = m + st.size();
                }
                if (pos < end) nx.push_back({-1, pos, end - pos});
            }
            fr.swap(nx);
        }
        bool prev_special = true;                      // SPM: space prefix at the start and after a special token
        for (const Frag &g : fr) {
            if (g.id >= 0) { out.push_back(g.id); prev_special = true; continue; }
            const std::string raw = text.substr(g.off, g.len);
            if (model_ == "llama") spm(raw, out, add_space_prefix_ && prev_special);
            else bpe(raw, out);
            prev_special = false;
        }
        return out;
    }
    // pre-tokenizer alone (tests): byte end offsets of the words of `text`
    static std::vector<size_t> pretokenize_offsets(const std::string &pre, const std::string &text) {
        std::vector<uint32_t> cp;
        std::vector<size_t> bend;
        decode_utf8(text, cp, bend);
        std::vector<size_t> out;
        for (size_t e : split_passes(make_passes(pre), cp)) out.push_back(bend[e - 1]);
        return out;
    }
    // text of one token as generate() streams it: llama_token_to_piece_impl with special = false
    // (src/llama-vocab.cpp:2007-2077): unknown / control tokens render nothing, user-defined tokens their text,
    // normal tokens unescaped (SPM: U+2581 -> space) or byte-decoded (BPE, llama_decode_text :1986-2004: a code
    // point outside the byte map renders as "[UNK_BYTE_0x<its utf8>" + token text + "]"), SPM byte tokens their
    // byte, every other type (undefined, unused, BPE byte) nothing
    // llama_token_to_piece_impl (src/llama-vocab.cpp:2007-2077): special = false suppresses UNKNOWN / CONTROL tokens,
    // special = true renders their raw text (koboldcpp's render_special)
    std::string piece(int id, bool special = false) const {
        if (id < 0 || id >= (int)vocab_.size()) return "";
        const int type = ttype_[id];
        const std::string &s = vocab_[id];
        if (type == 2 || type == 3) return special ? s : "";
        if (type == 4) return s;
        if (model_ == "llama") {
            if (type == 6) return s.size() >= 5 ? std::string(1, (char)strtol(s.substr(3, 2).c_str(), nullptr, 16)) : "";
            if (type != 1) return "";
            std::string r;
            for (size_t i = 0; i < s.size();) {
                if (s.compare(i, 3, "\xe2\x96\x81") == 0) { r += ' '; i += 3; }
                else r += s[i++];
            }
            return r;
        }
        if (type != 1) return "";
        std::string r;                                  // gpt2: unicode code points -> bytes
        for (size_t i = 0; i < s.size();) {
            uint32_t cp; int n = utf8_dec(s, i, cp);
            auto it = u2b_.find(cp);
            if (it != u2b_.end()) r += (char)it->second;
            else {
                static const char hx[] = "0123456789abcdef";
                r += "[UNK_BYTE_0x";
                for (int k = 0; k < n; ++k) { r += hx[(unsigned char)s[i + k] >> 4]; r += hx[(unsigned char)s[i + k] & 15]; }
                r += s + "]";
            }
            i += n;
        }
        return r;
    }

private:
    static int utf8_len(unsigned char c) { return c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1; }
    static int utf8_dec(const std::string &s, size_t i, uint32_t &cp) {
        const unsigned char c = (unsigned char)s[i];
        int n = utf8_len(c);
        if (i + n > s.size()) n = 1;
        if (n == 1) { cp = c; return 1; }
        cp = c & (0xFF >> (n + 1));
        for (int k = 1; k < n; ++k) cp = (cp << 6) | ((unsigned char)s[i + k] & 0x3F);
        return n;
    }
    static std::string utf8_enc(uint32_t cp) {
        std::string r;
        if (cp < 0x80) r += (char)cp;
        else if (cp < 0x800) { r += (char)(0xC0 | (cp >> 6)); r += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) { r += (char)(0xE0 | (cp >> 12)); r += (char)(0x80 | ((cp >> 6) & 0x3F)); r += (char)(0x80 | (cp & 0x3F)); }
        else { r += (char)(0xF0 | (cp >> 18)); r += (char)(0x80 | ((cp >> 12) & 0x3F)); r += (char)(0x80 | ((cp >> 6) & 0x3F)); r += (char)(0x80 | (cp & 0x3F)); }
        return r;
    }
    int find(const std::string &s) const { auto it = id_.find(s); return it == id_.end() ? -1 : it->second; }

    // ---- SentencePiece: highest-score adjacent merges (ties: leftmost)
    void spm(const std::string &text, std::vector<int> &out, bool space_prefix) const {
        std::string t = space_prefix ? " " + text : text;
        std::string n;
        for (char c : t) { if (c == ' ') n += "\xe2\x96\x81"; else n += c; }
        struct Sym { int prev, next; size_t off, len; };
        std::vector<Sym> sy;
        for (size_t i = 0; i < n.size();) {
            const int l = std::min<int>(utf8_len((unsigned char)n[i]), (int)(n.size() - i));
            sy.push_back({(int)sy.size() - 1, (int)sy.size() + 1, i, (size_t)l});
            i += l;
        }
        if (!sy.empty()) sy.back().next = -1;
        struct Big { float score; int left; size_t size; };
        auto cmp = [](const Big &a, const Big &b) { return a.score < b.score || (a.score == b.score && a.left > b.left); };
        std::priority_queue<Big, std::vector<Big>, decltype(cmp)> q(cmp);
        auto try_add = [&](int l, int r) {
            if (l < 0 || r < 0) return;
            const int id = find(n.substr(sy[l].off, sy[l].len + sy[r].len));
            if (id >= 0) q.push({scores_[id], l, sy[l].len + sy[r].len});
        };
        for (int i = 1; i < (int)sy.size(); ++i) try_add(i - 1, i);
        while (!q.empty()) {
            const Big b = q.top(); q.pop();
            Sym &l = sy[b.left];
            if (l.len == 0 || l.next < 0) continue;
            Sym &r = sy[l.next];
            if (l.len + r.len != b.size) continue;      // stale entry
            l.len += r.len;
            r.len = 0;
            l.next = r.next;
            if (r.next >= 0) sy[r.next].prev = b.left;
            try_add(l.prev, b.left);
            try_add(b.left, l.next);
        }
        for (int i = 0; i != -1 && i < (int)sy.size(); i = sy[i].next) {
            if (sy[i].len == 0) continue;
            const std::string s = n.substr(sy[i].off, sy[i].len);
            const int id = find(s);
            if (id >= 0) { out.push_back(id); continue; }
            for (unsigned char c : s) {                 // byte fallback
                char buf[8];
                snprintf(buf, sizeof buf, "<0x%02X>", c);
                const int bid = find(buf);
                if (bid >= 0) out.push_back(bid);
            }
        }
    }

    // ---- byte-level BPE
    void build_byte_map() {
        std::vector<int> bs;
        for (int b = 33; b <= 126; ++b) bs.push_back(b);
        for (int b = 161; b <= 172; ++b) bs.push_back(b);
        for (int b = 174; b <= 255; ++b) bs.push_back(b);
        std::vector<bool> has(256, false);
        for (int b : bs) has[b] = true;
        int extra = 0;
        for (int b = 0; b < 256; ++b) {
            const uint32_t cp = has[b] ? (uint32_t)b : (uint32_t)(256 + extra++);
            b2u_[b] = utf8_enc(cp);
            u2b_[cp] = b;
        }
    }
    // the collapsed form of an expression (src/unicode.cpp:757-795): \p{N} / \p{L} / \p{P} become a bracket of the
    // class byte and its ASCII members (inside an existing bracket: just those members)
    static std::string collapse_expr(const std::string &e) {
        static const char *members[3] = {"\xD1\x30-\x39", "\xD2\x41-\x5A\x61-\x7A",
                                         "\xD3\x21-\x23\x25-\x2A\x2C-\x2F\x3A-\x3B\x3F-\x40\\\x5B-\\\x5D\x5F\\\x7B\\\x7D"};
        std::string out;
        bool inside = false;
        for (size_t i = 0; i < e.size(); ++i) {
            if (e[i] == '[' && (i == 0 || e[i - 1] != '\\')) { out += '['; inside = true; continue; }
            if (inside && e[i] == ']' && e[i - 1] != '\\') { out += ']'; inside = false; continue; }
            if (e[i] == '\\' && i + 4 < e.size() && e[i + 1] == 'p' && e[i + 2] == '{' && e[i + 4] == '}') {
                const int k = e[i + 3] == 'N' ? 0 : e[i + 3] == 'L' ? 1 : e[i + 3] == 'P' ? 2 : -1;
                if (k >= 0) {
                    if (!inside) out += '[';
                    out += members[k];
                    if (!inside) out += ']';
                    i += 4;
                    continue;
                }
            }
            out += e[i];
        }
        return out;
    }
    // one byte per code point (src/unicode.cpp:697-723): ASCII as is; else whitespace 0x0B, N 0xD1, L 0xD2, P 0xD3,
    // anything else 0xD0
    static std::string collapse_text(const std::vector<uint32_t> &cp) {
        std::string t(cp.size(), '\0');
        for (size_t i = 0; i < cp.size(); ++i) {
            const uint32_t c = cp[i];
            if (c < 0x80) { t[i] = (char)c; continue; }
            const uint8_t f = cls(c);
            t[i] = (char)((f & 4) ? 0x0B : (f & 2) ? 0xD1 : (f & 1) ? 0xD2 : (f & 8) ? 0xD3 : 0xD0);
        }
        return t;
    }
    // word end positions (code point indices) after every pass; a pass splits each current piece into its matches
    // and the text between them (unicode_regex_split_stl, src/unicode.cpp:496-553)
    static std::vector<size_t> split_passes(const std::vector<Pass> &passes, const std::vector<uint32_t> &cp) {
        std::vector<size_t> ends{cp.size()};
        if (cp.empty()) return {};
        std::string coll;
        std::wstring wt;
        for (const Pass &ps : passes) {
            std::vector<size_t> nx;
            size_t b = 0;
            for (size_t e : ends) {
                if (ps.kind != PRE_STL) {
                    const std::vector<uint32_t> sub(cp.begin() + b, cp.begin() + e);
                    for (size_t w : split_words(ps.kind, sub)) nx.push_back(b + w);
                } else {
                    size_t last = b;
                    auto add = [&](size_t pos, size_t len) {
                        if (pos > last) nx.push_back(pos);
                        nx.push_back(pos + len);
                        last = pos + len;
                    };
                    if (ps.wide) {
                        if (wt.empty()) {
                            wt.assign(cp.begin(), cp.end());
                            for (auto &c : wt)
                                if ((uint32_t)c > 0x7F && (cls((uint32_t)c) & 4)) c = 0x0B;
                        }
                        for (std::wcregex_iterator it(wt.data() + b, wt.data() + e, *ps.wrx), end; it != end; ++it)
                            add(b + (size_t)it->position(), (size_t)it->length());
                    } else {
                        if (coll.empty()) coll = collapse_text(cp);
                        for (std::cregex_iterator it(coll.data() + b, coll.data() + e, *ps.rx), end; it != end; ++it)
                            add(b + (size_t)it->position(), (size_t)it->length());
                    }
                    if (last < e) nx.push_back(e);
                }
                b = e;
            }
            // empty matches leave zero-length pieces; the reference's BPE skips nothing for them either way
            std::vector<size_t> clean;
            size_t prev = 0;
            for (size_t e : nx)
                if (e > prev) { clean.push_back(e); prev = e; }
            ends.swap(clean);
        }
        return ends;
    }
    // ---- pre-tokenizers over code points
    static uint8_t cls(uint32_t c) {                   // 1 = \p{L}, 2 = \p{N}, 4 = \s
        if (c < 0x80) {
            if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') return 1;
            if (c >= '0' && c <= '9') return 2;
            return (c == ' ' || (c >= 9 && c <= 13)) ? 4 : 0;
        }
        int lo = 0, hi = ucd::kNumRanges - 1;
        while (lo <= hi) {
            const int mid = (lo + hi) / 2;
            if (c < ucd::kRanges[mid].lo) hi = mid - 1;
            else if (c > ucd::kRanges[mid].hi) lo = mid + 1;
            else return ucd::kRanges[mid].f;
        }
        return 0;
    }
    // code points and each one's byte end offset; an invalid or truncated sequence is one U+FFFD per byte
    static void decode_utf8(const std::string &s, std::vector<uint32_t> &cp, std::vector<size_t> &bend) {
        for (size_t i = 0; i < s.size();) {
            const unsigned char c = (unsigned char)s[i];
            int n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
            bool ok = n > 0 && i + n <= s.size();
            for (int k = 1; ok && k < n; ++k) ok = ((unsigned char)s[i + k] >> 6) == 2;
            if (!ok) { cp.push_back(0xFFFD); i += 1; bend.push_back(i); continue; }
            uint32_t v = n == 1 ? c : c & (0xFF >> (n + 1));
            for (int k = 1; k < n; ++k) v = (v << 6) | ((unsigned char)s[i + k] & 0x3F);
            cp.push_back(v);
            i += n;
            bend.push_back(i);
        }
    }
    static uint32_t lower_ascii(uint32_t c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }
    // word end positions (code point indices) -- llama3 / qwen2: unicode_regex_split_custom_llama3 semantics,
    // gpt2: unicode_regex_split_custom_gpt2 (src/unicode.cpp)
    static std::vector<size_t> split_words(Pre pre, const std::vector<uint32_t> &cp) {
        std::vector<size_t> ends;
        const size_t n = cp.size();
        auto F = [&](size_t k) -> int { return k < n ? cls(cp[k]) : -1; };   // -1: past the end (no flags)
        auto NL = [&](size_t k) { return k < n && (cp[k] == '\r' || cp[k] == '\n'); };
        size_t pos = 0;
        auto emit = [&](size_t e) { if (e > pos) ends.push_back(e); pos = e; };
        while (pos < n) {
            const uint32_t c = cp[pos];
            const int f = F(pos);
            if (c == '\'' && pos + 1 < n) {                // contractions (case-insensitive for llama3 / qwen2)
                const uint32_t c1 = pre == PRE_GPT2 ? cp[pos + 1] : lower_ascii(cp[pos + 1]);
                if (c1 == 's' || c1 == 't' || c1 == 'm' || c1 == 'd') { emit(pos + 2); continue; }
                if (pos + 2 < n) {
                    const uint32_t c2 = pre == PRE_GPT2 ? cp[pos + 2] : lower_ascii(cp[pos + 2]);
                    if ((c1 == 'r' && c2 == 'e') || (c1 == 'v' && c2 == 'e') || (c1 == 'l' && c2 == 'l')) { emit(pos + 3); continue; }
                }
            }
            if (pre == PRE_GPT2) {
                const int f2 = c == ' ' ? F(pos + 1) : f;
                if (f2 > 0 && (f2 & 1)) {                   //  ?\p{L}+
                    size_t e = pos + (c == ' ');
                    while (F(e) > 0 && (F(e) & 1)) ++e;
                    emit(e); continue;
                }
                if (f2 > 0 && (f2 & 2)) {                   //  ?\p{N}+
                    size_t e = pos + (c == ' ');
                    while (F(e) > 0 && (F(e) & 2)) ++e;
                    emit(e); continue;
                }
                if (f2 >= 0 && !(f2 & 7)) {                 //  ?[^\s\p{L}\p{N}]+
                    size_t e = pos + (c == ' ');
                    while (F(e) >= 0 && !(F(e) & 7)) ++e;
                    emit(e); continue;
                }
            } else {
                if (!(c == '\r' || c == '\n' || (f & 2))) {  // [^\r\n\p{L}\p{N}]?\p{L}+
                    if ((f & 1) || (F(pos + 1) > 0 && (F(pos + 1) & 1))) {
                        size_t e = pos + 1;
                        while (F(e) > 0 && (F(e) & 1)) ++e;
                        emit(e); continue;
                    }
                }
                if (f & 2) {                                // \p{N}{1,3} (qwen2: \p{N})
                    const size_t maxr = pre == PRE_QWEN2 ? 1 : 3;
                    size_t e = pos;
                    while (F(e) > 0 && (F(e) & 2) && e - pos < maxr) ++e;
                    emit(e); continue;
                }
                const int f2 = c == ' ' ? F(pos + 1) : f;   //  ?[^\s\p{L}\p{N}]+[\r\n]*
                if (f2 >= 0 && !(f2 & 7)) {
                    size_t e = pos + (c == ' ');
                    while (F(e) >= 0 && !(F(e) & 7)) ++e;
                    while (NL(e)) ++e;
                    emit(e); continue;
                }
            }
            size_t nws = 0, last_nl = 0;
            while (F(pos + nws) > 0 && (F(pos + nws) & 4)) {
                if (NL(pos + nws)) last_nl = pos + nws + 1;
                ++nws;
            }
            if (pre != PRE_GPT2 && last_nl > 0) { emit(last_nl); continue; }   // \s*[\r\n]+
            if (nws > 1 && pos + nws < n) { emit(pos + nws - 1); continue; }   // \s+(?!\S)
            if (nws > 0) { emit(pos + nws); continue; }                       // \s+
            emit(pos + 1);                                                    // no match
        }
        return ends;
    }
    void bpe(const std::string &text, std::vector<int> &out) const {
        std::vector<uint32_t> cp;
        std::vector<size_t> bend;
        decode_utf8(text, cp, bend);
        size_t w0 = 0;
        for (size_t e : split_passes(passes_, cp)) {
            std::string word;                           // the word's code points re-encoded (U+FFFD for bad bytes)
            for (size_t k = w0; k < e; ++k) word += utf8_enc(cp[k]);
            w0 = e;
            std::vector<std::string> parts;
            for (unsigned char c : word) parts.push_back(b2u_[c]);
            if (ignore_merges_) {
                std::string whole;
                for (const std::string &p : parts) whole += p;
                const int id = find(whole);
                if (id >= 0) { out.push_back(id); continue; }
            }
            while (parts.size() > 1) {
                int best = -1, br = INT32_MAX;
                for (size_t k = 0; k + 1 < parts.size(); ++k) {
                    auto it = rank_.find(parts[k] + " " + parts[k + 1]);
                    if (it != rank_.end() && it->second < br) { br = it->second; best = (int)k; }
                }
                if (best < 0) break;
                parts[best] += parts[best + 1];
                parts.erase(parts.begin() + best + 1);
            }
            for (const std::string &p : parts) {
                const int id = find(p);
                if (id >= 0) out.push_back(id);
            }
        }
    }

    std::string model_;
    Pre pre_ = PRE_LLAMA3;
    std::vector<Pass> passes_;
    bool ignore_merges_ = false;
    std::vector<int> special_;
    std::vector<std::string> vocab_;
    std::unordered_map<std::string, int> id_;
    std::vector<float> scores_;
    std::vector<int> ttype_;
    std::unordered_map<std::string, int> rank_;
    std::string b2u_[256];
    std::map<uint32_t, int> u2b_;
    int bos_ = 1, eos_ = 2, eot_ = -1;
    bool add_bos_ = true, add_space_prefix_ = true;
};
