// tokenizer.h -- GGUF-vocabulary tokenizers for the drop-in generate() path.
//   "llama" (SentencePiece BPE, llm_tokenizer_spm semantics, src/llama-vocab.cpp): "▁" for spaces, optional
//     space prefix, greedy highest-score bigram merges over UTF-8 characters, <0xXX> byte fallback.
//   "gpt2" (byte-level BPE, Llama-3): GPT-2 byte->unicode map, merges by rank; the pre-tokenizer follows the
//     Llama-3 split regex with ASCII character classes (bytes >= 0x80 count as letters) -- exact for ASCII
//     text, an approximation of \p{L}/\p{N} beyond it.
#pragma once
#include <cstdint>
#include <map>
#include <queue>
#include <string>
#include <unordered_map>
#include <vector>

#include "gguf.h"

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
        } else if (model_ != "llama") {
            err = "unsupported tokenizer model " + model_;
            return false;
        }
        return true;
    }
    int bos() const { return bos_; }
    int eos() const { return eos_; }
    int n_vocab() const { return (int)vocab_.size(); }

    std::vector<int> encode(const std::string &text, bool add_bos) const {
        std::vector<int> out;
        if (add_bos && add_bos_) out.push_back(bos_);
        if (text.empty()) return out;
        if (model_ == "llama") spm(text, out);
        else bpe(text, out);
        return out;
    }
    std::string piece(int id) const {            // text of one token (for streaming)
        if (id < 0 || id >= (int)vocab_.size()) return "";
        const int type = ttype_[id];
        if (type == 3 || type == 4) return "";       // control / unused: not rendered
        const std::string &s = vocab_[id];
        if (model_ == "llama") {
            if (type == 6 && s.size() == 6 && s.compare(0, 3, "<0x") == 0)        // byte token
                return std::string(1, (char)strtol(s.substr(3, 2).c_str(), nullptr, 16));
            std::string r;
            for (size_t i = 0; i < s.size();) {
                if (s.compare(i, 3, "\xe2\x96\x81") == 0) { r += ' '; i += 3; }
                else r += s[i++];
            }
            return r;
        }
        std::string r;                                  // gpt2: unicode code points -> bytes
        for (size_t i = 0; i < s.size();) {
            uint32_t cp; int n = utf8_dec(s, i, cp);
            auto it = u2b_.find(cp);
            if (it != u2b_.end()) r += (char)it->second;
            else r += s.substr(i, n);
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
    void spm(const std::string &text, std::vector<int> &out) const {
        std::string t = add_space_prefix_ ? " " + text : text;
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
    static bool is_letter(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c >= 0x80; }
    static bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }
    static bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
    static bool is_nl(unsigned char c) { return c == '\n' || c == '\r'; }
    std::vector<std::string> pretokenize(const std::string &s) const {
        std::vector<std::string> w;
        size_t i = 0, n = s.size();
        auto lower = [](char c) { return (char)(c >= 'A' && c <= 'Z' ? c + 32 : c); };
        while (i < n) {
            const unsigned char c = (unsigned char)s[i];
            if (c == '\'' && i + 1 < n) {              // contractions
                static const char *cs[] = {"s", "t", "re", "ve", "m", "ll", "d"};
                bool hit = false;
                for (const char *x : cs) {
                    const size_t L = strlen(x);
                    if (i + 1 + L <= n) {
                        bool ok = true;
                        for (size_t k = 0; k < L; ++k) ok &= lower(s[i + 1 + k]) == x[k];
                        if (ok) { w.push_back(s.substr(i, 1 + L)); i += 1 + L; hit = true; break; }
                    }
                }
                if (hit) continue;
            }
            if (is_letter(c) || (!is_nl(c) && !is_digit(c) && !is_letter(c) && i + 1 < n && is_letter((unsigned char)s[i + 1]) && !is_space(c))
                || (c == ' ' && i + 1 < n && is_letter((unsigned char)s[i + 1]))) {
                size_t j = is_letter(c) ? i : i + 1;
                while (j < n && is_letter((unsigned char)s[j])) ++j;
                w.push_back(s.substr(i, j - i)); i = j; continue;
            }
            if (is_digit(c)) {
                size_t j = i;
                while (j < n && j < i + 3 && is_digit((unsigned char)s[j])) ++j;
                w.push_back(s.substr(i, j - i)); i = j; continue;
            }
            if (!is_space(c) || (c == ' ' && i + 1 < n && !is_space((unsigned char)s[i + 1]) && !is_letter((unsigned char)s[i + 1]) && !is_digit((unsigned char)s[i + 1]))) {
                size_t j = (c == ' ') ? i + 1 : i;
                while (j < n && !is_space((unsigned char)s[j]) && !is_letter((unsigned char)s[j]) && !is_digit((unsigned char)s[j])) ++j;
                while (j < n && is_nl((unsigned char)s[j])) ++j;
                w.push_back(s.substr(i, j - i)); i = j; continue;
            }
            size_t j = i;                               // whitespace
            while (j < n && is_space((unsigned char)s[j])) ++j;
            size_t last_nl = std::string::npos;
            for (size_t k = i; k < j; ++k) if (is_nl((unsigned char)s[k])) last_nl = k;
            if (last_nl != std::string::npos) { w.push_back(s.substr(i, last_nl + 1 - i)); i = last_nl + 1; continue; }
            if (j < n && j - i > 1) { w.push_back(s.substr(i, j - 1 - i)); i = j - 1; continue; }   // \s+(?!\S)
            w.push_back(s.substr(i, j - i)); i = j;
        }
        return w;
    }
    void bpe(const std::string &text, std::vector<int> &out) const {
        for (const std::string &word : pretokenize(text)) {
            std::vector<std::string> parts;
            for (unsigned char c : word) parts.push_back(b2u_[c]);
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
    std::vector<std::string> vocab_;
    std::unordered_map<std::string, int> id_;
    std::vector<float> scores_;
    std::vector<int> ttype_;
    std::unordered_map<std::string, int> rank_;
    std::string b2u_[256];
    std::map<uint32_t, int> u2b_;
    int bos_ = 1, eos_ = 2;
    bool add_bos_ = true, add_space_prefix_ = true;
};
