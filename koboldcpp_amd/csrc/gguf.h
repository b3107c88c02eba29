// gguf.h -- minimal read-only GGUF (v2/v3) reader: metadata key/values and tensor directory over an mmap.
// Format: magic "GGUF", u32 version, u64 n_tensors, u64 n_kv, KV pairs (gguf string key, u32 type, value),
// tensor infos (name, u32 n_dims, u64 dims[], u32 ggml type, u64 offset), then tensor data aligned to
// general.alignment (default 32).  Tensor data are used in place (ggml block layout).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <climits>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace gguf {

enum VType { U8 = 0, I8, U16, I16, U32, I32, F32, BOOL, STR, ARR, U64, I64, F64 };

struct Value {
    int type = -1;
    int64_t i = 0;
    double f = 0;
    std::string s;
    int arr_type = -1;
    std::vector<std::string> astr;     // string arrays (tokens, merges)
    std::vector<double> anum;          // numeric arrays (scores, token types)
};

struct Tensor {
    std::string name;
    int type = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    const uint8_t *data = nullptr;
    uint64_t offset = 0;
    uint64_t nbytes = 0;
};

// (block elements, block bytes) of every ggml type id (ggml.h:363-398, block structs ggml-common.h:144-419);
// {0, 0} for ids that do not exist
inline void type_block(int t, uint64_t &be, uint64_t &bb) {
    static const uint16_t tab[36][2] = {
        {1, 4}, {1, 2}, {32, 18}, {32, 20}, {0, 0}, {0, 0}, {32, 22}, {32, 24}, {32, 34}, {32, 36},
        {256, 84}, {256, 110}, {256, 144}, {256, 176}, {256, 210}, {256, 292}, {256, 66}, {256, 74}, {256, 98},
        {256, 50}, {32, 18}, {256, 110}, {256, 82}, {256, 136}, {1, 1}, {1, 2}, {1, 4}, {1, 8}, {1, 8}, {256, 56},
        {1, 2}, {32, 18}, {32, 18}, {32, 18}, {256, 54}, {256, 66}};
    be = bb = 0;
    if (t >= 0 && t < 36) { be = tab[t][0]; bb = tab[t][1]; }
}

class File {
public:
    ~File() { close(); }
    bool open(const std::string &path, std::string &err) {
        fd_ = ::open(path.c_str(), O_RDONLY);
        if (fd_ < 0) { err = "cannot open " + path; return false; }
        struct stat st;
        if (fstat(fd_, &st) != 0) { err = "stat failed"; return false; }
        size_ = (size_t)st.st_size;
        map_ = (const uint8_t *)mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
        if (map_ == MAP_FAILED) { map_ = nullptr; err = "mmap failed"; return false; }
        pos_ = 0;
        try {
            if (rd<uint32_t>() != 0x46554747u) { err = "not a GGUF file"; return false; }
            version = rd<uint32_t>();
            if (version < 2) { err = "GGUF v1 not supported"; return false; }
            const uint64_t nt = rd<uint64_t>(), nkv = rd<uint64_t>();
            for (uint64_t k = 0; k < nkv; ++k) {
                std::string key = rds();
                Value v;
                v.type = (int)rd<uint32_t>();
                read_value(v.type, v);
                kv[key] = std::move(v);
            }
            uint64_t align = 32;
            auto it = kv.find("general.alignment");
            if (it != kv.end()) align = (uint64_t)it->second.i;
            if (align == 0 || (align & (align - 1)) != 0) throw std::string("general.alignment must be a power of two");
            for (uint64_t t = 0; t < nt; ++t) {
                Tensor tt;
                tt.name = rds();
                const uint32_t nd = rd<uint32_t>();
                if (nd > 4) throw std::string("tensor rank > 4");
                for (uint32_t d = 0; d < nd; ++d) tt.ne[d] = (int64_t)rd<uint64_t>();
                tt.type = (int)rd<uint32_t>();
                tt.offset = rd<uint64_t>();
                // byte size with overflow checks (llama.cpp:4379-4390 checks offset + size against the file)
                uint64_t be, bb, nel = 1;
                type_block(tt.type, be, bb);
                if (!be) throw std::string("unknown tensor type in " + tt.name);
                for (int d = 0; d < 4; ++d) {
                    if (tt.ne[d] < 0) throw std::string("negative dimension in " + tt.name);
                    if (tt.ne[d] && nel > UINT64_MAX / (uint64_t)tt.ne[d]) throw std::string("tensor too large: " + tt.name);
                    nel *= (uint64_t)tt.ne[d];
                }
                if (tt.ne[0] % be) throw std::string("row not a whole number of blocks: " + tt.name);
                if (nel / be > UINT64_MAX / bb) throw std::string("tensor too large: " + tt.name);
                tt.nbytes = nel / be * bb;
                tensors.push_back(tt);
            }
            const uint64_t data0 = (pos_ + align - 1) / align * align;
            for (auto &tt : tensors) {
                if (tt.offset > size_ || data0 > size_ - tt.offset || tt.nbytes > size_ - data0 - tt.offset)
                    throw std::string("tensor data past end of file: " + tt.name);
                tt.data = map_ + data0 + tt.offset;
                by_name[tt.name] = &tt - &tensors[0];
            }
        } catch (const std::string &e) {
            err = "GGUF parse error: " + e;
            return false;
        }
        return true;
    }
    void close() {
        if (map_) munmap((void *)map_, size_);
        if (fd_ >= 0) ::close(fd_);
        map_ = nullptr; fd_ = -1;
    }
    const Tensor *tensor(const std::string &n) const {
        auto it = by_name.find(n);
        return it == by_name.end() ? nullptr : &tensors[it->second];
    }
    const Value *get(const std::string &k) const {
        auto it = kv.find(k);
        return it == kv.end() ? nullptr : &it->second;
    }
    int64_t get_i(const std::string &k, int64_t def) const { const Value *v = get(k); return v ? v->i : def; }
    double get_f(const std::string &k, double def) const { const Value *v = get(k); return v ? v->f : def; }
    std::string get_s(const std::string &k, const std::string &def) const { const Value *v = get(k); return v ? v->s : def; }
    size_t file_size() const { return size_; }

    uint32_t version = 0;
    std::map<std::string, Value> kv;
    std::vector<Tensor> tensors;
    std::map<std::string, size_t> by_name;

private:
    template <typename T> T rd() {
        if (sizeof(T) > size_ - pos_) throw std::string("truncated");
        T v;
        memcpy(&v, map_ + pos_, sizeof(T));
        pos_ += sizeof(T);
        return v;
    }
    std::string rds() {
        const uint64_t n = rd<uint64_t>();
        if (n > size_ - pos_) throw std::string("truncated string");
        std::string s((const char *)map_ + pos_, (size_t)n);
        pos_ += n;
        return s;
    }
    void read_scalar(int t, Value &v) {
        switch (t) {
        case U8: v.i = rd<uint8_t>(); v.f = (double)v.i; break;
        case I8: v.i = rd<int8_t>(); v.f = (double)v.i; break;
        case U16: v.i = rd<uint16_t>(); v.f = (double)v.i; break;
        case I16: v.i = rd<int16_t>(); v.f = (double)v.i; break;
        case U32: v.i = rd<uint32_t>(); v.f = (double)v.i; break;
        case I32: v.i = rd<int32_t>(); v.f = (double)v.i; break;
        case F32: v.f = rd<float>(); v.i = (int64_t)v.f; break;
        case BOOL: v.i = rd<uint8_t>(); v.f = (double)v.i; break;
        case U64: v.i = (int64_t)rd<uint64_t>(); v.f = (double)v.i; break;
        case I64: v.i = rd<int64_t>(); v.f = (double)v.i; break;
        case F64: v.f = rd<double>(); v.i = (int64_t)v.f; break;
        case STR: v.s = rds(); break;
        default: throw std::string("bad value type");
        }
    }
    void read_value(int t, Value &v) {
        if (t != ARR) { read_scalar(t, v); return; }
        v.arr_type = (int)rd<uint32_t>();
        const uint64_t n = rd<uint64_t>();
        for (uint64_t k = 0; k < n; ++k) {
            Value e;
            if (v.arr_type == ARR) throw std::string("nested arrays unsupported");
            read_scalar(v.arr_type, e);
            if (v.arr_type == STR) v.astr.push_back(std::move(e.s));
            else v.anum.push_back(v.arr_type == F32 || v.arr_type == F64 ? e.f : (double)e.i);
        }
        v.i = (int64_t)n;
    }
    int fd_ = -1;
    const uint8_t *map_ = nullptr;
    size_t size_ = 0, pos_ = 0;
};

}  // namespace gguf
