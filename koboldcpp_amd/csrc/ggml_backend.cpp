// ggml_backend.cpp -- the ggml backend plugin over this library's HIP kernels.
//
// What llama.cpp / ggml-backend.cpp see is the reference's ROCm backend interface (ggml/src/ggml-cuda.cu): a
// registry "ROCm" with one device per GPU (GPU_FULL), per-device buffer types with 128-B alignment whose
// get_alloc_size pads quantized rows to 512 elements and whose init_tensor zeroes that pad, a pinned host buffer
// type, backends (one HIP stream each) with async tensor copies, events and graph_compute(ggml_cgraph *), and
// the koboldcpp switch ggml_cuda_set_mul_mat_q.  The vtable types are the restated ones of
// include/kcpp_ggml_backend.h (same layout as ggml-backend-impl.h).
//
// graph_compute walks the nodes in order (ggml_backend_cuda_graph_compute, ggml-cuda.cu:2508-2778 with CUDA
// graphs off) and dispatches each to a kernel of this library:
//   MUL_MAT      quantized weight: activation -> Q8_K/Q8_0 (kcpp_quantize_act), then the mat-vec (M <= 8) or the
//                MFMA GEMM on a device-native image of the weight (row-major Q4_K_RS / Q5_K_RS / Q6_K_RS planes, the
//                structure-of-arrays Q4_0 / Q8_0 / Q2_K / Q3_K / Q6_K layouts), built once per weight on first use and kept until
//                the weight's buffer is written again; F16 / F32 weight: kcpp_ggml_mul_mat_f
//   GET_ROWS     quantized: kcpp_get_rows on the native image; F16 / F32: kcpp_ggml_get_rows
//   MUL_MAT_ID   quantized experts: expert-indexed mat-vecs reading the ids on the device (few rows), else the ids
//                on the host and the gathered columns of all experts in one grouped GEMM (Q4_K / Q5_K / Q6_K) or
//                one mat-vec / GEMM per expert (mul_mat_id below)
//   FLASH_ATTN_EXT  kcpp_flash_attn_ext (graph-form Q view, F16 K/V cache views, F16 mask; head dim 64 / 128) or
//                kcpp_flash_attn_ext_q (Q8_0 / Q4_0 K/V views: --quantkv)
//   RMS_NORM, ROPE (NORM / NEOX, YaRN), SOFT_MAX, ADD/SUB/MUL/DIV (broadcast), SCALE, UNARY (SILU/NEG/RELU),
//   CPY/CONT/DUP (F32 <-> F16; F32 -> Q8_0 / Q4_0 cache stores), ARGSORT, SUM_ROWS: the general-layout kernels of
//   ggml_ops.hip / attn_kvq.hip
//   NONE/RESHAPE/VIEW/PERMUTE/TRANSPOSE: nothing (views)
// supports_op answers true for exactly these (placement decides the rest onto the CPU backend, as
// ggml_backend_sched does with the reference's supports_op, ggml-cuda.cu:2959-3185).
//
// Errors: the reference aborts on a CUDA error (CUDA_CHECK, common.cuh:64-75); across this ABI nothing is
// thrown -- graph_compute returns GGML_STATUS_FAILED with the reason in kcpp_ggml_backend_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/kcpp_ggml_backend.h"
#include "../../include/kcpp_mi355x.h"
#include "../../include/kcpp_synth.h"
#include "kcpp_internal.h"

namespace {

std::string g_last_error;
int g_last_nodes = 0;
int g_last_fused = 0;     // of those, nodes that ran inside a fused launch (fuse_at)
int g_last_fused_launches = 0;   // and the fused launches they took
bool g_mul_mat_q = true;

// ggml type traits (ggml.c type_traits: blck_size, type_size, is_quantized) for every ggml_type id
struct TypeTrait { int blck, size; bool quant; };
const TypeTrait kTraits[KGGML_TYPE_COUNT] = {
    {1, 4, false},     {1, 2, false},     {32, 18, true},    {32, 20, true},   {0, 0, false},    {0, 0, false},
    {32, 22, true},    {32, 24, true},    {32, 34, true},    {32, 36, true},   {256, 84, true},  {256, 110, true},
    {256, 144, true},  {256, 176, true},  {256, 210, true},  {256, 292, true}, {256, 66, true},  {256, 74, true},
    {256, 98, true},   {256, 50, true},   {32, 18, true},    {256, 110, true}, {256, 82, true},  {256, 136, true},
    {1, 1, false},     {1, 2, false},     {1, 4, false},     {1, 8, false},    {1, 8, false},    {256, 56, true},
    {1, 2, false},     {32, 18, true},    {32, 18, true},    {32, 18, true},   {256, 54, true},  {256, 66, true},
};

bool type_ok(int t) { return t >= 0 && t < KGGML_TYPE_COUNT && kTraits[t].blck > 0; }
bool is_quantized(int t) { return type_ok(t) && kTraits[t].quant; }
size_t row_size(int t, int64_t ne) { return (size_t)kTraits[t].size * ne / kTraits[t].blck; }
// ggml_nbytes (ggml.c)
size_t nbytes(const kggml_tensor *t) {
    const int b = kTraits[t->type].blck;
    size_t n;
    if (b == 1) {
        n = kTraits[t->type].size;
        for (int i = 0; i < KGGML_MAX_DIMS; ++i) n += (t->ne[i] - 1) * t->nb[i];
    } else {
        n = t->ne[0] * t->nb[0] / b;
        for (int i = 1; i < KGGML_MAX_DIMS; ++i) n += (t->ne[i] - 1) * t->nb[i];
    }
    return n;
}
bool is_contiguous(const kggml_tensor *t) {   // ggml_is_contiguous
    size_t next = kTraits[t->type].size;
    if (t->ne[0] != kTraits[t->type].blck && t->nb[0] != next) return false;
    next *= t->ne[0] / kTraits[t->type].blck;
    for (int i = 1; i < KGGML_MAX_DIMS; ++i) {
        if (t->ne[i] != 1) {
            if (t->nb[i] != next) return false;
            next *= t->ne[i];
        }
    }
    return true;
}
int64_t nrows(const kggml_tensor *t) { return t->ne[1] * t->ne[2] * t->ne[3]; }
kcpp_tdesc td_of(const kggml_tensor *t) {
    kcpp_tdesc d;
    for (int i = 0; i < 4; ++i) { d.ne[i] = t->ne[i]; d.nb[i] = (int64_t)t->nb[i]; }
    return d;
}
float op_f(const kggml_tensor *t, int i) { float f; memcpy(&f, &t->op_params[i], 4); return f; }

bool set_err(const std::string &s) { g_last_error = s; fprintf(stderr, "[kcpp ggml backend] %s\n", s.c_str()); return false; }

// ------------------------------------------------------------------ buffers
// a weight held in its device-native layout IN PLACE of its ggml bytes (weight buffers only: one copy of the model)
struct InPlace {
    int tt;                    // native layout (kcpp type id)
    int gtype;                 // ggml type
    int64_t K, N1, NS;         // row length, rows per slice, slices (MUL_MAT_ID experts)
};
struct BufCtx {
    int device;
    void *dev_ptr;
    std::string name;
    unsigned gen = 0;          // bumped by every write through the buffer interface (native-image invalidation)
    std::map<const void *, InPlace> native;   // tensors of this buffer converted in place, by data pointer
    std::map<const void *, int> shared;       // tensors asked for in two layouts: separate images instead
};
struct BuftCtx {
    int device;
    std::string name;
};

// device-native images of quantized weights, keyed by (device, data pointer, ggml type, K, N, target layout)
struct Image { void *d; kggml_backend_buffer_t buf; unsigned gen; };
std::mutex g_img_mu;
std::map<std::tuple<int, const void *, int, int64_t, int64_t, int>, Image> g_images;

void drop_images(kggml_backend_buffer_t buf) {
    std::lock_guard<std::mutex> lk(g_img_mu);
    for (auto it = g_images.begin(); it != g_images.end();) {
        if (it->second.buf == buf) { hipFree(it->second.d); it = g_images.erase(it); }
        else ++it;
    }
}

// ggml <-> native conversion of a whole in-place tensor through a transient device buffer (slice by slice for
// expert tensors); synchronous on the caller's stream
bool convert_inplace(void *data, const InPlace &ip, bool to_ggml, hipStream_t s) {
    const size_t sb = row_size(ip.gtype, ip.K) * ip.N1, bytes = sb * ip.NS;
    void *tmp = nullptr;
    if (hipMalloc(&tmp, bytes) != hipSuccess) { (void)hipGetLastError(); return false; }
    bool ok = true;
    for (int64_t e = 0; e < ip.NS && ok; ++e)
        ok = kcpp_weight_repack(ip.tt, (const char *)data + e * sb, (char *)tmp + e * sb, ip.K, ip.N1, to_ggml ? 1 : 0, s) == 0;
    ok = ok && hipMemcpyAsync(data, tmp, bytes, hipMemcpyDeviceToDevice, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    hipFree(tmp);
    return ok;
}
// the in-place tensor covering [p, p + n) of buffer c, or end()
std::map<const void *, InPlace>::iterator inplace_at(BufCtx *c, const void *p, size_t n) {
    for (auto it = c->native.begin(); it != c->native.end(); ++it) {
        const size_t bytes = row_size(it->second.gtype, it->second.K) * it->second.N1 * it->second.NS;
        const char *b = (const char *)it->first;
        if ((const char *)p < b + bytes && (const char *)p + n > b) return it;
    }
    return c->native.end();
}
// back to ggml bytes before anything but this backend's mat-mul kernels touches [p, p + n)
void restore_ggml(BufCtx *c, const void *p, size_t n) {
    std::lock_guard<std::mutex> lk(g_img_mu);
    for (auto it = inplace_at(c, p, n); it != c->native.end(); it = inplace_at(c, p, n)) {
        hipSetDevice(c->device);
        hipDeviceSynchronize();                       // pending kernels may still read the native bytes
        if (!convert_inplace((void *)it->first, it->second, true, hipStreamPerThread))
            fprintf(stderr, "[kcpp ggml backend] restoring a weight's ggml layout failed\n");
        c->native.erase(it);
    }
}

const char *buf_get_name(kggml_backend_buffer_t b) { return ((BufCtx *)b->context)->name.c_str(); }
bool buffer_is_ours(kggml_backend_buffer_t b) { return b && b->iface.get_name == buf_get_name; }
void buf_free(kggml_backend_buffer_t b) {
    BufCtx *c = (BufCtx *)b->context;
    drop_images(b);
    hipSetDevice(c->device);
    hipDeviceSynchronize();
    hipSetDevice(c->device);
    hipFree(c->dev_ptr);
    delete c;
    // the host's ggml_backend_buffer_free deletes the struct (ggml-backend.cpp); ours when freed here directly
}
void *buf_get_base(kggml_backend_buffer_t b) { return ((BufCtx *)b->context)->dev_ptr; }

size_t buft_get_alloc_size(kggml_backend_buffer_type_t, const kggml_tensor *t);

// ggml_backend_cuda_buffer_init_tensor (ggml-cuda.cu:443-461): zero the row padding of quantized weights so the
// kernels may read into it
void buf_init_tensor(kggml_backend_buffer_t b, kggml_tensor *t) {
    if (t->view_src != nullptr) return;
    if (is_quantized(t->type) && b->usage != KGGML_BACKEND_BUFFER_USAGE_COMPUTE) {
        const size_t orig = nbytes(t), padded = buft_get_alloc_size(b->buft, t);
        if (padded > orig) {
            hipSetDevice(((BufCtx *)b->context)->device);
            hipMemset((char *)t->data + orig, 0, padded - orig);
        }
    }
}
void buf_memset_tensor(kggml_backend_buffer_t b, kggml_tensor *t, uint8_t v, size_t off, size_t size) {
    BufCtx *c = (BufCtx *)b->context;
    restore_ggml(c, (char *)t->data + off, size);
    hipSetDevice(c->device);
    ++c->gen;
    hipMemsetAsync((char *)t->data + off, v, size, hipStreamPerThread);
    hipStreamSynchronize(hipStreamPerThread);
}
void buf_set_tensor(kggml_backend_buffer_t b, kggml_tensor *t, const void *data, size_t off, size_t size) {
    BufCtx *c = (BufCtx *)b->context;
    restore_ggml(c, (char *)t->data + off, size);
    hipSetDevice(c->device);
    ++c->gen;
    hipMemcpyAsync((char *)t->data + off, data, size, hipMemcpyHostToDevice, hipStreamPerThread);
    hipStreamSynchronize(hipStreamPerThread);
}
void buf_get_tensor(kggml_backend_buffer_t b, const kggml_tensor *t, void *data, size_t off, size_t size) {
    restore_ggml((BufCtx *)b->context, (const char *)t->data + off, size);
    hipSetDevice(((BufCtx *)b->context)->device);
    hipMemcpyAsync(data, (const char *)t->data + off, size, hipMemcpyDeviceToHost, hipStreamPerThread);
    hipStreamSynchronize(hipStreamPerThread);
}
bool buf_cpy_tensor(kggml_backend_buffer_t b, const kggml_tensor *src, kggml_tensor *dst) {
    if (!buffer_is_ours(src->buffer)) return false;
    BufCtx *sc = (BufCtx *)src->buffer->context, *dc = (BufCtx *)dst->buffer->context;
    restore_ggml(sc, src->data, nbytes(src));
    restore_ggml(dc, dst->data, nbytes(dst));
    ++dc->gen;
    if (sc->device == dc->device) {
        hipSetDevice(dc->device);
        hipMemcpyAsync(dst->data, src->data, nbytes(src), hipMemcpyDeviceToDevice, hipStreamPerThread);
    } else {
        hipMemcpyPeerAsync(dst->data, dc->device, src->data, sc->device, nbytes(src), hipStreamPerThread);
    }
    hipStreamSynchronize(hipStreamPerThread);
    return true;
    (void)b;
}
void buf_clear(kggml_backend_buffer_t b, uint8_t v) {
    BufCtx *c = (BufCtx *)b->context;
    hipSetDevice(c->device);
    ++c->gen;
    hipDeviceSynchronize();
    {
        std::lock_guard<std::mutex> lk(g_img_mu);
        c->native.clear();                            // every byte is overwritten: no layout to restore
        c->shared.clear();
    }
    hipMemset(c->dev_ptr, v, b->size);
    hipDeviceSynchronize();
}
const kggml_backend_buffer_i kBufIface = {buf_get_name, buf_free,      buf_get_base,   buf_init_tensor, buf_memset_tensor,
                                          buf_set_tensor, buf_get_tensor, buf_cpy_tensor, buf_clear,       nullptr};

const char *buft_get_name(kggml_backend_buffer_type_t bt) { return ((BuftCtx *)bt->context)->name.c_str(); }
bool buft_is_ours(kggml_backend_buffer_type_t bt) { return bt && bt->iface.get_name == buft_get_name; }
kggml_backend_buffer_t buft_alloc_buffer(kggml_backend_buffer_type_t bt, size_t size) {
    BuftCtx *c = (BuftCtx *)bt->context;
    hipSetDevice(c->device);
    size = std::max<size_t>(size, 1);
    void *p = nullptr;
    if (hipMalloc(&p, size) != hipSuccess) {
        (void)hipGetLastError();
        set_err("alloc_buffer: hipMalloc of " + std::to_string(size) + " bytes failed on device " + std::to_string(c->device));
        return nullptr;
    }
    BufCtx *bc = new BufCtx{c->device, p, KGGML_CUDA_NAME + std::to_string(c->device)};
    // ggml_backend_buffer_init (ggml-backend.cpp): {iface, buft, context, size, usage ANY}
    return new kggml_backend_buffer{kBufIface, bt, bc, size, KGGML_BACKEND_BUFFER_USAGE_ANY};
}
size_t buft_get_alignment(kggml_backend_buffer_type_t) { return 128; }   // ggml-cuda.cu:567-571
// ggml-cuda.cu:573-586: quantized rows padded to a multiple of MATRIX_ROW_PADDING = 512 elements
size_t buft_get_alloc_size(kggml_backend_buffer_type_t, const kggml_tensor *t) {
    size_t size = nbytes(t);
    const int64_t ne0 = t->ne[0];
    if (is_quantized(t->type) && ne0 % 512 != 0) size += row_size(t->type, 512 - ne0 % 512);
    return size;
}
const kggml_backend_buffer_type_i kBuftIface = {buft_get_name, buft_alloc_buffer, buft_get_alignment, nullptr,
                                                buft_get_alloc_size, nullptr};

// pinned host buffer type (ggml_backend_cuda_host_buffer_type): host-visible, hipHostMalloc'd
struct HostBufCtx { void *p; };
const char *hbuf_get_name(kggml_backend_buffer_t) { return KGGML_CUDA_NAME "_Host"; }
void hbuf_free(kggml_backend_buffer_t b) { hipHostFree(((HostBufCtx *)b->context)->p); delete (HostBufCtx *)b->context; }
void *hbuf_get_base(kggml_backend_buffer_t b) { return ((HostBufCtx *)b->context)->p; }
void hbuf_memset(kggml_backend_buffer_t, kggml_tensor *t, uint8_t v, size_t off, size_t size) { memset((char *)t->data + off, v, size); }
void hbuf_set(kggml_backend_buffer_t, kggml_tensor *t, const void *d, size_t off, size_t size) { memcpy((char *)t->data + off, d, size); }
void hbuf_get(kggml_backend_buffer_t, const kggml_tensor *t, void *d, size_t off, size_t size) { memcpy(d, (const char *)t->data + off, size); }
void hbuf_clear(kggml_backend_buffer_t b, uint8_t v) { memset(((HostBufCtx *)b->context)->p, v, b->size); }
const kggml_backend_buffer_i kHostBufIface = {hbuf_get_name, hbuf_free, hbuf_get_base, nullptr, hbuf_memset,
                                              hbuf_set,      hbuf_get,  nullptr,       hbuf_clear, nullptr};
const char *hbuft_get_name(kggml_backend_buffer_type_t) { return KGGML_CUDA_NAME "_Host"; }
kggml_backend_buffer_t hbuft_alloc(kggml_backend_buffer_type_t bt, size_t size) {
    void *p = nullptr;
    size = std::max<size_t>(size, 1);
    if (hipHostMalloc(&p, size, hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        set_err("host buffer: hipHostMalloc failed");
        return nullptr;
    }
    return new kggml_backend_buffer{kHostBufIface, bt, new HostBufCtx{p}, size, KGGML_BACKEND_BUFFER_USAGE_ANY};
}
size_t hbuft_alignment(kggml_backend_buffer_type_t) { return 32; }    // TENSOR_ALIGNMENT of the CPU buffer type
bool hbuft_is_host(kggml_backend_buffer_type_t) { return true; }
const kggml_backend_buffer_type_i kHostBuftIface = {hbuft_get_name, hbuft_alloc, hbuft_alignment, nullptr, nullptr,
                                                    hbuft_is_host};

// ------------------------------------------------------------------ devices, registry
struct DevCtx {
    int device;
    std::string name, description;
};
kggml_backend_reg g_reg;
std::vector<kggml_backend_device> g_devs;
std::vector<kggml_backend_buffer_type> g_bufts;
kggml_backend_buffer_type g_host_buft = {kHostBuftIface, nullptr, nullptr};
kggml_guid g_guid = {0x2c, 0xdd, 0xe8, 0x1c, 0x65, 0xb3, 0x65, 0x73, 0x6a, 0x12, 0x88, 0x61, 0x1c, 0xc9, 0xdc, 0x25};
std::once_flag g_init_once;
void init_registry();

// ------------------------------------------------------------------ backend (one HIP stream)
struct Scratch {
    void *p = nullptr;
    size_t sz = 0;
    void *get(size_t n) {
        if (n <= sz) return p;
        if (p) hipFree(p);
        p = nullptr;
        sz = 0;
        if (hipMalloc(&p, n) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
        sz = n;
        return p;
    }
};
struct BackendCtx {
    int device;
    std::string name;
    hipStream_t stream;
    Scratch act, ws, fa, ids, xg, yg, gcnt;
    bool fa_exact = false;     // attention in the reference CPU's order with its f16 accumulator (attn_exact.hip)
    // single-token MUL_MAT on the fused mat-vec (quantize prologue) and FLASH_ATTN_EXT on the split decode kernel;
    // KCPP_B1_UNFUSED=1: one kernel per step as before (A/B)
    bool no_fused_mv = getenv("KCPP_B1_UNFUSED") && atoi(getenv("KCPP_B1_UNFUSED")) != 0;
    // node fusion (fuse_at): off with KCPP_B1_UNFUSED or KCPP_B1_NOFUSE, or kcpp_ggml_backend_set_fusion(be, 0)
    bool no_fuse = no_fused_mv || (getenv("KCPP_B1_NOFUSE") && atoi(getenv("KCPP_B1_NOFUSE")) != 0);
};

// the native image of weight w for target layout `tt` (kcpp type id); w itself when the layouts coincide
// (a 3-D MUL_MAT_ID expert tensor is repacked slice by slice: expert e's image starts at e * nb[2], like its bytes)
// In a weight buffer (usage WEIGHTS, as llama.cpp marks its model buffers, src/llama.cpp:8982) the tensor is converted
// IN PLACE on first use, so the model occupies its size once; every other access through the buffer interface
// restores the ggml bytes first (restore_ggml).  Elsewhere a separate image is kept, invalidated by writes.
const void *native_image(BackendCtx *bc, const kggml_tensor *w, int tt) {
    const int64_t K = w->ne[0], N = w->ne[1] * w->ne[2] * w->ne[3], NS = w->ne[2] * w->ne[3];
    if (tt == w->type && (tt == KT_Q4_K || tt == KT_Q5_K)) return w->data;      // kcpp layout = ggml layout
    kggml_backend_buffer_t buf = w->view_src ? w->view_src->buffer : w->buffer;
    if (buffer_is_ours(buf) && buf->usage == KGGML_BACKEND_BUFFER_USAGE_WEIGHTS && w->view_src != nullptr) {
        // a view of a weight: its separate image is packed from ggml bytes, so a root already converted in place goes
        // back to the ggml layout and keeps separate images from now on (no in-place layout under a live view)
        // (once the root is marked shared and nothing in place overlaps the view, there is nothing to restore: no host
        // sync on every MUL_MAT against the view; restore_ggml synchronises the device itself when it converts)
        BufCtx *c = (BufCtx *)buf->context;
        bool todo;
        {
            std::lock_guard<std::mutex> lk(g_img_mu);
            todo = !c->shared.count(w->view_src->data) || inplace_at(c, w->data, nbytes(w)) != c->native.end();
        }
        if (todo) {
            restore_ggml(c, w->data, nbytes(w));
            std::lock_guard<std::mutex> lk(g_img_mu);
            c->shared[w->view_src->data] = 1;
        }
    }
    if (buffer_is_ours(buf) && buf->usage == KGGML_BACKEND_BUFFER_USAGE_WEIGHTS && w->view_src == nullptr) {
        BufCtx *c = (BufCtx *)buf->context;
        std::lock_guard<std::mutex> lk(g_img_mu);
        auto it = c->native.find(w->data);
        if (it != c->native.end() && it->second.tt == tt) return w->data;
        if (it != c->native.end()) {                  // a second layout (e.g. tied embeddings): back to ggml bytes,
            hipStreamSynchronize(bc->stream);         // separate images for both from now on
            if (!convert_inplace(w->data, it->second, true, bc->stream)) return nullptr;
            c->native.erase(it);
            c->shared[w->data] = 1;
        } else if (!c->shared.count(w->data)) {
            const InPlace ip{tt, w->type, K, N / NS, NS};
            if (!convert_inplace(w->data, ip, false, bc->stream)) return nullptr;
            c->native[w->data] = ip;
            return w->data;
        }
    }
    const unsigned gen = buffer_is_ours(buf) ? ((BufCtx *)buf->context)->gen : 0;
    const auto key = std::make_tuple(bc->device, (const void *)w->data, w->type, K, N, tt);
    std::lock_guard<std::mutex> lk(g_img_mu);
    auto it = g_images.find(key);
    if (it != g_images.end() && it->second.gen == gen) return it->second.d;
    if (it != g_images.end()) { hipStreamSynchronize(bc->stream); hipFree(it->second.d); g_images.erase(it); }
    void *d = nullptr;
    if (hipMalloc(&d, row_size(w->type, K) * N) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
    const int64_t N1 = N / NS, sb = (int64_t)row_size(w->type, K) * N1;
    for (int64_t e = 0; e < NS; ++e)
        if (kcpp_weight_repack(tt, (const char *)w->data + e * sb, (char *)d + e * sb, K, N1, 0, bc->stream) != 0) {
            hipFree(d);
            return nullptr;
        }
    g_images[key] = Image{d, buf, gen};
    return d;
}

// decode-layout choice for mat-mul weights (as kcpp_model_create picks it)
int matmul_layout(int t, int64_t K) {
    if (t == KT_Q4_K && kcpp_rs_supported(KT_Q4_K_RS, K)) return KT_Q4_K_RS;
    if (t == KT_Q5_K && kcpp_rs_supported(KT_Q5_K_RS, K)) return KT_Q5_K_RS;
    if (t == KT_Q6_K && kcpp_rs_supported(KT_Q6_K_RS, K)) return KT_Q6_K_RS;
    return t;
}
bool matmul_quant_ok(int t) {
    return t == KT_Q4_0 || t == KT_Q4_1 || t == KT_Q5_0 || t == KT_Q5_1 || t == KT_Q8_0 || t == KT_Q2_K || t == KT_Q3_K ||
           t == KT_Q4_K || t == KT_Q5_K || t == KT_Q6_K || t == KT_IQ4_NL || t == KT_IQ4_XS ||
           t == KT_IQ2_XXS || t == KT_IQ2_XS || t == KT_IQ2_S || t == KT_IQ3_XXS || t == KT_IQ3_S || t == KT_IQ1_S || t == KT_IQ1_M;
}

// ------------------------------------------------------------------ split buffers (LLAMA_SPLIT_MODE_ROW)
// ggml_backend_cuda_split_buffer_type (ggml-cuda.cu:625-955): a weight's rows are spread over the devices by
// tensor_split (kcpp_row_split_range: cumulative normalised starts, bounds rounded down to 128 rows).  Each lane
// (device) holds its rows as a [K][rows] tensor already in the device layout of the type (one copy, repacked at
// set_tensor); tensor->extra points at the slices.  A MUL_MAT on such a weight runs on the main device's backend:
// the activation is quantized there, every other lane takes it by a peer copy, multiplies its slice on its own
// stream and copies its rows of the result back (ggml_cuda_op_mul_mat's split branch, ggml-cuda.cu:1403-1700).
// KCPP_VIRTUAL_DEVICES=n (tests) splits over n lanes on the visible GPUs (lane i on GPU i % count).
struct SplitExtra {
    int n;                                   // lanes
    int tt, gtype;                           // device layout, ggml type
    int64_t K;
    int64_t lo[KGGML_CUDA_MAX_DEVICES], hi[KGGML_CUDA_MAX_DEVICES];
    void *d[KGGML_CUDA_MAX_DEVICES];
};
struct SplitBuftCtx { float split[KGGML_CUDA_MAX_DEVICES]; int n; };
struct SplitBufCtx { std::vector<SplitExtra *> extras; };
struct SplitLane {                           // a lane's stream and scratch for the split mat-mul
    int dev = 0;
    hipStream_t s = nullptr;
    hipEvent_t done = nullptr;
    Scratch act, ws, y;
};
std::mutex g_split_mu;
std::map<std::vector<float>, kggml_backend_buffer_type> g_split_bufts;
SplitLane g_lanes[KGGML_CUDA_MAX_DEVICES];      // fixed slots: pointers to them stay valid

int n_lanes() {
    int n = (int)g_devs.size();
    if (const char *v = getenv("KCPP_VIRTUAL_DEVICES")) n = std::max(1, atoi(v));
    return std::min(n, (int)KGGML_CUDA_MAX_DEVICES);
}
int lane_device(int i) { return g_devs.empty() ? 0 : i % (int)g_devs.size(); }
SplitLane *get_lane(int i) {
    std::lock_guard<std::mutex> lk(g_split_mu);
    if (i < 0 || i >= (int)KGGML_CUDA_MAX_DEVICES) return nullptr;
    SplitLane &l = g_lanes[i];
    if (!l.s) {
        l.dev = lane_device(i);
        hipSetDevice(l.dev);
        if (hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&l.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        for (size_t j = 0; j < g_devs.size(); ++j)     // xGMI peer access both ways
            if ((int)j != l.dev) {
                hipDeviceEnablePeerAccess((int)j, 0);
                (void)hipGetLastError();
            }
    }
    return &l;
}
void split_rows(const SplitBuftCtx *c, int64_t nrows, int id, int64_t &lo, int64_t &hi) {
    kcpp_row_split_range(nrows, c->n, c->split, id, &lo, &hi);
}
size_t split_pad(int type, int64_t ne0) {    // pad of the last row to 512 elements (ggml-cuda.cu:732-735)
    return ne0 % 512 ? row_size(type, 512 - ne0 % 512) : 0;
}

const char *sbuf_get_name(kggml_backend_buffer_t) { return KGGML_CUDA_NAME "_Split"; }
bool buffer_is_split(kggml_backend_buffer_t b) { return b && b->iface.get_name == sbuf_get_name; }
void sbuf_free(kggml_backend_buffer_t b) {
    SplitBufCtx *c = (SplitBufCtx *)b->context;
    for (SplitExtra *x : c->extras) {
        for (int i = 0; i < x->n; ++i)
            if (x->d[i]) { hipSetDevice(lane_device(i)); hipFree(x->d[i]); }
        delete x;
    }
    delete c;
}
void *sbuf_get_base(kggml_backend_buffer_t) { return (void *)0x1000; }    // never dereferenced (the extras hold the data)
void sbuf_init_tensor(kggml_backend_buffer_t b, kggml_tensor *t) {
    const SplitBuftCtx *bc = (const SplitBuftCtx *)b->buft->context;
    SplitExtra *x = new SplitExtra{};
    x->n = bc->n; x->gtype = t->type; x->K = t->ne[0];
    x->tt = matmul_layout(t->type, t->ne[0]);
    const int64_t nr = nrows(t);
    for (int i = 0; i < x->n; ++i) {
        split_rows(bc, nr, i, x->lo[i], x->hi[i]);
        const int64_t n = x->hi[i] - x->lo[i];
        if (n <= 0) continue;
        const size_t sz = row_size(t->type, x->K) * n + split_pad(t->type, x->K);
        hipSetDevice(lane_device(i));
        if (hipMalloc(&x->d[i], sz) != hipSuccess) { (void)hipGetLastError(); x->d[i] = nullptr; set_err("split buffer: hipMalloc failed"); continue; }
        hipMemset(x->d[i], 0, sz);
    }
    ((SplitBufCtx *)b->context)->extras.push_back(x);
    t->extra = x;
}
// split tensors are written and read whole (ggml-cuda.cu:750-752, 795-797)
void sbuf_set_tensor(kggml_backend_buffer_t, kggml_tensor *t, const void *data, size_t off, size_t size) {
    SplitExtra *x = (SplitExtra *)t->extra;
    if (!x || off != 0 || size != nbytes(t)) { set_err("split buffer: tensors are set whole"); return; }
    const size_t rb = row_size(t->type, x->K);
    for (int i = 0; i < x->n; ++i) {
        const int64_t n = x->hi[i] - x->lo[i];
        if (n <= 0 || !x->d[i]) continue;
        hipSetDevice(lane_device(i));
        void *tmp = nullptr;
        if (hipMalloc(&tmp, rb * n) != hipSuccess) { (void)hipGetLastError(); set_err("split buffer: upload scratch"); return; }
        hipMemcpy(tmp, (const char *)data + x->lo[i] * rb, rb * n, hipMemcpyHostToDevice);
        kcpp_weight_repack(x->tt, tmp, x->d[i], x->K, n, 0, nullptr);
        hipDeviceSynchronize();
        hipFree(tmp);
    }
}
void sbuf_get_tensor(kggml_backend_buffer_t, const kggml_tensor *t, void *data, size_t off, size_t size) {
    const SplitExtra *x = (const SplitExtra *)t->extra;
    if (!x || off != 0 || size != nbytes(t)) { set_err("split buffer: tensors are read whole"); return; }
    const size_t rb = row_size(t->type, x->K);
    for (int i = 0; i < x->n; ++i) {
        const int64_t n = x->hi[i] - x->lo[i];
        if (n <= 0 || !x->d[i]) continue;
        hipSetDevice(lane_device(i));
        void *tmp = nullptr;
        if (hipMalloc(&tmp, rb * n) != hipSuccess) { (void)hipGetLastError(); set_err("split buffer: download scratch"); return; }
        kcpp_weight_repack(x->tt, x->d[i], tmp, x->K, n, 1, nullptr);
        hipMemcpy((char *)data + x->lo[i] * rb, tmp, rb * n, hipMemcpyDeviceToHost);
        hipFree(tmp);
    }
}
void sbuf_clear(kggml_backend_buffer_t b, uint8_t v) {
    for (SplitExtra *x : ((SplitBufCtx *)b->context)->extras)
        for (int i = 0; i < x->n; ++i)
            if (x->d[i]) {
                hipSetDevice(lane_device(i));
                hipMemset(x->d[i], v, row_size(x->gtype, x->K) * (x->hi[i] - x->lo[i]));
            }
}
const kggml_backend_buffer_i kSplitBufIface = {sbuf_get_name, sbuf_free,       sbuf_get_base, sbuf_init_tensor, nullptr,
                                               sbuf_set_tensor, sbuf_get_tensor, nullptr,     sbuf_clear,       nullptr};
const char *sbuft_get_name(kggml_backend_buffer_type_t) { return KGGML_CUDA_NAME "_Split"; }
bool buft_is_split(kggml_backend_buffer_type_t bt) { return bt && bt->iface.get_name == sbuft_get_name; }
kggml_backend_buffer_t sbuft_alloc(kggml_backend_buffer_type_t bt, size_t size) {
    // the slices are allocated per tensor in init_tensor; size bounds their sum (ggml-cuda.cu:860-868)
    return new kggml_backend_buffer{kSplitBufIface, bt, new SplitBufCtx, size, KGGML_BACKEND_BUFFER_USAGE_ANY};
}
size_t sbuft_alignment(kggml_backend_buffer_type_t) { return 128; }
size_t sbuft_alloc_size(kggml_backend_buffer_type_t bt, const kggml_tensor *t) {
    const SplitBuftCtx *c = (const SplitBuftCtx *)bt->context;
    size_t total = 0;
    for (int i = 0; i < c->n; ++i) {
        int64_t lo, hi;
        split_rows(c, nrows(t), i, lo, hi);
        if (hi > lo) total += row_size(t->type, t->ne[0]) * (hi - lo) + split_pad(t->type, t->ne[0]);
    }
    return total;
}
bool sbuft_is_host(kggml_backend_buffer_type_t) { return false; }
const kggml_backend_buffer_type_i kSplitBuftIface = {sbuft_get_name, sbuft_alloc, sbuft_alignment, nullptr,
                                                     sbuft_alloc_size, sbuft_is_host};

bool supports(const kggml_tensor *op) {
    auto f32 = [](const kggml_tensor *t) { return t && t->type == KGGML_TYPE_F32; };
    for (int i = 0; i < KGGML_MAX_SRC; ++i) {     // a split weight feeds only a quantized MUL_MAT (src0)
        const kggml_tensor *sr = op->src[i];
        if (!sr || !sr->buffer || !buffer_is_split(sr->buffer)) continue;
        if (op->op != KGGML_OP_MUL_MAT || i != 0 || !matmul_quant_ok(sr->type) || sr->ne[2] != 1 || sr->ne[3] != 1 ||
            !f32(op->src[1]) || op->src[1]->nb[0] != 4 || op->src[1]->ne[2] != 1 || op->src[1]->ne[3] != 1 ||
            !is_contiguous(op) || sr->ne[0] % 256 != 0)
            return false;
        return true;
    }
    switch (op->op) {
    case KGGML_OP_NONE: case KGGML_OP_RESHAPE: case KGGML_OP_VIEW: case KGGML_OP_PERMUTE: case KGGML_OP_TRANSPOSE:
        return true;
    case KGGML_OP_ADD: case KGGML_OP_SUB: case KGGML_OP_MUL: case KGGML_OP_DIV:
        return f32(op) && f32(op->src[0]) && f32(op->src[1]);
    case KGGML_OP_SCALE: case KGGML_OP_RMS_NORM:
        return f32(op) && f32(op->src[0]);
    case KGGML_OP_UNARY: {
        const int u = op->op_params[0];
        return (u == KGGML_UNARY_OP_SILU || u == KGGML_UNARY_OP_NEG || u == KGGML_UNARY_OP_RELU) && f32(op) &&
               f32(op->src[0]);
    }
    case KGGML_OP_CPY: case KGGML_OP_CONT: case KGGML_OP_DUP: {
        const int s = op->src[0]->type, d = op->op == KGGML_OP_CPY ? op->src[1]->type : op->type;
        if (op->op == KGGML_OP_CPY && s == KGGML_TYPE_F32 && (d == KGGML_TYPE_Q8_0 || d == KGGML_TYPE_Q4_0))
            return is_contiguous(op->src[0]) && is_contiguous(op->src[1]) && op->src[0]->ne[0] % 32 == 0;   // KV store
        return (s == KGGML_TYPE_F32 || s == KGGML_TYPE_F16) && (d == KGGML_TYPE_F32 || d == KGGML_TYPE_F16);
    }
    case KGGML_OP_ROPE: {
        const int mode = op->op_params[2];
        return f32(op) && f32(op->src[0]) && (mode == 0 || mode == 2) && op->src[0]->nb[0] == 4;
    }
    case KGGML_OP_SOFT_MAX:
        return f32(op) && f32(op->src[0]) && op_f(op, 1) == 0.0f &&
               (!op->src[1] || op->src[1]->type == KGGML_TYPE_F16 || op->src[1]->type == KGGML_TYPE_F32);
    case KGGML_OP_ARGSORT:
        return f32(op->src[0]) && op->type == KGGML_TYPE_I32;
    case KGGML_OP_SUM_ROWS:
        return f32(op) && f32(op->src[0]);
    case KGGML_OP_GET_ROWS: {
        const kggml_tensor *a = op->src[0], *ids = op->src[1];
        if (!f32(op) || ids->type != KGGML_TYPE_I32) return false;
        if (a->type == KGGML_TYPE_F32 || a->type == KGGML_TYPE_F16) return true;
        return matmul_quant_ok(a->type) && a->ne[2] == 1 && a->ne[3] == 1 && is_contiguous(a) && is_contiguous(ids) &&
               ids->ne[1] == 1 && ids->ne[2] == 1 && op->nb[0] == 4;
    }
    case KGGML_OP_MUL_MAT: {
        const kggml_tensor *a = op->src[0], *b = op->src[1];
        if (!f32(op) || !f32(b)) return false;
        if (a->type == KGGML_TYPE_F32 || a->type == KGGML_TYPE_F16) return true;
        return matmul_quant_ok(a->type) && a->ne[2] == 1 && a->ne[3] == 1 && is_contiguous(a) && b->nb[0] == 4 &&
               b->ne[2] == 1 && b->ne[3] == 1 && is_contiguous(op) && a->ne[0] % 256 == 0;
    }
    case KGGML_OP_MUL_MAT_ID: {             // ggml_cuda_mul_mat_id (ggml-cuda.cu:2003-2139): quantized experts
        const kggml_tensor *a = op->src[0], *b = op->src[1], *ids = op->src[2];
        return f32(op) && f32(b) && ids && ids->type == KGGML_TYPE_I32 && matmul_quant_ok(a->type) && a->ne[3] == 1 &&
               is_contiguous(a) && a->ne[0] % 256 == 0 && b->nb[0] == 4 && op->nb[0] == 4 && ids->nb[0] == 4 &&
               b->ne[3] == 1 && ids->ne[1] == b->ne[2] && op->ne[1] == ids->ne[0] && op->ne[2] == ids->ne[1];
    }
    case KGGML_OP_FLASH_ATTN_EXT: {
        // ggml_cuda_flash_attn_ext (fattn.cu:210-218, 298-345): head dim 64 or 128; K / V both F16 cache views
        // [n_kv][HKV][D], or both quantized Q8_0 / Q4_0 (--quantkv) views of ggml blocks at any block-aligned strides
        const kggml_tensor *q = op->src[0], *k = op->src[1], *v = op->src[2], *m = op->src[3];
        if (!f32(op) || !f32(q) || op_f(op, 1) != 0.0f || op_f(op, 2) != 0.0f || q->ne[3] != 1) return false;
        const int64_t D = q->ne[0], HKV = k->ne[2];
        if ((D != 64 && D != 128) || k->ne[0] != D || v->ne[0] != D) return false;
        if (v->ne[1] != k->ne[1] || v->ne[2] != HKV || q->ne[2] % HKV || q->nb[0] != 4 || !is_contiguous(op) ||
            (m && !(m->type == KGGML_TYPE_F16 && m->nb[0] == 2)))
            return false;
        const bool kq = k->type == KGGML_TYPE_Q8_0 || k->type == KGGML_TYPE_Q4_0;
        const bool vq = v->type == KGGML_TYPE_Q8_0 || v->type == KGGML_TYPE_Q4_0;
        if (kq && vq) {
            const size_t kb = kTraits[k->type].size, vb = kTraits[v->type].size;
            return k->nb[2] % kb == 0 && k->nb[1] % kb == 0 && v->nb[2] % vb == 0 && v->nb[1] % vb == 0 && k->nb[1] % 2 == 0;
        }
        if (k->type != KGGML_TYPE_F16 || v->type != KGGML_TYPE_F16) return false;
        return k->nb[1] == (size_t)(HKV * D * 2) && k->nb[2] == (size_t)(D * 2) && v->nb[1] == k->nb[1] &&
               v->nb[2] == (size_t)(D * 2);
    }
    default:
        return false;
    }
}

// GGML_OP_MUL_MAT_ID (ggml_cuda_mul_mat_id, ggml-cuda.cu:2003-2139): dst[:, j, t] = as[:, :, ids[j, t]] . b[:, j % ne11, t].
// A handful of rows (decode): one expert-indexed mat-vec per (j, t) that reads its expert id on the device
// (DecArgs.eid) and quantizes its own column (prologue 2) -- no host synchronisation.  More rows (prefill): the ids
// come to the host (the reference synchronises here too), the columns of each expert are gathered, quantized and
// multiplied by one grouped MFMA GEMM over all experts (kcpp_gemm_grouped; other types: one mat-vec / GEMM per
// expert), and the rows scattered back.
bool mul_mat_id(BackendCtx *bc, kggml_tensor *n) {
    hipStream_t s = bc->stream;
    const kggml_tensor *as = n->src[0], *b = n->src[1], *ids = n->src[2];
    const int64_t K = as->ne[0], N = as->ne[1], E = as->ne[2];
    const int64_t n_ids = ids->ne[0], n_tok = ids->ne[1], ne11 = b->ne[1];
    const int tt = matmul_layout(as->type, K);
    const char *W = (const char *)native_image(bc, as, tt);
    if (!W) return set_err("mul_mat_id: native image allocation failed");
    const int64_t eb = (int64_t)as->nb[2];
    auto chk = [&](int rc, const char *what) {
        if (rc == 0) return true;
        char msg[256];
        snprintf(msg, sizeof msg, "mul_mat_id: %s failed rc=%d on node '%s' (%s)", what, rc, n->name, kcpp_last_error());
        return set_err(msg);
    };
    if (n_ids * n_tok <= 16) {
        int rc = 0;
        for (int64_t t = 0; t < n_tok && rc == 0; ++t)
            for (int64_t j = 0; j < n_ids && rc == 0; ++j) {
                DecArgs d;
                memset(&d, 0, sizeof d);
                d.K = K; d.nseg = 1; d.W[0] = (const uint8_t *)W; d.N[0] = N;
                d.Y[0] = (float *)((char *)n->data + j * n->nb[1] + t * n->nb[2]);
                d.x = (const float *)((const char *)b->data + (j % ne11) * b->nb[1] + t * b->nb[2]);
                d.eid = (const int32_t *)((const char *)ids->data + j * ids->nb[0] + t * ids->nb[1]);
                d.ebytes = eb;
                d.n_exp = E;
                rc = kcpp_gemv_dec(tt, &d, 0, 2, 1, s);
                if (rc != 0 && (t > 0 || j > 0)) return chk(rc, "expert mat-vec");
            }
        if (rc == 0) return true;
        // rc on the first (j, t): this type / shape has no fused expert mat-vec (Q4_1 / Q5_1): per (j, t) the
        // column quantized on its own, then the generic mat-vec on the expert slice its device-resident id selects
        void *act1 = bc->act.get((size_t)kcpp_act_bytes(as->type, K, 1) + 256);
        if (act1) {
            rc = 0;
            for (int64_t t = 0; t < n_tok && rc == 0; ++t)
                for (int64_t j = 0; j < n_ids && rc == 0; ++j) {
                    const float *x = (const float *)((const char *)b->data + (j % ne11) * b->nb[1] + t * b->nb[2]);
                    float *y = (float *)((char *)n->data + j * n->nb[1] + t * n->nb[2]);
                    const int32_t *eid = (const int32_t *)((const char *)ids->data + j * ids->nb[0] + t * ids->nb[1]);
                    rc = kcpp_quantize_act(kcpp_vec_dot_type(as->type), x, K, act1, K, 1, s);
                    if (rc == 0) rc = kcpp_gemv_expert(tt, W, nullptr, K, N, act1, y, eid, eb, (int)E, nullptr, 0, s);
                }
            if (rc == 0) return true;
            return chk(rc, "expert mat-vec (generic)");
        }
        // otherwise the grouped path below
    }
    std::vector<int32_t> idh((size_t)n_ids * n_tok);
    if (hipStreamSynchronize(s) != hipSuccess) return set_err("mul_mat_id: stream error");
    for (int64_t t = 0; t < n_tok; ++t)
        if (hipMemcpy(idh.data() + t * n_ids, (const char *)ids->data + t * ids->nb[1], (size_t)n_ids * 4,
                      hipMemcpyDeviceToHost) != hipSuccess)
            return set_err("mul_mat_id: ids copy failed");
    // per expert: the (source column, destination row) byte offsets of its (j, t), in (t, j) order
    std::vector<std::vector<int64_t>> so(E), dof(E);
    for (int64_t t = 0; t < n_tok; ++t)
        for (int64_t j = 0; j < n_ids; ++j) {
            const int32_t e = idh[t * n_ids + j];
            if (e < 0 || e >= E) return set_err("mul_mat_id: expert id out of range");
            so[e].push_back((j % ne11) * (int64_t)b->nb[1] + t * (int64_t)b->nb[2]);
            dof[e].push_back(j * (int64_t)n->nb[1] + t * (int64_t)n->nb[2]);
        }
    const int64_t rows = n_ids * n_tok;
    int64_t *offs = (int64_t *)bc->ids.get((size_t)rows * 16 + 256);
    float *xg = (float *)bc->xg.get((size_t)rows * K * 4 + 256);
    float *yg = (float *)bc->yg.get((size_t)rows * N * 4 + 256);
    void *act = bc->act.get((size_t)kcpp_act_bytes(as->type, K, rows) + 256);
    if (!offs || !xg || !yg || !act) return set_err("mul_mat_id: scratch allocation failed");
    std::vector<int64_t> hoff;
    hoff.reserve((size_t)rows * 2);
    for (int64_t e = 0; e < E; ++e) hoff.insert(hoff.end(), so[e].begin(), so[e].end());
    for (int64_t e = 0; e < E; ++e) hoff.insert(hoff.end(), dof[e].begin(), dof[e].end());
    if (hipMemcpy(offs, hoff.data(), hoff.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        return set_err("mul_mat_id: offsets upload failed");
    // Q4_K / Q5_K / Q6_K (RS) experts: every expert's GEMM in one launch (kcpp_gemm_grouped) -- one gather, one
    // quantization, one scatter, grids over all experts' rows
    // (the int8 kernel's 16-B DMA of the Q8_K bsums plane needs rows * (K / 256) % 4 == 0, e.g. not K 11008 / 6400 at an
    // odd row count: those take the per-expert loop; the Q6_K kernel reads an f16 fragment image instead)
    const bool grouped = (((tt == KT_Q4_K || tt == KT_Q4_K_RS || tt == KT_Q5_K || tt == KT_Q5_K_RS) &&
                           (rows * (K / 256)) % 4 == 0) || tt == KT_Q6_K_RS) &&
                         K % 256 == 0 && E <= 64 && rows > 16;
    if (grouped) {
        std::vector<int32_t> cnt((size_t)E);
        for (int64_t e = 0; e < E; ++e) cnt[e] = (int32_t)so[e].size();
        int32_t *cnt_dev = (int32_t *)bc->gcnt.get(256);
        const int64_t gwb = kcpp_gemm_grouped_ws_bytes(tt, K, rows, (int)E);
        void *gws = gwb > 0 ? bc->ws.get((size_t)gwb + 256) : nullptr;
        if (!cnt_dev || (gwb > 0 && !gws)) return set_err("mul_mat_id: grouped scratch allocation failed");
        if (hipMemcpy(cnt_dev, cnt.data(), (size_t)E * 4, hipMemcpyHostToDevice) != hipSuccess)
            return set_err("mul_mat_id: counts upload failed");
        return chk(kcpp_rows_move_f32(b->data, offs, 0, xg, nullptr, K * 4, K, (int)rows, s), "gather") &&
               chk(kcpp_quantize_act(kcpp_vec_dot_type(as->type), xg, K, act, K, rows, s), "quantize_act") &&
               chk(kcpp_gemm_grouped(tt, W, nullptr, eb, K, N, act, rows, cnt.data(), cnt_dev, (int)E, yg, nullptr, 0,
                                     gws, s), "grouped gemm") &&
               chk(kcpp_rows_move_f32(yg, nullptr, N * 4, n->data, offs + rows, 0, N, (int)rows, s), "scatter");
    }
    int64_t r0 = 0;
    for (int64_t e = 0; e < E; ++e) {
        const int64_t c = (int64_t)so[e].size();
        if (c == 0) continue;
        if (!chk(kcpp_rows_move_f32(b->data, offs + r0, 0, xg, nullptr, K * 4, K, (int)c, s), "gather") ||
            !chk(kcpp_quantize_act(kcpp_vec_dot_type(as->type), xg, K, act, K, c, s), "quantize_act"))
            return false;
        const void *We = W + e * eb;
        if (c <= 8) {
            if (!chk(kcpp_gemv(tt, We, nullptr, K, N, act, c, yg, N, nullptr, 0, 0, s), "gemv")) return false;
        } else {
            void *ws = bc->ws.get((size_t)kcpp_gemm_workspace_bytes(tt, K, N, c) + 256);
            if (!ws) return set_err("mul_mat_id: GEMM workspace allocation failed");
            if (!chk(kcpp_gemm(tt, We, nullptr, K, N, act, c, yg, N, nullptr, 0, 0, ws, s), "gemm")) return false;
        }
        if (!chk(kcpp_rows_move_f32(yg, nullptr, N * 4, n->data, offs + rows + r0, 0, N, (int)c, s), "scatter"))
            return false;
        r0 += c;
    }
    return true;
}

// MUL_MAT on a split weight (see the split buffers above)
bool mul_mat_split(BackendCtx *bc, kggml_tensor *n) {
    hipStream_t s = bc->stream;
    const kggml_tensor *a = n->src[0], *b = n->src[1];
    const SplitExtra *x = (const SplitExtra *)a->extra;
    if (!x) return set_err("mul_mat: split weight without slices");
    const int64_t K = a->ne[0], N = a->ne[1], M = b->ne[1];
    const size_t abytes = (size_t)kcpp_act_bytes(a->type, K, M);
    void *act = bc->act.get(abytes + 256);
    if (!act) return set_err("mul_mat(split): activation scratch allocation failed");
    if (kcpp_quantize_act(kcpp_vec_dot_type(a->type), (const float *)b->data, (int64_t)(b->nb[1] / 4), act, K, M, s))
        return set_err("mul_mat(split): quantize_act failed");
    auto mm = [&](const void *W, int64_t rows, const void *ac, float *Y, int64_t ldy, Scratch &ws, hipStream_t st) {
        if (M <= 8) return kcpp_gemv(x->tt, W, nullptr, K, rows, ac, M, Y, ldy, nullptr, 0, 0, st);
        void *w = ws.get((size_t)kcpp_gemm_workspace_bytes(x->tt, K, rows, M) + 256);
        if (!w) return -100;
        return kcpp_gemm(x->tt, W, nullptr, K, rows, ac, M, Y, ldy, nullptr, 0, 0, w, st);
    };
    hipEvent_t ev_in = nullptr;
    int inl = -1;
    std::vector<SplitLane *> used;
    for (int i = 0; i < x->n; ++i) {
        const int64_t rows = x->hi[i] - x->lo[i];
        if (rows <= 0 || !x->d[i]) continue;
        if (inl < 0 && lane_device(i) == bc->device) { inl = i; continue; }
        SplitLane *l = get_lane(i);
        if (!l) return set_err("mul_mat(split): lane setup failed");
        if (!ev_in) {
            hipEventCreateWithFlags(&ev_in, hipEventDisableTiming);
            hipEventRecord(ev_in, s);
        }
        hipSetDevice(l->dev);
        void *lact = l->act.get(abytes + 256);
        float *ly = (float *)l->y.get((size_t)rows * M * 4 + 256);
        if (!lact || !ly) return set_err("mul_mat(split): lane scratch allocation failed");
        hipStreamWaitEvent(l->s, ev_in, 0);
        hipMemcpyPeerAsync(lact, l->dev, act, bc->device, abytes, l->s);
        const int rc = mm(x->d[i], rows, lact, ly, rows, l->ws, l->s);
        if (rc) { hipSetDevice(bc->device); return set_err("mul_mat(split): lane mat-mul failed rc=" + std::to_string(rc)); }
        hipMemcpy2DAsync((float *)n->data + x->lo[i], N * 4, ly, rows * 4, rows * 4, M, hipMemcpyDefault, l->s);
        hipEventRecord(l->done, l->s);
        used.push_back(l);
        hipSetDevice(bc->device);
    }
    if (inl >= 0) {
        const int rc = mm(x->d[inl], x->hi[inl] - x->lo[inl], act, (float *)n->data + x->lo[inl], N, bc->ws, s);
        if (rc) return set_err("mul_mat(split): main-device slice failed rc=" + std::to_string(rc));
    }
    for (SplitLane *l : used) hipStreamWaitEvent(s, l->done, 0);
    if (ev_in) hipEventDestroy(ev_in);
    return true;
}

bool compute_node(BackendCtx *bc, kggml_tensor *n) {
    hipStream_t s = bc->stream;
    const kcpp_tdesc td = td_of(n);
    kggml_tensor *a = n->src[0], *b = n->src[1];
    auto chk = [&](int rc, const char *what) {
        if (rc == 0) return true;
        char msg[256];
        snprintf(msg, sizeof msg, "%s failed rc=%d on node '%s' (%s)", what, rc, n->name, kcpp_last_error());
        return set_err(msg);
    };
    switch (n->op) {
    case KGGML_OP_NONE: case KGGML_OP_RESHAPE: case KGGML_OP_VIEW: case KGGML_OP_PERMUTE: case KGGML_OP_TRANSPOSE:
        return true;
    case KGGML_OP_ADD: case KGGML_OP_SUB: case KGGML_OP_MUL: case KGGML_OP_DIV: {
        const int op = n->op == KGGML_OP_ADD ? KCPP_BIN_ADD : n->op == KGGML_OP_SUB ? KCPP_BIN_SUB
                     : n->op == KGGML_OP_MUL ? KCPP_BIN_MUL : KCPP_BIN_DIV;
        const kcpp_tdesc ta = td_of(a), tb = td_of(b);
        return chk(kcpp_ggml_binary(op, a->data, &ta, b->data, &tb, n->data, &td, s), "binary");
    }
    case KGGML_OP_SCALE: {
        const kcpp_tdesc ta = td_of(a);
        return chk(kcpp_ggml_unary(KCPP_UN_SCALE, a->data, &ta, n->data, &td, op_f(n, 0), s), "scale");
    }
    case KGGML_OP_UNARY: {
        const int u = n->op_params[0];
        const int k = u == KGGML_UNARY_OP_SILU ? KCPP_UN_SILU : u == KGGML_UNARY_OP_NEG ? KCPP_UN_NEG : KCPP_UN_RELU;
        const kcpp_tdesc ta = td_of(a);
        return chk(kcpp_ggml_unary(k, a->data, &ta, n->data, &td, 0.0f, s), "unary");
    }
    case KGGML_OP_RMS_NORM: {
        const kcpp_tdesc ta = td_of(a);
        return chk(kcpp_ggml_rms_norm(a->data, &ta, n->data, &td, op_f(n, 0), s), "rms_norm");
    }
    case KGGML_OP_CPY: case KGGML_OP_CONT: case KGGML_OP_DUP: {
        const kcpp_tdesc ta = td_of(a);
        if (n->type == KGGML_TYPE_Q8_0 || n->type == KGGML_TYPE_Q4_0) {   // f32 -> quantized cache view (--quantkv)
            const int64_t ne = a->ne[0] * a->ne[1] * a->ne[2] * a->ne[3];
            return chk(kcpp_cpy_f32_q(n->type == KGGML_TYPE_Q8_0 ? KT_Q8_0 : KT_Q4_0, (const float *)a->data, ne, n->data, s),
                       "cpy(f32 -> quantized)");
        }
        // GGML_OP_CPY's node is a view of src[1]: writing the node writes the destination
        return chk(kcpp_ggml_cpy(a->type, a->data, &ta, n->type, n->data, &td, s), "cpy");
    }
    case KGGML_OP_ROPE: {
        const kcpp_tdesc ta = td_of(a);
        const kggml_tensor *ff = n->src[2];
        return chk(kcpp_ggml_rope(a->data, &ta, n->data, &td, (const int32_t *)b->data, ff ? (const float *)ff->data : nullptr,
                                  n->op_params[1], n->op_params[2], n->op_params[4], op_f(n, 5), op_f(n, 6), op_f(n, 7),
                                  op_f(n, 8), op_f(n, 9), op_f(n, 10), s),
                   "rope");
    }
    case KGGML_OP_SOFT_MAX: {
        const kcpp_tdesc ta = td_of(a);
        const kggml_tensor *m = b;
        const int mt = m ? (m->type == KGGML_TYPE_F16 ? KT_F16 : KT_F32) : KT_F32;
        const int64_t mld = m ? (int64_t)(m->nb[1] / kTraits[m->type].size) : 0;
        return chk(kcpp_ggml_soft_max(a->data, &ta, m ? m->data : nullptr, mt, mld, m ? m->ne[1] : 1, n->data, &td,
                                      op_f(n, 0), s),
                   "soft_max");
    }
    case KGGML_OP_ARGSORT: {
        const kcpp_tdesc ta = td_of(a);
        return chk(kcpp_ggml_argsort(a->data, &ta, (int32_t *)n->data, (int64_t)(n->nb[1] / 4), n->op_params[0] == 1, s),
                   "argsort");
    }
    case KGGML_OP_SUM_ROWS: {
        const kcpp_tdesc ta = td_of(a);
        return chk(kcpp_ggml_sum_rows(a->data, &ta, n->data, &td, s), "sum_rows");
    }
    case KGGML_OP_GET_ROWS: {
        if (a->type == KGGML_TYPE_F32 || a->type == KGGML_TYPE_F16) {
            const kcpp_tdesc ta = td_of(a), ti = td_of(b);
            return chk(kcpp_ggml_get_rows(a->type, a->data, &ta, (const int32_t *)b->data, &ti, n->data, &td, s),
                       "get_rows");
        }
        const void *img = native_image(bc, a, a->type);
        if (!img) return set_err("get_rows: native image allocation failed");
        return chk(kcpp_get_rows(a->type, img, a->ne[0], a->ne[1], (const int32_t *)b->data, b->ne[0], (float *)n->data,
                                 (int64_t)(n->nb[1] / 4), s),
                   "get_rows(quantized)");
    }
    case KGGML_OP_MUL_MAT: {
        if (a->buffer && buffer_is_split(a->buffer)) return mul_mat_split(bc, n);
        if (a->type == KGGML_TYPE_F32 || a->type == KGGML_TYPE_F16) {
            const kcpp_tdesc ta = td_of(a), tb = td_of(b);
            // F16 weights: the reference CPU (AVX2/F16C build) hands contiguous f32 src1 with K % 8 == 0 to
            // tinyBLAS unrounded (llamafile/sgemm.cpp:1094-1103), otherwise rounds src1 to f16 (vec_dot_f16)
            const int wt = a->type == KGGML_TYPE_F16 && is_contiguous(b) && a->ne[0] % 8 == 0 ? KCPP_MM_F16_X32 : a->type;
            return chk(kcpp_ggml_mul_mat_f(wt, a->data, &ta, (const float *)b->data, &tb, (float *)n->data, &td, s),
                       "mul_mat_f");
        }
        const int64_t K = a->ne[0], N = a->ne[1], M = b->ne[1];
        const int tt = matmul_layout(a->type, K);
        const void *W = native_image(bc, a, tt);
        if (!W) return set_err("mul_mat: native image allocation failed");
        if (M == 1 && b->nb[0] == 4 && (uintptr_t)b->data % 16 == 0 && !bc->no_fused_mv) {
            // one token (decode): the fused single-token mat-vec quantizes src1 in its own prologue (the same Q8_K /
            // Q8_0 bytes as kcpp_quantize_act) -- one launch per MUL_MAT instead of two; -3: type without it
            DecArgs d;
            memset(&d, 0, sizeof d);
            d.K = K; d.nseg = 1; d.W[0] = (const uint8_t *)W; d.N[0] = N; d.Y[0] = (float *)n->data;
            d.x = (const float *)b->data;
            if (kcpp_gemv_dec(tt, &d, 0, 2, N > 16384 ? 4 : (N > 4096 ? 2 : 1), s) == 0) return true;
            (void)hipGetLastError();            // not covered (type / shape): the two-launch path below
        }
        void *act = bc->act.get((size_t)kcpp_act_bytes(a->type, K, M) + 256);
        if (!act) return set_err("mul_mat: activation scratch allocation failed");
        if (!chk(kcpp_quantize_act(kcpp_vec_dot_type(a->type), (const float *)b->data, (int64_t)(b->nb[1] / 4), act, K, M, s),
                 "quantize_act"))
            return false;
        if (M <= 8)
            return chk(kcpp_gemv(tt, W, nullptr, K, N, act, M, (float *)n->data, N, nullptr, 0, 0, s), "gemv");
        void *ws = bc->ws.get((size_t)kcpp_gemm_workspace_bytes(tt, K, N, M) + 256);
        if (!ws) return set_err("mul_mat: GEMM workspace allocation failed");
        return chk(kcpp_gemm(tt, W, nullptr, K, N, act, M, (float *)n->data, N, nullptr, 0, 0, ws, s), "gemm");
    }
    case KGGML_OP_MUL_MAT_ID:
        return mul_mat_id(bc, n);
    case KGGML_OP_FLASH_ATTN_EXT: {
        const kggml_tensor *q = a, *k = b, *v = n->src[2], *m = n->src[3];
        const int T = (int)q->ne[1], H = (int)q->ne[2], HKV = (int)k->ne[2], n_kv = (int)k->ne[1], D = (int)q->ne[0];
        const uint16_t *mk = m ? (const uint16_t *)m->data : nullptr;
        const int64_t mld = m ? (int64_t)(m->nb[1] / 2) : 0;
        if (k->type != KGGML_TYPE_F16) {    // quantized K / V (the reference quantizes q to Q8_0, integer block dots)
            const int tk = k->type == KGGML_TYPE_Q8_0 ? KT_Q8_0 : KT_Q4_0, tv = v->type == KGGML_TYPE_Q8_0 ? KT_Q8_0 : KT_Q4_0;
            return chk(kcpp_flash_attn_ext_q(tk, tv, (const float *)q->data, (int64_t)q->nb[1], (int64_t)q->nb[2], k->data,
                                             (int64_t)k->nb[1], (int64_t)k->nb[2], v->data, (int64_t)v->nb[1],
                                             (int64_t)v->nb[2], mk, mld, (float *)n->data, T, H, HKV, D, n_kv, op_f(n, 0), s),
                       "flash_attn_ext(quantized K/V)");
        }
        if (bc->fa_exact)
            return chk(kcpp_flash_attn_ext_exact((const float *)q->data, (int64_t)q->nb[1], (int64_t)q->nb[2],
                                                 (const uint16_t *)k->data, (const uint16_t *)v->data, mk, mld,
                                                 (float *)n->data, T, H, HKV, D, n_kv, op_f(n, 0), s),
                       "flash_attn_ext(exact)");
        void *ws = bc->fa.get((size_t)kcpp_fa_ext_workspace_bytes(T, H, n_kv, D));
        if (!ws) return set_err("flash_attn_ext: workspace allocation failed");
        if (T == 1 && !bc->no_fused_mv) {   // one query: the production split kernel under the graph's mask, q rounded in it
            const int rc = kcpp_flash_attn_ext_dec((const float *)q->data, (int64_t)q->nb[2], (const uint16_t *)k->data,
                                                   (const uint16_t *)v->data, (int64_t)(k->nb[1] / 2), (int64_t)(k->nb[2] / 2),
                                                   mk, (float *)n->data, ws, H, HKV, D, n_kv, op_f(n, 0), s);
            if (rc != -3) return chk(rc, "flash_attn_ext(decode)");
        }
        return chk(kcpp_flash_attn_ext((const float *)q->data, (int64_t)q->nb[1], (int64_t)q->nb[2], (const uint16_t *)k->data,
                                       (const uint16_t *)v->data, mk, mld, (float *)n->data, ws, T, H, HKV, D, n_kv,
                                       op_f(n, 0), s),
                   "flash_attn_ext");
    }
    default:
        return set_err(std::string("unsupported op ") + std::to_string(n->op) + " on node '" + n->name + "'");
    }
}

// ------------------------------------------------------------------ node fusion (decode)
// Three node sequences of every llama-family token graph (build_norm, the residual ADD after wo / ffn_down, build_ffn's
// parallel SiLU GLU) run as one launch each.  A fused launch still writes EVERY node's output tensor, per element in
// node order, so the graph's tensors hold afterwards exactly what the node-by-node sequence leaves: no use counting is
// needed (a split view -- ggml_graph_view, ggml.c:19059 -- cannot see consumers in other splits, and an OUTPUT-flagged
// intermediate stays materialised).  What the fusion does need: the nodes consecutive in the graph, every output a
// plain contiguous f32 vector of one shape, and no output overlapping an input that other workgroups still read (the
// allocator may hand a dead input's bytes to a later node); outputs may coincide exactly with each other or with an
// element-wise input (ggml-alloc's in-place reuse).  Anything else runs node by node.  KCPP_B1_UNFUSED=1 disables it.
namespace {
bool mem_overlap(const kggml_tensor *a, const kggml_tensor *b) {
    const char *pa = (const char *)a->data, *pb = (const char *)b->data;
    return pa < pb + nbytes(b) && pb < pa + nbytes(a);
}
// the same bytes element for element: same start and size, both contiguous (a reshape of the other counts)
bool same_bytes(const kggml_tensor *a, const kggml_tensor *b) {
    return a->data == b->data && nbytes(a) == nbytes(b) && a->type == b->type && is_contiguous(a) && is_contiguous(b);
}
bool exact_or_disjoint(const kggml_tensor *a, const kggml_tensor *b) { return same_bytes(a, b) || !mem_overlap(a, b); }
bool f32_vec(const kggml_tensor *t, int64_t n) {   // a contiguous f32 [n, 1, 1, 1]
    return t && t->type == KGGML_TYPE_F32 && t->ne[0] == n && t->ne[1] == 1 && t->ne[2] == 1 && t->ne[3] == 1 &&
           t->nb[0] == 4 && t->data;
}
bool same_shape(const kggml_tensor *a, const kggml_tensor *b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}
// a single-token quantized MUL_MAT the fused mat-vec (compute_node's M == 1 path) runs
bool mv_node(const kggml_tensor *m) {
    const kggml_tensor *a = m->src[0], *b = m->src[1];
    return m->op == KGGML_OP_MUL_MAT && supports(m) && a && b && is_quantized(a->type) &&
           !(a->buffer && buffer_is_split(a->buffer)) && f32_vec(m, a->ne[1]) && f32_vec(b, a->ne[0]) && a->data &&
           (uintptr_t)b->data % 16 == 0;          // the quantize prologue reads the row 16 B at a time
}

// RMS_NORM -> MUL(norm, w): kcpp_ggml_rms_norm_mul writes the norm row, then the product row
// an RMS_NORM -> MUL(w) pair run inside the prologue of the mat-vec that consumes it (x, w: the norm's input and
// weight; r, y: the two nodes' tensors, stored by that launch's workgroup 0; eps: the norm's)
struct NormIn {
    kggml_tensor *x, *w, *r, *y;
    float eps;
    mutable bool write_r, write_y;
};
// the launch reads x (every workgroup) instead of y, so no output of it may touch x or w.  When ggml-alloc has already
// handed r's or y's bytes to an output of this launch, that tensor is dead (the allocator reuses only freed bytes:
// r's one consumer is the MUL, y's may all be inside this launch, as the GLU's gate and up) and the node sequence
// leaves the output there, so it is not written (r == y exactly: r, then y, in one thread).
bool fuse_dbg() { static const bool on = getenv("KCPP_B1_FUSE_DEBUG") != nullptr; return on; }
bool normin_ok(const NormIn *ni, std::initializer_list<const kggml_tensor *> outs) {
    if (!ni) return true;
    ni->write_r = ni->write_y = true;
    for (const kggml_tensor *o : outs) {
        if (!o) continue;
        if (mem_overlap(o, ni->x) || mem_overlap(o, ni->w)) {
            if (fuse_dbg()) fprintf(stderr, "[fuse] norm-in: output '%s' overlaps the norm input / weight\n", o->name);
            return false;
        }
        if (mem_overlap(o, ni->r)) ni->write_r = false;
        if (mem_overlap(o, ni->y)) ni->write_y = false;
    }
    return !mem_overlap(ni->r, ni->x) && !mem_overlap(ni->y, ni->x) && !mem_overlap(ni->r, ni->w) &&
           !mem_overlap(ni->y, ni->w) && exact_or_disjoint(ni->r, ni->y);
}
void normin_args(const NormIn *ni, DecArgs &d, AuxOut &o) {
    if (!ni) return;
    d.x = (const float *)ni->x->data;
    d.nw = (const float *)ni->w->data;
    d.eps = ni->eps;
    o.rn = ni->write_r ? (float *)ni->r->data : nullptr;
    o.yn = ni->write_y ? (float *)ni->y->data : nullptr;
}

int fuse_norm_mul(BackendCtx *bc, kggml_cgraph *g, int i) {
    if (i + 1 >= g->n_nodes) return 0;
    kggml_tensor *nn = g->nodes[i], *m = g->nodes[i + 1];
    if (nn->op != KGGML_OP_RMS_NORM || m->op != KGGML_OP_MUL || m->src[0] != nn || !supports(nn) || !supports(m)) return 0;
    kggml_tensor *x = nn->src[0], *w = m->src[1];
    if (!x || !w || w->type != KGGML_TYPE_F32 || !same_shape(x, nn) || !same_shape(nn, m)) return 0;
    if (x->nb[0] != 4 || nn->nb[0] != 4 || m->nb[0] != 4 || w->nb[0] != 4) return 0;
    for (int d = 0; d < 4; ++d)
        if (w->ne[d] <= 0 || m->ne[d] % w->ne[d] != 0) return 0;           // ggml_can_repeat
    if (!exact_or_disjoint(nn, m) || !exact_or_disjoint(x, nn) || !exact_or_disjoint(x, m) || mem_overlap(w, nn) ||
        mem_overlap(w, m))
        return 0;
    const kcpp_tdesc tx = td_of(x), tr = td_of(nn), ty = td_of(m), tw = td_of(w);
    if (kcpp_ggml_rms_norm_mul(x->data, &tx, nn->data, &tr, m->data, &ty, (const float *)w->data, &tw, op_f(nn, 0),
                               bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return 2;
}

// MUL_MAT(W, x) -> ADD(product, r): the mat-vec with the residual in its epilogue (aux[0] = the product node's output;
// the RS kernels' AUX instances -- other layouts return -3 and the two nodes run one by one)
int fuse_mv_add(BackendCtx *bc, kggml_cgraph *g, int i) {
    if (i + 1 >= g->n_nodes) return 0;
    kggml_tensor *mm = g->nodes[i], *ad = g->nodes[i + 1];
    if (ad->op != KGGML_OP_ADD || !supports(ad) || !mv_node(mm)) return 0;
    kggml_tensor *r = ad->src[0] == mm ? ad->src[1] : (ad->src[1] == mm ? ad->src[0] : nullptr);
    const int64_t N = mm->ne[0];
    kggml_tensor *x = mm->src[1];
    if (!r || r == mm || !f32_vec(r, N) || !f32_vec(ad, N)) return 0;
    kggml_tensor *a = mm->src[0];
    const int tt = matmul_layout(a->type, a->ne[0]);
    if (tt != KT_Q4_K_RS && tt != KT_Q5_K_RS && tt != KT_Q6_K_RS) return 0;
    if (mem_overlap(mm, x) || mem_overlap(ad, x) || !exact_or_disjoint(mm, ad) || !exact_or_disjoint(r, ad) ||
        !exact_or_disjoint(r, mm))
        return 0;
    const void *W = native_image(bc, a, tt);
    if (!W) return 0;
    DecArgs d;
    memset(&d, 0, sizeof d);
    d.K = a->ne[0]; d.nseg = 1; d.W[0] = (const uint8_t *)W; d.N[0] = N; d.Y[0] = (float *)ad->data;
    d.x = (const float *)x->data; d.res = (const float *)r->data;
    AuxOut o{};
    o.p0 = (float *)mm->data;
    if (kcpp_gemv_rs_aux(tt, &d, 0, &o, bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return 2;
}

// build_ffn's LLM_FFN_SILU + LLM_FFN_PAR: gate = MUL_MAT(Wg, x), s = SILU(gate), up = MUL_MAT(Wu, x), MUL(s, up), in
// either evaluation order of the two mat-vecs: the GLU mat-vec (mode 1, quantize prologue) writing gate, s, up, then
// the product (RS layouts; -3 elsewhere and the nodes run one by one)
int fuse_glu(BackendCtx *bc, kggml_cgraph *g, int i, const NormIn *ni = nullptr) {
    if (i + 3 >= g->n_nodes) return 0;
    kggml_tensor *p[3] = {g->nodes[i], g->nodes[i + 1], g->nodes[i + 2]}, *mu = g->nodes[i + 3];
    if (mu->op != KGGML_OP_MUL || !supports(mu)) return 0;
    auto in_window = [&](const kggml_tensor *t) { return t == p[0] || t == p[1] || t == p[2]; };
    auto is_silu = [](const kggml_tensor *t) {
        return t && t->op == KGGML_OP_UNARY && t->op_params[0] == KGGML_UNARY_OP_SILU && supports(t);
    };
    kggml_tensor *s = is_silu(mu->src[0]) ? mu->src[0] : (is_silu(mu->src[1]) ? mu->src[1] : nullptr);
    if (!s || !in_window(s)) return 0;
    kggml_tensor *up = mu->src[0] == s ? mu->src[1] : mu->src[0], *gate = s->src[0];
    if (!gate || !up || gate == up || !in_window(gate) || !in_window(up) || !mv_node(gate) || !mv_node(up)) return 0;
    kggml_tensor *x = gate->src[1], *wg = gate->src[0], *wu = up->src[0];
    if (up->src[1] != x || wg->type != wu->type || !same_shape(wg, wu)) return 0;
    if (ni && (x != ni->y || !normin_ok(ni, {gate, s, up, mu}))) return 0;
    const int64_t N = gate->ne[0];
    if (!f32_vec(s, N) || !f32_vec(mu, N)) return 0;
    kggml_tensor *outs[4] = {gate, s, up, mu};
    for (int j = 0; j < 4; ++j) {
        if (mem_overlap(outs[j], ni ? ni->x : x)) return 0;   // the row every workgroup reads
        for (int k = j + 1; k < 4; ++k)
            if (!exact_or_disjoint(outs[j], outs[k])) return 0;
    }
    const int tt = matmul_layout(wg->type, wg->ne[0]);
    if (tt != KT_Q4_K_RS && tt != KT_Q5_K_RS && tt != KT_Q6_K_RS) return 0;
    const void *Wg = native_image(bc, wg, tt), *Wu = native_image(bc, wu, tt);
    if (!Wg || !Wu) return 0;
    DecArgs d;
    memset(&d, 0, sizeof d);
    d.K = wg->ne[0]; d.nseg = 1; d.W[0] = (const uint8_t *)Wg; d.W2 = (const uint8_t *)Wu; d.N[0] = N;
    d.Y[0] = (float *)mu->data; d.x = (const float *)x->data;
    AuxOut o{};
    o.p0 = (float *)gate->data; o.p1 = (float *)s->data; o.p2 = (float *)up->data;
    normin_args(ni, d, o);
    if (kcpp_gemv_rs_aux(tt, &d, 1, &o, bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return 4;
}

// node i's output stored into an F16 cache slot right after: view-only nodes (no work here), then a CPY whose source
// holds node i's bytes (node i itself or a reshape of it: same data, both contiguous, same element count) and whose
// destination is a contiguous F16 view (llm_build_kv_store: ggml_cpy(k_cur / v_cur, ggml_view_1d(k_l / v_l, ...))).
// Returns the CPY's index (0: no such CPY).
int cpy16_after(kggml_cgraph *g, int i) {
    kggml_tensor *src = g->nodes[i];
    for (int j = i + 1; j < g->n_nodes && j <= i + 3; ++j) {
        kggml_tensor *n = g->nodes[j];
        if (n->op == KGGML_OP_NONE || n->op == KGGML_OP_RESHAPE || n->op == KGGML_OP_VIEW || n->op == KGGML_OP_PERMUTE ||
            n->op == KGGML_OP_TRANSPOSE)
            continue;
        if (n->op != KGGML_OP_CPY || !supports(n)) return 0;
        kggml_tensor *a = n->src[0], *d = n->src[1];
        if (!a || !d || a->type != KGGML_TYPE_F32 || d->type != KGGML_TYPE_F16 || !is_contiguous(a) || !is_contiguous(d) ||
            !is_contiguous(src) || a->data != src->data || nbytes(a) != nbytes(src))
            return 0;
        const int64_t ne = src->ne[0] * src->ne[1] * src->ne[2] * src->ne[3];
        if (d->ne[0] * d->ne[1] * d->ne[2] * d->ne[3] != ne || n->data != d->data) return 0;
        return j;
    }
    return 0;
}

// ROPE -> CPY into the F16 cache: the rope kernel stores each value as f16 too (kcpp_ggml_rope_f16)
int fuse_rope_cpy(BackendCtx *bc, kggml_cgraph *g, int i) {
    kggml_tensor *n = g->nodes[i];
    if (n->op != KGGML_OP_ROPE || !supports(n)) return 0;
    const int j = cpy16_after(g, i);
    if (!j) return 0;
    kggml_tensor *x = n->src[0], *d = g->nodes[j]->src[1];
    if (mem_overlap(d, n) || mem_overlap(d, x) || (n->src[1] && mem_overlap(d, n->src[1]))) return 0;
    const int mode = n->op_params[2];
    const kcpp_tdesc ta = td_of(x), td = td_of(n);
    const float *ff = n->src[2] ? (const float *)n->src[2]->data : nullptr;
    if (kcpp_ggml_rope_f16(x->data, &ta, n->data, &td, d->data, (const int32_t *)n->src[1]->data, ff, n->op_params[1],
                           mode, n->op_params[4], op_f(n, 5), op_f(n, 6), op_f(n, 7), op_f(n, 8), op_f(n, 9), op_f(n, 10),
                           bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return j - i + 1;
}

// single-token MUL_MAT -> CPY into the F16 cache (the V store): the mat-vec also stores the product as f16 (AuxOut h0)
int fuse_mv_cpy(BackendCtx *bc, kggml_cgraph *g, int i) {
    kggml_tensor *mm = g->nodes[i];
    if (!mv_node(mm)) return 0;
    const int j = cpy16_after(g, i);
    if (!j) return 0;
    kggml_tensor *a = mm->src[0], *x = mm->src[1], *d = g->nodes[j]->src[1];
    const int tt = matmul_layout(a->type, a->ne[0]);
    if (tt != KT_Q4_K_RS && tt != KT_Q5_K_RS && tt != KT_Q6_K_RS) return 0;
    if (mem_overlap(mm, x) || mem_overlap(d, x) || mem_overlap(d, mm)) return 0;
    const void *W = native_image(bc, a, tt);
    if (!W) return 0;
    DecArgs dd;
    memset(&dd, 0, sizeof dd);
    dd.K = a->ne[0]; dd.nseg = 1; dd.W[0] = (const uint8_t *)W; dd.N[0] = mm->ne[0]; dd.Y[0] = (float *)mm->data;
    dd.x = (const float *)x->data;
    AuxOut o{};
    o.h0 = (uint16_t *)d->data;
    if (kcpp_gemv_rs_aux(tt, &dd, 0, &o, bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return j - i + 1;
}

// single-token MUL_MAT -> RESHAPE -> ROPE (NORM, n_dims = head size) [-> CPY into the F16 cache]: the q / k path of
// build_llama; the mat-vec stores the product, the roped values (two rows per group: a pair per lane, ggml_rope_cs --
// the ROPE kernel's own code) and their f16 copy
int fuse_mv_rope(BackendCtx *bc, kggml_cgraph *g, int i, const NormIn *ni = nullptr) {
    kggml_tensor *mm = g->nodes[i];
    if (!mv_node(mm)) return 0;
    int k = i + 1;
    while (k < g->n_nodes && k <= i + 2 && (g->nodes[k]->op == KGGML_OP_RESHAPE || g->nodes[k]->op == KGGML_OP_VIEW)) ++k;
    if (k >= g->n_nodes) return 0;
    kggml_tensor *rp = g->nodes[k];
    if (rp->op != KGGML_OP_ROPE || !supports(rp)) return 0;
    kggml_tensor *rx = rp->src[0], *pos = rp->src[1];
    const int n_dims = rp->op_params[1], mode = rp->op_params[2];
    if (!rx || !pos || pos->type != KGGML_TYPE_I32 || mode != 0 || rx->data != mm->data || !is_contiguous(rx) ||
        nbytes(rx) != nbytes(mm) || n_dims != rx->ne[0] || rx->ne[0] % 2 || rx->ne[2] != 1 || rx->ne[3] != 1 ||
        !is_contiguous(rp) || !same_shape(rp, rx) || rp->type != KGGML_TYPE_F32)
        return 0;
    if (rp->src[2] && rp->src[2]->type != KGGML_TYPE_F32) return 0;
    kggml_tensor *a = mm->src[0], *x = mm->src[1];
    const int tt = matmul_layout(a->type, a->ne[0]);
    if (tt != KT_Q4_K_RS && tt != KT_Q5_K_RS && tt != KT_Q6_K_RS) return 0;
    const int j = cpy16_after(g, k);
    kggml_tensor *d = j ? g->nodes[j]->src[1] : nullptr;
    const kggml_tensor *xin = ni ? ni->x : x;   // the row every workgroup reads
    if (mem_overlap(mm, xin) || mem_overlap(rp, xin) || !exact_or_disjoint(mm, rp) || mem_overlap(pos, rp) ||
        mem_overlap(pos, mm))
        return 0;
    if (d && (mem_overlap(d, xin) || mem_overlap(d, mm) || mem_overlap(d, rp))) return 0;
    if (ni && (x != ni->y || !normin_ok(ni, {mm, rp, d}))) return 0;
    const void *W = native_image(bc, a, tt);
    if (!W) return 0;
    DecArgs dd;
    memset(&dd, 0, sizeof dd);
    dd.K = a->ne[0]; dd.nseg = 1; dd.W[0] = (const uint8_t *)W; dd.N[0] = mm->ne[0]; dd.Y[0] = (float *)mm->data;
    dd.x = (const float *)x->data;
    AuxOut o{};
    o.h0 = d ? (uint16_t *)d->data : nullptr;
    float cst[4];
    kcpp_ggml_rope_consts(n_dims, rp->op_params[4], op_f(rp, 5), op_f(rp, 6), op_f(rp, 8), op_f(rp, 9), op_f(rp, 10), cst);
    o.rope.out = (float *)rp->data;
    o.rope.pos = (const int32_t *)pos->data;
    o.rope.ff = rp->src[2] ? (const float *)rp->src[2]->data : nullptr;
    o.rope.D = (int)rx->ne[0];
    o.rope.theta_scale = cst[0]; o.rope.corr0 = cst[1]; o.rope.corr1 = cst[2]; o.rope.mscale_ext = cst[3];
    o.rope.freq_scale = op_f(rp, 6); o.rope.ext_factor = op_f(rp, 7); o.rope.attn_factor = op_f(rp, 8);
    normin_args(ni, dd, o);
    if (kcpp_gemv_rs_aux(tt, &dd, 0, &o, bc->stream) != 0) {
        (void)hipGetLastError();
        return 0;
    }
    return (j ? j : k) - i + 1;
}

// RMS_NORM -> MUL(w) -> its first consumer as one launch: the consumer mat-vec (the GLU quadruple or a MUL_MAT ->
// ROPE chain) normalises x in its prologue -- the plugin's norm kernels sum in that prologue's order for rows up to
// 4096 (ggml_ops.hip row_sumsq16), so r, y and the consumer's result are the node sequence's bits -- and its
// workgroup 0 stores r and y for the later consumers
int fuse_norm_into(BackendCtx *bc, kggml_cgraph *g, int i) {
    if (i + 2 >= g->n_nodes) return 0;
    kggml_tensor *nn = g->nodes[i], *m = g->nodes[i + 1];
    if (nn->op != KGGML_OP_RMS_NORM || m->op != KGGML_OP_MUL || m->src[0] != nn || !supports(nn) || !supports(m)) return 0;
    kggml_tensor *x = nn->src[0], *w = m->src[1];
    const int64_t K = nn->ne[0];
    if (!x || !w || K > 4096 || K % 256 || !f32_vec(x, K) || !f32_vec(nn, K) || !f32_vec(m, K) || !f32_vec(w, K)) return 0;
    for (const kggml_tensor *t : {x, w, nn, m})     // the prologue moves 16 B per access
        if ((uintptr_t)t->data % 16) return 0;
    const NormIn ni{x, w, nn, m, op_f(nn, 0), true, true};
    if (g->nodes[i + 2]->op != KGGML_OP_MUL_MAT) return 0;
    int k = fuse_glu(bc, g, i + 2, &ni);
    if (!k) k = fuse_mv_rope(bc, g, i + 2, &ni);
    if (!k && fuse_dbg()) fprintf(stderr, "[fuse] norm-in: no consumer pattern at '%s' after '%s'\n", g->nodes[i + 2]->name, nn->name);
    return k ? k + 2 : 0;
}

// the number of nodes node i starts a fused launch for (0: none)
int fuse_at(BackendCtx *bc, kggml_cgraph *g, int i) {
    switch (g->nodes[i]->op) {
    case KGGML_OP_RMS_NORM: {
        const int k = fuse_norm_into(bc, g, i);
        return k ? k : fuse_norm_mul(bc, g, i);
    }
    case KGGML_OP_ROPE: return fuse_rope_cpy(bc, g, i);
    case KGGML_OP_MUL_MAT: {
        int k = fuse_glu(bc, g, i);
        if (!k) k = fuse_mv_add(bc, g, i);
        if (!k) k = fuse_mv_rope(bc, g, i);
        return k ? k : fuse_mv_cpy(bc, g, i);
    }
    default: return 0;
    }
}
}  // namespace

const char *be_get_name(kggml_backend_t be) { return ((BackendCtx *)be->context)->name.c_str(); }
void be_free(kggml_backend_t be) {
    BackendCtx *c = (BackendCtx *)be->context;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    for (Scratch *sc : {&c->act, &c->ws, &c->fa, &c->ids, &c->xg, &c->yg, &c->gcnt}) if (sc->p) hipFree(sc->p);
    hipStreamDestroy(c->stream);
    delete c;
    delete be;
}
kggml_backend_buffer_type_t be_default_buft(kggml_backend_t be) {
    return ggml_backend_cuda_buffer_type(((BackendCtx *)be->context)->device);
}
void be_set_async(kggml_backend_t be, kggml_tensor *t, const void *data, size_t off, size_t size) {
    BackendCtx *c = (BackendCtx *)be->context;
    kggml_backend_buffer_t buf = t->view_src ? t->view_src->buffer : t->buffer;
    if (buffer_is_ours(buf)) {
        restore_ggml((BufCtx *)buf->context, (char *)t->data + off, size);
        ++((BufCtx *)buf->context)->gen;
    }
    hipSetDevice(c->device);
    hipMemcpyAsync((char *)t->data + off, data, size, hipMemcpyHostToDevice, c->stream);
}
void be_get_async(kggml_backend_t be, const kggml_tensor *t, void *data, size_t off, size_t size) {
    BackendCtx *c = (BackendCtx *)be->context;
    kggml_backend_buffer_t buf = t->view_src ? t->view_src->buffer : t->buffer;
    if (buffer_is_ours(buf)) restore_ggml((BufCtx *)buf->context, (const char *)t->data + off, size);
    hipSetDevice(c->device);
    hipMemcpyAsync(data, (const char *)t->data + off, size, hipMemcpyDeviceToHost, c->stream);
}
// device-to-device between two of our backends, ordered on the source stream, then the destination waits
// (ggml_backend_cuda_cpy_tensor_async, ggml-cuda.cu:2392-2445)
bool be_cpy_async(kggml_backend_t src_be, kggml_backend_t dst_be, const kggml_tensor *src, kggml_tensor *dst) {
    if (!ggml_backend_is_cuda(src_be) || !ggml_backend_is_cuda(dst_be)) return false;
    kggml_backend_buffer_t sb = src->view_src ? src->view_src->buffer : src->buffer;
    kggml_backend_buffer_t db = dst->view_src ? dst->view_src->buffer : dst->buffer;
    if (!buffer_is_ours(sb) || !buffer_is_ours(db)) return false;
    BackendCtx *sc = (BackendCtx *)src_be->context, *dc = (BackendCtx *)dst_be->context;
    restore_ggml((BufCtx *)sb->context, src->data, nbytes(src));
    restore_ggml((BufCtx *)db->context, dst->data, nbytes(dst));
    ++((BufCtx *)db->context)->gen;
    hipSetDevice(sc->device);
    if (sc->device == dc->device) {
        hipMemcpyAsync(dst->data, src->data, nbytes(dst), hipMemcpyDeviceToDevice, sc->stream);
    } else {
        hipMemcpyPeerAsync(dst->data, dc->device, src->data, sc->device, nbytes(dst), sc->stream);
    }
    if (src_be != dst_be) {
        hipEvent_t ev;
        hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        hipEventRecord(ev, sc->stream);
        hipSetDevice(dc->device);
        hipStreamWaitEvent(dc->stream, ev, 0);
        hipEventDestroy(ev);
    }
    return true;
}
void be_synchronize(kggml_backend_t be) {
    BackendCtx *c = (BackendCtx *)be->context;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
}
int be_graph_compute(kggml_backend_t be, kggml_cgraph *g) {
    BackendCtx *c = (BackendCtx *)be->context;
    hipSetDevice(c->device);
    g_last_nodes = 0;
    g_last_fused = 0;
    g_last_fused_launches = 0;
    for (int i = 0; i < g->n_nodes; ++i) {
        kggml_tensor *n = g->nodes[i];
        if (n->ne[0] == 0 || n->ne[1] == 0 || n->ne[2] == 0 || n->ne[3] == 0) continue;   // ggml_is_empty
        if (!supports(n)) { set_err(std::string("graph_compute: unsupported node '") + n->name + "'"); return KGGML_STATUS_FAILED; }
        if (!c->no_fuse) {
            const int k = fuse_at(c, g, i);
            if (k) {
                g_last_nodes += k;
                g_last_fused += k;
                ++g_last_fused_launches;
                i += k - 1;
                continue;
            }
        }
        if (!compute_node(c, n)) return KGGML_STATUS_FAILED;
        ++g_last_nodes;
    }
    if (hipGetLastError() != hipSuccess) { set_err("graph_compute: HIP launch error"); return KGGML_STATUS_FAILED; }
    return KGGML_STATUS_SUCCESS;
}
void be_event_record(kggml_backend_t be, kggml_backend_event_t ev) {
    hipEventRecord((hipEvent_t)ev->context, ((BackendCtx *)be->context)->stream);
}
void be_event_wait(kggml_backend_t be, kggml_backend_event_t ev) {
    hipStreamWaitEvent(((BackendCtx *)be->context)->stream, (hipEvent_t)ev->context, 0);
}
const kggml_backend_i kBackendIface = {be_get_name,  be_free,        be_default_buft, be_set_async,    be_get_async,
                                       be_cpy_async, be_synchronize, nullptr,         nullptr,         nullptr,
                                       nullptr,      be_graph_compute, nullptr,       nullptr,         nullptr,
                                       be_event_record, be_event_wait};

const char *dev_get_name(kggml_backend_dev_t d) { return ((DevCtx *)d->context)->name.c_str(); }
const char *dev_get_description(kggml_backend_dev_t d) { return ((DevCtx *)d->context)->description.c_str(); }
void dev_get_memory(kggml_backend_dev_t d, size_t *free, size_t *total) {
    hipSetDevice(((DevCtx *)d->context)->device);
    hipMemGetInfo(free, total);
}
int dev_get_type(kggml_backend_dev_t) { return KGGML_BACKEND_DEVICE_TYPE_GPU_FULL; }
void dev_get_props(kggml_backend_dev_t d, kggml_backend_dev_props *p) {
    p->name = dev_get_name(d);
    p->description = dev_get_description(d);
    p->type = dev_get_type(d);
    dev_get_memory(d, &p->memory_free, &p->memory_total);
    p->caps = {true, getenv("GGML_CUDA_NO_PINNED") == nullptr, false, true};
}
kggml_backend_t dev_init_backend(kggml_backend_dev_t d, const char *) { return ggml_backend_cuda_init(((DevCtx *)d->context)->device); }
kggml_backend_buffer_type_t dev_get_buft(kggml_backend_dev_t d) { return ggml_backend_cuda_buffer_type(((DevCtx *)d->context)->device); }
kggml_backend_buffer_type_t dev_get_host_buft(kggml_backend_dev_t) { return ggml_backend_cuda_host_buffer_type(); }
bool dev_supports_op(kggml_backend_dev_t, const kggml_tensor *op) { return supports(op); }
bool dev_supports_buft(kggml_backend_dev_t d, kggml_backend_buffer_type_t bt) {
    if (buft_is_split(bt)) return true;                       // ggml-cuda.cu:3188-3190
    return buft_is_ours(bt) && ((BuftCtx *)bt->context)->device == ((DevCtx *)d->context)->device;
}
// ggml-cuda.cu:3201-3208: batches of >= 32 pull CPU-resident weights over
bool dev_offload_op(kggml_backend_dev_t, const kggml_tensor *op) {
    return (op->ne[1] >= 32 && op->op != KGGML_OP_GET_ROWS) || (op->ne[2] >= 32 && op->op == KGGML_OP_MUL_MAT_ID);
}
kggml_backend_event_t dev_event_new(kggml_backend_dev_t d) {
    hipSetDevice(((DevCtx *)d->context)->device);
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return nullptr;
    return new kggml_backend_event{d, ev};
}
void dev_event_free(kggml_backend_dev_t, kggml_backend_event_t ev) {
    hipEventDestroy((hipEvent_t)ev->context);
    delete ev;
}
void dev_event_sync(kggml_backend_dev_t, kggml_backend_event_t ev) { hipEventSynchronize((hipEvent_t)ev->context); }
const kggml_backend_device_i kDevIface = {dev_get_name,    dev_get_description, dev_get_memory,  dev_get_type,
                                          dev_get_props,   dev_init_backend,    dev_get_buft,    dev_get_host_buft,
                                          nullptr,         dev_supports_op,     dev_supports_buft, dev_offload_op,
                                          dev_event_new,   dev_event_free,      dev_event_sync};

const char *reg_get_name(kggml_backend_reg_t) { return KGGML_CUDA_NAME; }
size_t reg_get_device_count(kggml_backend_reg_t) { return g_devs.size(); }
kggml_backend_dev_t reg_get_device(kggml_backend_reg_t, size_t i) { return i < g_devs.size() ? &g_devs[i] : nullptr; }
void *reg_get_proc_address(kggml_backend_reg_t, const char *name) {
    if (!strcmp(name, "ggml_backend_split_buffer_type")) return (void *)ggml_backend_cuda_split_buffer_type;
    if (!strcmp(name, "ggml_backend_register_host_buffer")) return (void *)ggml_backend_cuda_register_host_buffer;
    if (!strcmp(name, "ggml_backend_unregister_host_buffer")) return (void *)ggml_backend_cuda_unregister_host_buffer;
    return nullptr;
}
const kggml_backend_reg_i kRegIface = {reg_get_name, reg_get_device_count, reg_get_device, reg_get_proc_address};

void init_registry() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); n = 0; }
    n = std::min(n, KGGML_CUDA_MAX_DEVICES);
    g_reg = kggml_backend_reg{kRegIface, nullptr};
    g_devs.resize(n);
    g_bufts.resize(n);
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        std::string desc = "AMD GPU";
        if (hipGetDeviceProperties(&prop, i) == hipSuccess) desc = prop.name;
        g_devs[i] = kggml_backend_device{kDevIface, &g_reg, new DevCtx{i, KGGML_CUDA_NAME + std::to_string(i), desc}};
        g_bufts[i] = kggml_backend_buffer_type{kBuftIface, &g_devs[i], new BuftCtx{i, KGGML_CUDA_NAME + std::to_string(i)}};
    }
    g_host_buft.device = n > 0 ? &g_devs[0] : nullptr;
}

}  // namespace

extern "C" {

kggml_backend_reg_t ggml_backend_cuda_reg(void) {
    std::call_once(g_init_once, init_registry);
    return &g_reg;
}
int ggml_backend_cuda_get_device_count(void) {
    std::call_once(g_init_once, init_registry);
    return (int)g_devs.size();
}
kggml_backend_buffer_type_t ggml_backend_cuda_buffer_type(int device) {
    std::call_once(g_init_once, init_registry);
    if (device < 0 || device >= (int)g_bufts.size()) return nullptr;
    return &g_bufts[device];
}
// one buffer type per split (ggml-cuda.cu:918-955); all zero = an even split
kggml_backend_buffer_type_t ggml_backend_cuda_split_buffer_type(const float *tensor_split) {
    std::call_once(g_init_once, init_registry);
    if (g_devs.empty()) return nullptr;
    const int n = n_lanes();
    std::vector<float> key(n, 0.0f);
    bool zero = true;
    for (int i = 0; i < n; ++i) zero &= !tensor_split || tensor_split[i] == 0.0f;
    for (int i = 0; i < n; ++i) key[i] = zero ? 1.0f : tensor_split[i];
    std::lock_guard<std::mutex> lk(g_split_mu);
    auto it = g_split_bufts.find(key);
    if (it != g_split_bufts.end()) return &it->second;
    SplitBuftCtx *c = new SplitBuftCtx{};
    c->n = n;
    for (int i = 0; i < n; ++i) c->split[i] = key[i];
    auto r = g_split_bufts.emplace(key, kggml_backend_buffer_type{kSplitBuftIface, &g_devs[0], c});
    return &r.first->second;
}
kggml_backend_buffer_type_t ggml_backend_cuda_host_buffer_type(void) {
    std::call_once(g_init_once, init_registry);
    return &g_host_buft;
}
kggml_backend_t ggml_backend_cuda_init(int device) {
    std::call_once(g_init_once, init_registry);
    if (device < 0 || device >= (int)g_devs.size()) { set_err("ggml_backend_cuda_init: invalid device"); return nullptr; }
    hipSetDevice(device);
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) { set_err("stream create failed"); return nullptr; }
    BackendCtx *c = new BackendCtx{device, KGGML_CUDA_NAME + std::to_string(device), s};
    c->fa_exact = getenv("KCPP_FA_EXACT") && atoi(getenv("KCPP_FA_EXACT")) != 0;
    return new kggml_backend{&g_guid, kBackendIface, &g_devs[device], c};
}
bool ggml_backend_is_cuda(kggml_backend_t be) {
    return be != nullptr && be->guid != nullptr && memcmp(*be->guid, g_guid, sizeof(kggml_guid)) == 0;
}
void ggml_backend_cuda_get_device_description(int device, char *description, size_t description_size) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { (void)hipGetLastError(); snprintf(description, description_size, "?"); return; }
    snprintf(description, description_size, "%s", prop.name);
}
void ggml_backend_cuda_get_device_memory(int device, size_t *free, size_t *total) {
    hipSetDevice(device);
    hipMemGetInfo(free, total);
}
// ggml-cuda.cu: opt-in through GGML_CUDA_REGISTER_HOST, as the reference
bool ggml_backend_cuda_register_host_buffer(void *buffer, size_t size) {
    if (getenv("GGML_CUDA_REGISTER_HOST") == nullptr) return false;
    if (hipHostRegister(buffer, size, hipHostRegisterPortable | hipHostRegisterReadOnly) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}
void ggml_backend_cuda_unregister_host_buffer(void *buffer) {
    if (getenv("GGML_CUDA_REGISTER_HOST") == nullptr) return;
    if (hipHostUnregister(buffer) != hipSuccess) (void)hipGetLastError();
}
// koboldcpp: MMQ (integer tiles) vs the hipBLAS dequantize+GEMM route.  Here every quantized mat-mul runs on the
// exact-integer MFMA GEMM, which is the MMQ numerics; the switch is recorded and has no other effect.
void ggml_cuda_set_mul_mat_q(bool mul_mat_q) { g_mul_mat_q = mul_mat_q; }

int kcpp_ggml_backend_last_nodes(void) { return g_last_nodes; }
int kcpp_ggml_backend_last_fused(void) { return g_last_fused; }
int kcpp_ggml_backend_last_fused_launches(void) { return g_last_fused_launches; }
// device bytes held by separate native images (weights outside weight buffers, or asked for in two layouts); the
// weights of a weight buffer are converted in place and hold none
int64_t kcpp_ggml_backend_image_bytes(void) {
    std::lock_guard<std::mutex> lk(g_img_mu);
    int64_t n = 0;
    for (const auto &kv : g_images) n += (int64_t)row_size(std::get<2>(kv.first), std::get<3>(kv.first)) * std::get<4>(kv.first);
    return n;
}
int kcpp_ggml_backend_set_fa_exact(kggml_backend_t be, int on) {
    if (!ggml_backend_is_cuda(be)) return -1;
    ((BackendCtx *)be->context)->fa_exact = on != 0;
    return 0;
}
int kcpp_ggml_backend_set_fusion(kggml_backend_t be, int on) {
    if (!ggml_backend_is_cuda(be)) return -1;
    ((BackendCtx *)be->context)->no_fuse = on == 0;
    return 0;
}
const char *kcpp_ggml_backend_last_error(void) { return g_last_error.c_str(); }

}  // extern "C"
