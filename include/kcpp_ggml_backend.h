/* kcpp_ggml_backend.h -- the ggml backend plugin boundary, restated.
 *
 * koboldcpp's llama.cpp reaches its GPU through the ggml-backend interface: a registry entry
 * (ggml_backend_cuda_reg, reference ggml/src/ggml-cuda.cu:3302) that hands out devices, backends (streams),
 * buffer types and buffers as C structs of function pointers, and graph_compute(backend, ggml_cgraph *).
 * This header restates exactly the types that cross that boundary -- ggml_tensor, ggml_cgraph and the five
 * vtable structs of ggml-backend-impl.h -- so this library can implement them without compiling against the
 * reference's headers.  Member order and types follow the reference (file:line on each); the layout is checked
 * against the reference build at run time by tests/test_ggml_backend_layout.py (tensors, graphs, backends, buffer
 * types, buffers, devices and registries created by oracle/_ref/libggml_ref.so are read through these
 * declarations).  The implementation is koboldcpp_amd/csrc/ggml_backend.cpp.
 *
 * Everything here is plain C: pointers, sizes, enums.  No torch or HIP types.
 */
#ifndef KCPP_GGML_BACKEND_H
#define KCPP_GGML_BACKEND_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ggml/include/ggml.h:218-227 */
#define KGGML_MAX_DIMS 4
#define KGGML_MAX_SRC 10
#define KGGML_MAX_OP_PARAMS 64
#define KGGML_MAX_NAME 128
/* ggml/include/ggml-cuda.h:10-20 (GGML_USE_HIPBLAS build) */
#define KGGML_CUDA_NAME "ROCm"
#define KGGML_CUDA_MAX_DEVICES 16

/* ggml/include/ggml.h:362-400 (ids used by the Llama path; the enum is the ggml one) */
enum kggml_type {
    KGGML_TYPE_F32 = 0, KGGML_TYPE_F16 = 1, KGGML_TYPE_Q4_0 = 2, KGGML_TYPE_Q4_1 = 3, KGGML_TYPE_Q5_0 = 6,
    KGGML_TYPE_Q5_1 = 7, KGGML_TYPE_Q8_0 = 8, KGGML_TYPE_Q8_1 = 9, KGGML_TYPE_Q2_K = 10, KGGML_TYPE_Q3_K = 11,
    KGGML_TYPE_Q4_K = 12, KGGML_TYPE_Q5_K = 13, KGGML_TYPE_Q6_K = 14, KGGML_TYPE_Q8_K = 15, KGGML_TYPE_I8 = 24,
    KGGML_TYPE_I16 = 25, KGGML_TYPE_I32 = 26, KGGML_TYPE_I64 = 27, KGGML_TYPE_F64 = 28, KGGML_TYPE_BF16 = 30,
    KGGML_TYPE_COUNT = 36
};

/* ggml/include/ggml.h:446-540 enum ggml_op (positional; the values this backend dispatches on) */
enum kggml_op {
    KGGML_OP_NONE = 0, KGGML_OP_DUP = 1, KGGML_OP_ADD = 2, KGGML_OP_ADD1 = 3, KGGML_OP_ACC = 4, KGGML_OP_SUB = 5,
    KGGML_OP_MUL = 6, KGGML_OP_DIV = 7, KGGML_OP_SUM_ROWS = 14, KGGML_OP_RMS_NORM = 23, KGGML_OP_MUL_MAT = 26,
    KGGML_OP_MUL_MAT_ID = 27, KGGML_OP_SCALE = 29, KGGML_OP_CPY = 31, KGGML_OP_CONT = 32, KGGML_OP_RESHAPE = 33,
    KGGML_OP_VIEW = 34, KGGML_OP_PERMUTE = 35, KGGML_OP_TRANSPOSE = 36, KGGML_OP_GET_ROWS = 37,
    KGGML_OP_SOFT_MAX = 42, KGGML_OP_ROPE = 44, KGGML_OP_ARGSORT = 58, KGGML_OP_FLASH_ATTN_EXT = 60,
    KGGML_OP_UNARY = 69
};
/* ggml/include/ggml.h:541-558 */
enum kggml_unary_op {
    KGGML_UNARY_OP_ABS = 0, KGGML_UNARY_OP_NEG = 2, KGGML_UNARY_OP_RELU = 6, KGGML_UNARY_OP_SILU = 10
};
/* ggml/include/ggml.h:331-336 */
enum kggml_status { KGGML_STATUS_ALLOC_FAILED = -2, KGGML_STATUS_FAILED = -1, KGGML_STATUS_SUCCESS = 0 };
/* ggml/include/ggml-backend.h:35-39 */
enum kggml_backend_buffer_usage {
    KGGML_BACKEND_BUFFER_USAGE_ANY = 0, KGGML_BACKEND_BUFFER_USAGE_WEIGHTS = 1, KGGML_BACKEND_BUFFER_USAGE_COMPUTE = 2
};
/* ggml/include/ggml-backend.h:116-122 */
enum kggml_backend_dev_type {
    KGGML_BACKEND_DEVICE_TYPE_CPU, KGGML_BACKEND_DEVICE_TYPE_GPU, KGGML_BACKEND_DEVICE_TYPE_CPU_FULL,
    KGGML_BACKEND_DEVICE_TYPE_GPU_FULL
};

struct kggml_backend_buffer;
struct kggml_backend_buffer_type;
struct kggml_backend;
struct kggml_backend_device;
struct kggml_backend_reg;
struct kggml_backend_event;

/* ggml/include/ggml.h:584-620 struct ggml_tensor */
struct kggml_tensor {
    int type;                                   /* enum ggml_type */
    int backend;                                /* deprecated enum ggml_backend_type */
    struct kggml_backend_buffer *buffer;
    int64_t ne[KGGML_MAX_DIMS];
    size_t nb[KGGML_MAX_DIMS];
    int op;                                     /* enum ggml_op */
    int32_t op_params[KGGML_MAX_OP_PARAMS / sizeof(int32_t)];
    int32_t flags;
    struct kggml_tensor *grad;
    struct kggml_tensor *src[KGGML_MAX_SRC];
    struct kggml_tensor *view_src;
    size_t view_offs;
    void *data;
    char name[KGGML_MAX_NAME];
    void *extra;
};

/* ggml/src/ggml-impl.h:80-84, 183-195 */
struct kggml_hash_set {
    size_t size;
    uint32_t *used;
    struct kggml_tensor **keys;
};
struct kggml_cgraph {
    int size;
    int n_nodes;
    int n_leafs;
    struct kggml_tensor **nodes;
    struct kggml_tensor **grads;
    struct kggml_tensor **leafs;
    struct kggml_hash_set visited_hash_set;
    int order;                                  /* enum ggml_cgraph_eval_order */
};

typedef struct kggml_backend_buffer_type *kggml_backend_buffer_type_t;
typedef struct kggml_backend_buffer *kggml_backend_buffer_t;
typedef struct kggml_backend *kggml_backend_t;
typedef struct kggml_backend_device *kggml_backend_dev_t;
typedef struct kggml_backend_reg *kggml_backend_reg_t;
typedef struct kggml_backend_event *kggml_backend_event_t;
typedef void *kggml_backend_graph_plan_t;
typedef uint8_t kggml_guid[16];                 /* ggml/include/ggml.h:694 */

/* ggml/src/ggml-backend-impl.h:15-33 */
struct kggml_backend_buffer_type_i {
    const char *(*get_name)(kggml_backend_buffer_type_t buft);
    kggml_backend_buffer_t (*alloc_buffer)(kggml_backend_buffer_type_t buft, size_t size);
    size_t (*get_alignment)(kggml_backend_buffer_type_t buft);
    size_t (*get_max_size)(kggml_backend_buffer_type_t buft);
    size_t (*get_alloc_size)(kggml_backend_buffer_type_t buft, const struct kggml_tensor *tensor);
    bool (*is_host)(kggml_backend_buffer_type_t buft);
};
struct kggml_backend_buffer_type {
    struct kggml_backend_buffer_type_i iface;
    kggml_backend_dev_t device;
    void *context;
};

/* ggml/src/ggml-backend-impl.h:39-66 */
struct kggml_backend_buffer_i {
    const char *(*get_name)(kggml_backend_buffer_t buffer);
    void (*free_buffer)(kggml_backend_buffer_t buffer);
    void *(*get_base)(kggml_backend_buffer_t buffer);
    void (*init_tensor)(kggml_backend_buffer_t buffer, struct kggml_tensor *tensor);
    void (*memset_tensor)(kggml_backend_buffer_t buffer, struct kggml_tensor *tensor, uint8_t value, size_t offset,
                          size_t size);
    void (*set_tensor)(kggml_backend_buffer_t buffer, struct kggml_tensor *tensor, const void *data, size_t offset,
                       size_t size);
    void (*get_tensor)(kggml_backend_buffer_t buffer, const struct kggml_tensor *tensor, void *data, size_t offset,
                       size_t size);
    bool (*cpy_tensor)(kggml_backend_buffer_t buffer, const struct kggml_tensor *src, struct kggml_tensor *dst);
    void (*clear)(kggml_backend_buffer_t buffer, uint8_t value);
    void (*reset)(kggml_backend_buffer_t buffer);
};
struct kggml_backend_buffer {
    struct kggml_backend_buffer_i iface;
    kggml_backend_buffer_type_t buft;
    void *context;
    size_t size;
    int usage;                                  /* enum ggml_backend_buffer_usage */
};

/* ggml/src/ggml-backend-impl.h:86-134 */
struct kggml_backend_i {
    const char *(*get_name)(kggml_backend_t backend);
    void (*free)(kggml_backend_t backend);
    kggml_backend_buffer_type_t (*get_default_buffer_type)(kggml_backend_t backend);
    void (*set_tensor_async)(kggml_backend_t backend, struct kggml_tensor *tensor, const void *data, size_t offset,
                             size_t size);
    void (*get_tensor_async)(kggml_backend_t backend, const struct kggml_tensor *tensor, void *data, size_t offset,
                             size_t size);
    bool (*cpy_tensor_async)(kggml_backend_t backend_src, kggml_backend_t backend_dst, const struct kggml_tensor *src,
                             struct kggml_tensor *dst);
    void (*synchronize)(kggml_backend_t backend);
    kggml_backend_graph_plan_t (*graph_plan_create)(kggml_backend_t backend, const struct kggml_cgraph *cgraph);
    void (*graph_plan_free)(kggml_backend_t backend, kggml_backend_graph_plan_t plan);
    void (*graph_plan_update)(kggml_backend_t backend, kggml_backend_graph_plan_t plan, const struct kggml_cgraph *cgraph);
    int (*graph_plan_compute)(kggml_backend_t backend, kggml_backend_graph_plan_t plan);
    int (*graph_compute)(kggml_backend_t backend, struct kggml_cgraph *cgraph);   /* enum ggml_status */
    bool (*supports_op)(kggml_backend_t backend, const struct kggml_tensor *op);
    bool (*supports_buft)(kggml_backend_t backend, kggml_backend_buffer_type_t buft);
    bool (*offload_op)(kggml_backend_t backend, const struct kggml_tensor *op);
    void (*event_record)(kggml_backend_t backend, kggml_backend_event_t event);
    void (*event_wait)(kggml_backend_t backend, kggml_backend_event_t event);
};
struct kggml_backend {
    kggml_guid *guid;                           /* ggml_guid_t */
    struct kggml_backend_i iface;
    kggml_backend_dev_t device;
    void *context;
};
struct kggml_backend_event {
    struct kggml_backend_device *device;
    void *context;
};

/* ggml/include/ggml-backend.h:125-144 */
struct kggml_backend_dev_caps {
    bool async;
    bool host_buffer;
    bool buffer_from_host_ptr;
    bool events;
};
struct kggml_backend_dev_props {
    const char *name;
    const char *description;
    size_t memory_free;
    size_t memory_total;
    int type;                                   /* enum ggml_backend_dev_type */
    struct kggml_backend_dev_caps caps;
};

/* ggml/src/ggml-backend-impl.h:146-193 */
struct kggml_backend_device_i {
    const char *(*get_name)(kggml_backend_dev_t dev);
    const char *(*get_description)(kggml_backend_dev_t dev);
    void (*get_memory)(kggml_backend_dev_t dev, size_t *free, size_t *total);
    int (*get_type)(kggml_backend_dev_t dev);
    void (*get_props)(kggml_backend_dev_t dev, struct kggml_backend_dev_props *props);
    kggml_backend_t (*init_backend)(kggml_backend_dev_t dev, const char *params);
    kggml_backend_buffer_type_t (*get_buffer_type)(kggml_backend_dev_t dev);
    kggml_backend_buffer_type_t (*get_host_buffer_type)(kggml_backend_dev_t dev);
    kggml_backend_buffer_t (*buffer_from_host_ptr)(kggml_backend_dev_t dev, void *ptr, size_t size, size_t max_tensor_size);
    bool (*supports_op)(kggml_backend_dev_t dev, const struct kggml_tensor *op);
    bool (*supports_buft)(kggml_backend_dev_t dev, kggml_backend_buffer_type_t buft);
    bool (*offload_op)(kggml_backend_dev_t dev, const struct kggml_tensor *op);
    kggml_backend_event_t (*event_new)(kggml_backend_dev_t dev);
    void (*event_free)(kggml_backend_dev_t dev, kggml_backend_event_t event);
    void (*event_synchronize)(kggml_backend_dev_t dev, kggml_backend_event_t event);
};
struct kggml_backend_device {
    struct kggml_backend_device_i iface;
    kggml_backend_reg_t reg;
    void *context;
};

/* ggml/src/ggml-backend-impl.h:195-210 */
struct kggml_backend_reg_i {
    const char *(*get_name)(kggml_backend_reg_t reg);
    size_t (*get_device_count)(kggml_backend_reg_t reg);
    kggml_backend_dev_t (*get_device)(kggml_backend_reg_t reg, size_t index);
    void *(*get_proc_address)(kggml_backend_reg_t reg, const char *name);
};
struct kggml_backend_reg {
    struct kggml_backend_reg_i iface;
    void *context;
};

/* ---- exported entry points: the public API of ggml/include/ggml-cuda.h:22-44 under their reference names,
 * plus koboldcpp's ggml_cuda_set_mul_mat_q (gpttype_adapter.cpp:1883) */
kggml_backend_reg_t ggml_backend_cuda_reg(void);
kggml_backend_t ggml_backend_cuda_init(int device);
bool ggml_backend_is_cuda(kggml_backend_t backend);
kggml_backend_buffer_type_t ggml_backend_cuda_buffer_type(int device);
/* row split across devices (ggml-cuda.cu:625-955, LLAMA_SPLIT_MODE_ROW): one buffer type per tensor_split (all
 * zero or NULL = an even split); each weight's rows are spread over the devices, already in the device layout of
 * its type, and a MUL_MAT on it runs on the main device with every other device multiplying its own rows
 * (ggml_backend.cpp, "split buffers").  NULL only when no device is present. */
kggml_backend_buffer_type_t ggml_backend_cuda_split_buffer_type(const float *tensor_split);
kggml_backend_buffer_type_t ggml_backend_cuda_host_buffer_type(void);
int ggml_backend_cuda_get_device_count(void);
void ggml_backend_cuda_get_device_description(int device, char *description, size_t description_size);
void ggml_backend_cuda_get_device_memory(int device, size_t *free, size_t *total);
bool ggml_backend_cuda_register_host_buffer(void *buffer, size_t size);
void ggml_backend_cuda_unregister_host_buffer(void *buffer);
void ggml_cuda_set_mul_mat_q(bool mul_mat_q);

/* diagnostics (this backend only): nodes executed by the last graph_compute, and the last dispatch error */
int kcpp_ggml_backend_last_nodes(void);
/* of those, the nodes that ran inside a fused launch (RMS_NORM+MUL, MUL_MAT+ADD, the SiLU GLU; 0 with KCPP_B1_UNFUSED=1) */
int kcpp_ggml_backend_last_fused(void);
/* and the number of fused launches they ran as */
int kcpp_ggml_backend_last_fused_launches(void);
/* device bytes held in separate native weight images (0 when every weight sits in a weight buffer: those are
 * converted in place, one copy of the model) */
int64_t kcpp_ggml_backend_image_bytes(void);
/* strict-parity attention for this backend's FLASH_ATTN_EXT nodes (default from KCPP_FA_EXACT at init) */
int kcpp_ggml_backend_set_fa_exact(kggml_backend_t backend, int on);
/* node fusion (RMS_NORM+MUL, MUL_MAT+ADD, the SiLU GLU at one token) on / off for this backend (default on; off with
 * KCPP_B1_UNFUSED=1 or KCPP_B1_NOFUSE=1 at init) */
int kcpp_ggml_backend_set_fusion(kggml_backend_t backend, int on);
const char *kcpp_ggml_backend_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
