/*
 * kcpp_expose.h -- the koboldcpp drop-in C ABI exported by koboldcpp_amd/koboldcpp_hipblas.so.
 *
 * Mirrors the reference's expose.h (reference: expose.h:4-175, expose.cpp:23-298) field for field, so the
 * ctypes structures of koboldcpp.py (koboldcpp.py:95-230) bind unchanged: same member order, same C types
 * (bool = 1 byte, enums = int, fixed arrays inline).  Semantics follow gpttype_adapter.cpp where noted.
 * Every function returns a status instead of throwing; strings returned point at library-owned storage that
 * stays valid until the next call of the same function (the reference's rule, gpttype_adapter.cpp:3529-3532).
 */
#ifndef KCPP_EXPOSE_H
#define KCPP_EXPOSE_H
#include <stdbool.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define KCPP_STOP_TOKEN_MAX 32      /* expose.h:4  stop_token_max */
#define KCPP_BAN_TOKEN_MAX 48       /* expose.h:5  ban_token_max */
#define KCPP_TENSOR_SPLIT_MAX 16    /* expose.h:6  tensor_split_max */
#define KCPP_LOGIT_BIAS_MAX 32      /* expose.h:7  logit_bias_max */
#define KCPP_DRY_SEQ_BREAK_MAX 24   /* expose.h:8  dry_seq_break_max */
#define KCPP_IMAGES_MAX 4           /* expose.h:9  images_max */
#define KCPP_SAMPLER_MAX 7          /* expose.h:12-22 enum samplers */

enum kcpp_stop_reason { KCPP_STOP_INVALID = -1, KCPP_STOP_OUT_OF_TOKENS = 0, KCPP_STOP_EOS_TOKEN_HIT = 1,
                        KCPP_STOP_CUSTOM_STOPPER = 2 };   /* expose.h:23-29 */

typedef struct logit_bias { int32_t token_id; float bias; } logit_bias;

typedef struct load_model_inputs {          /* expose.h:34-64 */
    int threads;
    int blasthreads;
    int max_context_length;
    bool low_vram;
    bool use_mmq;
    bool use_rowsplit;
    const char *executable_path;
    const char *model_filename;
    const char *lora_filename;
    const char *lora_base;
    const char *mmproj_filename;
    bool use_mmap;
    bool use_mlock;
    bool use_smartcontext;
    bool use_contextshift;
    int clblast_info;
    int cublas_info;
    const char *vulkan_info;
    int blasbatchsize;
    int debugmode;
    int forceversion;
    int gpulayers;
    float rope_freq_scale;
    float rope_freq_base;
    bool flash_attention;
    float tensor_split[KCPP_TENSOR_SPLIT_MAX];
    int quant_k;
    int quant_v;
} load_model_inputs;

typedef struct generation_inputs {          /* expose.h:65-115 */
    int seed;
    const char *prompt;
    const char *memory;
    const char *images[KCPP_IMAGES_MAX];
    int max_context_length;
    int max_length;
    float temperature;
    int top_k;
    float top_a;
    float top_p;
    float min_p;
    float typical_p;
    float tfs;
    float rep_pen;
    int rep_pen_range;
    float rep_pen_slope;
    float presence_penalty;
    int mirostat;
    float mirostat_eta;
    float mirostat_tau;
    float dry_multiplier;
    float dry_base;
    int dry_allowed_length;
    int dry_penalty_last_n;
    const char *dry_sequence_breakers[KCPP_DRY_SEQ_BREAK_MAX];
    float xtc_threshold;
    float xtc_probability;
    int sampler_order[KCPP_SAMPLER_MAX];     /* enum samplers */
    int sampler_len;
    bool allow_eos_token;
    bool bypass_eos_token;
    bool render_special;
    const char *stop_sequence[KCPP_STOP_TOKEN_MAX];
    bool stream_sse;
    const char *grammar;
    bool grammar_retain_state;
    bool quiet;
    float dynatemp_range;
    float dynatemp_exponent;
    float smoothing_factor;
    logit_bias logit_biases[KCPP_LOGIT_BIAS_MAX];
    const char *banned_tokens[KCPP_BAN_TOKEN_MAX];
} generation_inputs;

typedef struct generation_outputs { int status; int stopreason; const char *text; } generation_outputs;
typedef struct token_count_outputs { int count; int *ids; } token_count_outputs;

typedef struct sd_load_model_inputs {       /* expose.h:121-135 (image generation: not provided here) */
    const char *model_filename; const char *executable_path; int clblast_info; int cublas_info;
    const char *vulkan_info; int threads; int quant; bool taesd; const char *vae_filename;
    const char *lora_filename; float lora_multiplier; int debugmode;
} sd_load_model_inputs;
typedef struct sd_generation_inputs {
    const char *prompt; const char *negative_prompt; const char *init_images; float denoising_strength;
    float cfg_scale; int sample_steps; int width; int height; int seed; const char *sample_method; int clip_skip;
    bool quiet;
} sd_generation_inputs;
typedef struct sd_generation_outputs { int status; const char *data; } sd_generation_outputs;
typedef struct whisper_load_model_inputs {
    const char *model_filename; const char *executable_path; int clblast_info; int cublas_info;
    const char *vulkan_info; int debugmode;
} whisper_load_model_inputs;
typedef struct whisper_generation_inputs { const char *prompt; const char *audio_data; bool quiet; } whisper_generation_inputs;
typedef struct whisper_generation_outputs { int status; const char *text; } whisper_generation_outputs;

/* text generation (expose.cpp:32-220): GGUF Llama-architecture models on the MI355X runtime */
bool load_model(const load_model_inputs inputs);
generation_outputs generate(const generation_inputs inputs);
/* streaming / status polls (expose.cpp:240-295) */
const char *new_token(int idx);
int get_stream_count(void);
bool has_finished(void);
float get_last_eval_time(void);      /* ms per generated token */
float get_last_process_time(void);   /* ms per prompt token */
int get_last_token_count(void);
int get_last_seed(void);
int get_total_gens(void);
int get_total_img_gens(void);
int get_last_stop_reason(void);
const char *get_pending_output(void);
bool abort_generate(void);
token_count_outputs token_count(const char *input, bool addbos);
/* present so koboldcpp.py's symbol lookups succeed; they report failure (out of scope here) */
bool sd_load_model(const sd_load_model_inputs inputs);
sd_generation_outputs sd_generate(const sd_generation_inputs inputs);
bool whisper_load_model(const whisper_load_model_inputs inputs);
whisper_generation_outputs whisper_generate(const whisper_generation_inputs inputs);

#ifdef __cplusplus
}
#endif
#endif
