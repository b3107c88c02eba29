"""ctypes mirror of the koboldcpp C ABI (include/kcpp_expose.h), laid out exactly like koboldcpp.py's
own structures (reference koboldcpp.py:95-230) so the same calls work against koboldcpp_hipblas.so.
This is what koboldcpp.py's `init_library()` binds (koboldcpp.py:415-441); INTEGRATION.md shows the
handful of lines it needs."""
import ctypes

from . import LIB_PATH

STOP_TOKEN_MAX, BAN_TOKEN_MAX, TENSOR_SPLIT_MAX, LOGIT_BIAS_MAX, DRY_SEQ_BREAK_MAX, IMAGES_MAX, SAMPLER_MAX = \
    32, 48, 16, 32, 24, 4, 7
c_char_p, c_int, c_float, c_bool = ctypes.c_char_p, ctypes.c_int, ctypes.c_float, ctypes.c_bool


class logit_bias(ctypes.Structure):
    _fields_ = [("token_id", ctypes.c_int32), ("bias", c_float)]


class load_model_inputs(ctypes.Structure):
    _fields_ = [("threads", c_int), ("blasthreads", c_int), ("max_context_length", c_int), ("low_vram", c_bool),
                ("use_mmq", c_bool), ("use_rowsplit", c_bool), ("executable_path", c_char_p),
                ("model_filename", c_char_p), ("lora_filename", c_char_p), ("lora_base", c_char_p),
                ("mmproj_filename", c_char_p), ("use_mmap", c_bool), ("use_mlock", c_bool),
                ("use_smartcontext", c_bool), ("use_contextshift", c_bool), ("clblast_info", c_int),
                ("cublas_info", c_int), ("vulkan_info", c_char_p), ("blasbatchsize", c_int), ("debugmode", c_int),
                ("forceversion", c_int), ("gpulayers", c_int), ("rope_freq_scale", c_float),
                ("rope_freq_base", c_float), ("flash_attention", c_bool),
                ("tensor_split", c_float * TENSOR_SPLIT_MAX), ("quant_k", c_int), ("quant_v", c_int)]


class generation_inputs(ctypes.Structure):
    _fields_ = [("seed", c_int), ("prompt", c_char_p), ("memory", c_char_p), ("images", c_char_p * IMAGES_MAX),
                ("max_context_length", c_int), ("max_length", c_int), ("temperature", c_float), ("top_k", c_int),
                ("top_a", c_float), ("top_p", c_float), ("min_p", c_float), ("typical_p", c_float), ("tfs", c_float),
                ("rep_pen", c_float), ("rep_pen_range", c_int), ("rep_pen_slope", c_float),
                ("presence_penalty", c_float), ("mirostat", c_int), ("mirostat_eta", c_float),
                ("mirostat_tau", c_float), ("dry_multiplier", c_float), ("dry_base", c_float),
                ("dry_allowed_length", c_int), ("dry_penalty_last_n", c_int),
                ("dry_sequence_breakers", c_char_p * DRY_SEQ_BREAK_MAX), ("xtc_threshold", c_float),
                ("xtc_probability", c_float), ("sampler_order", c_int * SAMPLER_MAX), ("sampler_len", c_int),
                ("allow_eos_token", c_bool), ("bypass_eos_token", c_bool), ("render_special", c_bool),
                ("stop_sequence", c_char_p * STOP_TOKEN_MAX), ("stream_sse", c_bool), ("grammar", c_char_p),
                ("grammar_retain_state", c_bool), ("quiet", c_bool), ("dynatemp_range", c_float),
                ("dynatemp_exponent", c_float), ("smoothing_factor", c_float),
                ("logit_biases", logit_bias * LOGIT_BIAS_MAX), ("banned_tokens", c_char_p * BAN_TOKEN_MAX)]


class generation_outputs(ctypes.Structure):
    _fields_ = [("status", c_int), ("stopreason", c_int), ("text", c_char_p)]


class token_count_outputs(ctypes.Structure):
    _fields_ = [("count", c_int), ("ids", ctypes.POINTER(c_int))]


def init_library(path=LIB_PATH):
    """the binding list of koboldcpp.py:415-441 against this library"""
    h = ctypes.CDLL(path)
    h.load_model.argtypes = [load_model_inputs]
    h.load_model.restype = c_bool
    h.generate.argtypes = [generation_inputs]
    h.generate.restype = generation_outputs
    h.new_token.restype = c_char_p
    h.new_token.argtypes = [c_int]
    h.get_stream_count.restype = c_int
    h.has_finished.restype = c_bool
    h.get_last_eval_time.restype = c_float
    h.get_last_process_time.restype = c_float
    h.get_last_token_count.restype = c_int
    h.get_last_seed.restype = c_int
    h.get_total_gens.restype = c_int
    h.get_last_stop_reason.restype = c_int
    h.abort_generate.restype = c_bool
    h.token_count.restype = token_count_outputs
    h.token_count.argtypes = [c_char_p, c_bool]
    h.get_pending_output.restype = c_char_p
    return h
