"""The koboldcpp C-ABI structs in include/kcpp_expose.h must have the exact layout of the reference's
expose.h (koboldcpp.py's ctypes mirror binds against that): every member's offset and every struct's
size are compared between a C++ translation unit compiled from the reference header (in this
container only -- /root/reference does not exist on the GPU box, so the test skips there) and a C
unit compiled from ours."""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_H = "/root/reference/expose.h"

FIELDS = {
    "load_model_inputs": ["threads", "blasthreads", "max_context_length", "low_vram", "use_mmq", "use_rowsplit",
                          "executable_path", "model_filename", "lora_filename", "lora_base", "mmproj_filename",
                          "use_mmap", "use_mlock", "use_smartcontext", "use_contextshift", "clblast_info",
                          "cublas_info", "vulkan_info", "blasbatchsize", "debugmode", "forceversion", "gpulayers",
                          "rope_freq_scale", "rope_freq_base", "flash_attention", "tensor_split", "quant_k", "quant_v"],
    "generation_inputs": ["seed", "prompt", "memory", "images", "max_context_length", "max_length", "temperature",
                          "top_k", "top_a", "top_p", "min_p", "typical_p", "tfs", "rep_pen", "rep_pen_range",
                          "rep_pen_slope", "presence_penalty", "mirostat", "mirostat_eta", "mirostat_tau",
                          "dry_multiplier", "dry_base", "dry_allowed_length", "dry_penalty_last_n",
                          "dry_sequence_breakers", "xtc_threshold", "xtc_probability", "sampler_order", "sampler_len",
                          "allow_eos_token", "bypass_eos_token", "render_special", "stop_sequence", "stream_sse",
                          "grammar", "grammar_retain_state", "quiet", "dynatemp_range", "dynatemp_exponent",
                          "smoothing_factor", "logit_biases", "banned_tokens"],
    "generation_outputs": ["status", "stopreason", "text"],
    "token_count_outputs": ["count", "ids"],
    "sd_load_model_inputs": ["model_filename", "executable_path", "clblast_info", "cublas_info", "vulkan_info",
                             "threads", "quant", "taesd", "vae_filename", "lora_filename", "lora_multiplier",
                             "debugmode"],
    "sd_generation_inputs": ["prompt", "negative_prompt", "init_images", "denoising_strength", "cfg_scale",
                             "sample_steps", "width", "height", "seed", "sample_method", "clip_skip", "quiet"],
    "sd_generation_outputs": ["status", "data"],
    "whisper_load_model_inputs": ["model_filename", "executable_path", "clblast_info", "cublas_info",
                                  "vulkan_info", "debugmode"],
    "whisper_generation_inputs": ["prompt", "audio_data", "quiet"],
    "whisper_generation_outputs": ["status", "text"],
}


def _probe(src, lang, incl):
    lines = ["#include <stdio.h>", "#include <stddef.h>"] + incl + ["int main(void) {"]
    for st, fs in FIELDS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (st, st if lang == "c" else "struct " + st))
        for f in fs:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (st, f, st if lang == "c" else "struct " + st, f))
    lines.append("return 0; }")
    d = tempfile.mkdtemp()
    cfile = os.path.join(d, "p." + ("c" if lang == "c" else "cpp"))
    open(cfile, "w").write("\n".join(lines))
    exe = os.path.join(d, "p")
    cc = ["gcc", "-std=c11"] if lang == "c" else ["g++", "-std=c++17", "-include", "string", "-include", "vector"]
    subprocess.run(cc + ["-I", os.path.join(ROOT, "include"), cfile, "-o", exe], check=True, capture_output=True)
    return subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split("\n")


@pytest.mark.skipif(not os.path.exists(REF_H), reason="reference headers only exist in the build container")
def test_expose_struct_layout_matches_reference():
    ours = _probe(None, "c", ['#include "kcpp_expose.h"'])
    ref = _probe(None, "cpp", ['#include "%s"' % REF_H])
    assert ours == ref
