"""GGUF parse robustness of load_model (csrc/gguf.h) on the host: a truncated file, a tensor whose data runs past
the end of the file, a zero or non-power-of-two general.alignment and an unknown tensor type must make
load_model() return false before any device work (the reference checks offset + size against the file,
src/llama.cpp:4379-4390).  No GPU needed: the parser rejects these files before the first HIP call."""
import os

import numpy as np
import pytest

import gguf_writer as GW

Q4_K = 12


def _tiny(path, align=32, extra_kv=None, t_type=Q4_K):
    kv = {"general.architecture": "llama", "general.alignment": align, "llama.block_count": 1,
          "llama.embedding_length": 256, "tokenizer.ggml.model": "llama",
          "tokenizer.ggml.tokens": (GW.STR, ["<unk>", "<s>", "</s>", "a"]),
          "tokenizer.ggml.scores": (GW.F32, [0.0] * 4), "tokenizer.ggml.token_type": (GW.I32, [2, 3, 3, 1])}
    kv.update(extra_kv or {})
    data = np.zeros(144 * 4, dtype=np.uint8).tobytes()                 # 4 rows of one Q4_K block
    GW.write(path, kv, [("token_embd.weight", t_type, [256, 4], data)], align=align if align > 0 else 32)


def _check(path):
    import ctypes
    import koboldcpp_amd.lib as K
    buf = ctypes.create_string_buffer(512)
    rc = K.raw().kcpp_gguf_check(path.encode(), buf, 512)
    return rc, buf.value.decode()


def _load(path):
    from koboldcpp_amd import expose as X
    h = X.init_library()
    li = X.load_model_inputs()
    li.model_filename = path.encode()
    li.max_context_length = 64
    return h.load_model(li)


def test_intact_file_parses(tmp_path):
    p = str(tmp_path / "ok.gguf")
    _tiny(p)
    assert _check(p) == (0, "")


@pytest.mark.parametrize("cut", [1, 100, 400])
def test_truncated_gguf_is_rejected(tmp_path, cut):
    p = str(tmp_path / "t.gguf")
    _tiny(p)
    sz = os.path.getsize(p)
    with open(p, "r+b") as f:
        f.truncate(sz - cut)
    rc, err = _check(p)
    assert rc == -1 and "past end of file" in err, err
    assert not _load(p)


def test_zero_alignment_is_rejected(tmp_path):
    p = str(tmp_path / "a0.gguf")
    _tiny(p, align=0)
    rc, err = _check(p)
    assert rc == -1 and "alignment" in err, err


def test_non_power_of_two_alignment_is_rejected(tmp_path):
    p = str(tmp_path / "a24.gguf")
    _tiny(p, align=24)
    rc, err = _check(p)
    assert rc == -1 and "alignment" in err, err


def test_unknown_tensor_type_is_rejected(tmp_path):
    p = str(tmp_path / "ty.gguf")
    _tiny(p, t_type=4)                                                  # Q4_2: removed from ggml
    rc, err = _check(p)
    assert rc == -1 and "unknown tensor type" in err, err
