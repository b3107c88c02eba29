"""The restated ggml-backend boundary types (include/kcpp_ggml_backend.h) against the REFERENCE build.

The plugin implements ggml_tensor / ggml_cgraph readers and the five vtable structs of ggml-backend-impl.h
without compiling against the reference headers.  This test pins those declarations to the reference binary
(oracle/_ref/libggml_ref.so, built from the reference sources by oracle/Makefile): member offsets come from a
C probe compiled against OUR header, and each member is read at that offset out of objects the reference
library itself created and filled -- tensors (shape, strides, op, op_params, flags, sources, view, data, name),
graphs (size, node count, node array), and the CPU backend's backend / device / registry / buffer type / buffer
(function pointers called through our offsets must answer like the reference accessors).  CPU only; skipped
where the reference build is absent (the GPU box)."""
import ctypes
import os
import struct
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFLIB = os.path.join(ROOT, "oracle", "_ref", "libggml_ref.so")
HDR = os.path.join(ROOT, "include", "kcpp_ggml_backend.h")

pytestmark = pytest.mark.skipif(not os.path.exists(REFLIB), reason="reference build (make -C oracle ref) absent")

MEMBERS = {
    "kggml_tensor": ["type", "buffer", "ne", "nb", "op", "op_params", "flags", "grad", "src", "view_src", "view_offs",
                     "data", "name", "extra"],
    "kggml_cgraph": ["size", "n_nodes", "n_leafs", "nodes", "grads", "leafs", "visited_hash_set", "order"],
    "kggml_backend_buffer_type": ["iface", "device", "context"],
    "kggml_backend_buffer_type_i": ["get_name", "alloc_buffer", "get_alignment", "get_max_size", "get_alloc_size",
                                    "is_host"],
    "kggml_backend_buffer": ["iface", "buft", "context", "size", "usage"],
    "kggml_backend_buffer_i": ["get_name", "free_buffer", "get_base", "init_tensor", "memset_tensor", "set_tensor",
                               "get_tensor", "cpy_tensor", "clear", "reset"],
    "kggml_backend": ["guid", "iface", "device", "context"],
    "kggml_backend_i": ["get_name", "free", "get_default_buffer_type", "set_tensor_async", "get_tensor_async",
                        "cpy_tensor_async", "synchronize", "graph_plan_create", "graph_plan_free", "graph_plan_update",
                        "graph_plan_compute", "graph_compute", "supports_op", "supports_buft", "offload_op",
                        "event_record", "event_wait"],
    "kggml_backend_device": ["iface", "reg", "context"],
    "kggml_backend_device_i": ["get_name", "get_description", "get_memory", "get_type", "get_props", "init_backend",
                               "get_buffer_type", "get_host_buffer_type", "buffer_from_host_ptr", "supports_op",
                               "supports_buft", "offload_op", "event_new", "event_free", "event_synchronize"],
    "kggml_backend_reg": ["iface", "context"],
    "kggml_backend_reg_i": ["get_name", "get_device_count", "get_device", "get_proc_address"],
}


@pytest.fixture(scope="module")
def off():
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "%s"' % HDR, "int main(void) {"]
    for st, ms in MEMBERS.items():
        lines.append('printf("%s.sizeof %%zu\\n", sizeof(struct %s));' % (st, st))
        for m in ms:
            lines.append('printf("%s.%s %%zu\\n", offsetof(struct %s, %s));' % (st, m, st, m))
    lines.append("return 0; }")
    d = tempfile.mkdtemp()
    src, exe = os.path.join(d, "p.c"), os.path.join(d, "p")
    open(src, "w").write("\n".join(lines))
    subprocess.run(["gcc", "-std=c11", src, "-o", exe], check=True, capture_output=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return {out[i]: int(out[i + 1]) for i in range(0, len(out), 2)}


class InitParams(ctypes.Structure):
    _fields_ = [("mem_size", ctypes.c_size_t), ("mem_buffer", ctypes.c_void_p), ("no_alloc", ctypes.c_bool)]


@pytest.fixture(scope="module")
def ref():
    L = ctypes.CDLL(REFLIB)
    P, I, I64, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float
    sigs = {"ggml_init": ([InitParams], P), "ggml_free": ([P], None),
            "ggml_new_tensor_2d": ([P, I, I64, I64], P), "ggml_add": ([P, P, P], P), "ggml_scale": ([P, P, F], P),
            "ggml_view_1d": ([P, P, I64, ctypes.c_size_t], P), "ggml_set_name": ([P, ctypes.c_char_p], P),
            "ggml_set_input": ([P], None), "ggml_get_data": ([P], P), "ggml_new_graph": ([P], P),
            "ggml_build_forward_expand": ([P, P], None), "ggml_graph_n_nodes": ([P], I), "ggml_graph_node": ([P, I], P),
            "ggml_graph_size": ([P], I), "ggml_tensor_overhead": ([], ctypes.c_size_t),
            "ggml_backend_cpu_init": ([], P), "ggml_backend_free": ([P], None), "ggml_backend_name": ([P], ctypes.c_char_p),
            "ggml_backend_get_device": ([P], P), "ggml_backend_dev_name": ([P], ctypes.c_char_p),
            "ggml_backend_dev_backend_reg": ([P], P), "ggml_backend_reg_name": ([P], ctypes.c_char_p),
            "ggml_backend_reg_dev_count": ([P], ctypes.c_size_t), "ggml_backend_cpu_buffer_type": ([], P),
            "ggml_backend_buft_name": ([P], ctypes.c_char_p), "ggml_backend_buft_get_alignment": ([P], ctypes.c_size_t),
            "ggml_backend_buft_alloc_buffer": ([P, ctypes.c_size_t], P), "ggml_backend_buffer_get_base": ([P], P), "ggml_backend_buffer_get_size": ([P], ctypes.c_size_t),
            "ggml_backend_buffer_set_usage": ([P, I], None), "ggml_backend_buffer_free": ([P], None),
            "ggml_backend_dev_get_props": ([P, P], None)}
    for n, (a, r) in sigs.items():
        f = getattr(L, n)
        f.argtypes, f.restype = a, r
    L.ggml_init(InitParams(1 << 20, None, False))
    return L


def rd(addr, fmt):
    n = struct.calcsize(fmt)
    return struct.unpack(fmt, ctypes.string_at(addr, n))


def rd_ptr(addr):
    return rd(addr, "Q")[0]


def fnptr(addr, restype, *argtypes):
    return ctypes.CFUNCTYPE(restype, *argtypes)(rd_ptr(addr))


def test_tensor_layout(ref, off):
    L = ref
    ctx = L.ggml_init(InitParams(16 << 20, None, False))
    a = L.ggml_new_tensor_2d(ctx, 0, 48, 5)            # F32 [48, 5]
    b = L.ggml_new_tensor_2d(ctx, 0, 48, 5)
    c = L.ggml_add(ctx, a, b)
    s = L.ggml_scale(ctx, a, 0.75)
    v = L.ggml_view_1d(ctx, a, 16, 64)
    L.ggml_set_name(a, b"tensor-a")
    L.ggml_set_input(a)
    o = lambda m: off["kggml_tensor." + m]
    assert rd(a + o("type"), "i")[0] == 0
    assert rd(a + o("ne"), "4q") == (48, 5, 1, 1)
    assert rd(a + o("nb"), "4Q") == (4, 192, 960, 960)
    assert rd(c + o("op"), "i")[0] == 2                 # GGML_OP_ADD
    assert rd(s + o("op"), "i")[0] == 29                # GGML_OP_SCALE
    assert rd(s + o("op_params"), "f")[0] == 0.75
    assert rd(a + o("flags"), "i")[0] & 1               # GGML_TENSOR_FLAG_INPUT
    assert rd_ptr(c + o("src")) == a and rd_ptr(c + o("src") + 8) == b
    assert rd_ptr(v + o("view_src")) == a and rd(v + o("view_offs"), "Q")[0] == 64
    assert rd_ptr(a + o("data")) == L.ggml_get_data(a)
    assert ctypes.string_at(a + o("name")).decode() == "tensor-a"
    assert off["kggml_tensor.sizeof"] == L.ggml_tensor_overhead() - 32   # GGML_OBJECT_SIZE = 32 (ggml.c)
    L.ggml_free(ctx)


def test_cgraph_layout(ref, off):
    L = ref
    ctx = L.ggml_init(InitParams(32 << 20, None, False))
    a = L.ggml_new_tensor_2d(ctx, 0, 8, 2)
    b = L.ggml_new_tensor_2d(ctx, 0, 8, 2)
    t = L.ggml_scale(ctx, L.ggml_add(ctx, a, b), 2.0)
    g = L.ggml_new_graph(ctx)
    L.ggml_build_forward_expand(g, t)
    o = lambda m: off["kggml_cgraph." + m]
    n = L.ggml_graph_n_nodes(g)
    assert n == 2
    assert rd(g + o("size"), "i")[0] == L.ggml_graph_size(g)
    assert rd(g + o("n_nodes"), "i")[0] == n
    nodes = rd_ptr(g + o("nodes"))
    assert [rd_ptr(nodes + 8 * i) for i in range(n)] == [L.ggml_graph_node(g, i) for i in range(n)]
    assert rd(g + o("n_leafs"), "i")[0] == 2
    L.ggml_free(ctx)


def test_backend_vtables_layout(ref, off):
    """the CPU backend's objects, walked through our struct offsets and called through our vtable slots"""
    L = ref
    P = ctypes.c_void_p
    be = L.ggml_backend_cpu_init()
    bi = off["kggml_backend.iface"]
    get_name = fnptr(be + bi + off["kggml_backend_i.get_name"], ctypes.c_char_p, P)
    assert get_name(be) == L.ggml_backend_name(be) == b"CPU"
    dev = rd_ptr(be + off["kggml_backend.device"])
    assert dev == L.ggml_backend_get_device(be)
    di = off["kggml_backend_device.iface"]
    assert fnptr(dev + di + off["kggml_backend_device_i.get_name"], ctypes.c_char_p, P)(dev) == L.ggml_backend_dev_name(dev)
    assert fnptr(dev + di + off["kggml_backend_device_i.get_type"], ctypes.c_int, P)(dev) == 2     # CPU_FULL
    reg = rd_ptr(dev + off["kggml_backend_device.reg"])
    assert reg == L.ggml_backend_dev_backend_reg(dev)
    ri = off["kggml_backend_reg.iface"]
    assert fnptr(reg + ri + off["kggml_backend_reg_i.get_name"], ctypes.c_char_p, P)(reg) == L.ggml_backend_reg_name(reg)
    assert fnptr(reg + ri + off["kggml_backend_reg_i.get_device_count"], ctypes.c_size_t, P)(reg) == L.ggml_backend_reg_dev_count(reg)
    assert fnptr(reg + ri + off["kggml_backend_reg_i.get_device"], P, P, ctypes.c_size_t)(reg, 0) == dev
    buft = L.ggml_backend_cpu_buffer_type()
    assert rd_ptr(buft + off["kggml_backend_buffer_type.device"]) == dev
    ti = off["kggml_backend_buffer_type.iface"]
    assert fnptr(buft + ti + off["kggml_backend_buffer_type_i.get_name"], ctypes.c_char_p, P)(buft) == L.ggml_backend_buft_name(buft)
    assert fnptr(buft + ti + off["kggml_backend_buffer_type_i.get_alignment"], ctypes.c_size_t, P)(buft) == \
        L.ggml_backend_buft_get_alignment(buft)
    assert fnptr(buft + ti + off["kggml_backend_buffer_type_i.is_host"], ctypes.c_bool, P)(buft)
    buf = L.ggml_backend_buft_alloc_buffer(buft, 4096)
    assert rd_ptr(buf + off["kggml_backend_buffer.buft"]) == buft
    assert rd(buf + off["kggml_backend_buffer.size"], "Q")[0] == L.ggml_backend_buffer_get_size(buf) >= 4096
    L.ggml_backend_buffer_set_usage(buf, 1)
    assert rd(buf + off["kggml_backend_buffer.usage"], "i")[0] == 1
    gi = off["kggml_backend_buffer.iface"]
    assert fnptr(buf + gi + off["kggml_backend_buffer_i.get_base"], P, P)(buf) == L.ggml_backend_buffer_get_base(buf)
    assert rd_ptr(buf + gi + off["kggml_backend_buffer_i.free_buffer"]) != 0
    L.ggml_backend_buffer_free(buf)
    # struct sizes: the vtables are arrays of pointers of the reference's member counts
    assert off["kggml_backend_i.sizeof"] == 17 * 8 and off["kggml_backend_device_i.sizeof"] == 15 * 8
    assert off["kggml_backend_buffer_i.sizeof"] == 10 * 8 and off["kggml_backend_buffer_type_i.sizeof"] == 6 * 8
    assert off["kggml_backend_reg_i.sizeof"] == 4 * 8
    L.ggml_backend_free(be)
