"""koboldcpp_amd -- MI355X-native (gfx950) ggml backend for koboldcpp's llama.cpp token-generation path.

The product is the C-ABI shared library ``koboldcpp_amd/koboldcpp_hipblas.so`` (hand-written HIP
kernels + C++ runtime); this package only holds its ctypes binding (``lib``) for tests, the
benchmark and Python callers.  There is no CPU fallback: if the library is missing, importing
``koboldcpp_amd.lib`` raises.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KCPP_LIB") or os.path.join(PKG_DIR, "koboldcpp_hipblas.so")   # KCPP_LIB: A/B builds
