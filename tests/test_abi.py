"""CPU-side checks of the drop-in boundary: the native library loads and exports every symbol the
public headers declare (no compute calls -- there is no GPU here)."""
import glob
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "koboldcpp_amd", "koboldcpp_hipblas.so")


def declared(header):
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\((?!\s*\*)", txt))   # not "type (*member)(...)"
    keywords = {"if", "for", "while", "return", "sizeof", "defined"}
    return {n for n in names if n not in keywords and not n.startswith("__")}


def exported():
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    ex = exported()
    for h in glob.glob(os.path.join(ROOT, "include", "kcpp_*.h")):
        if h.endswith("kcpp_synth.h"):
            continue  # header-only inline helpers
        missing = sorted(n for n in declared(h) if n not in ex)
        assert not missing, (os.path.basename(h), missing)


def test_python_binding_loads():
    import koboldcpp_amd.lib as K
    assert K.act_bytes(K.Q4_K, 4096, 1) == 4096 + 16 * 4 + 256 * 2
    assert K.vec_dot_type(K.Q4_0) == K.Q8_0 and K.vec_dot_type(K.Q6_K) == K.Q8_K
