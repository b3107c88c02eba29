"""koboldcpp's automatic RoPE base (CalcGradientAIRopeFreqBase, gpttype_adapter.cpp:1598-1640) restated in the
drop-in (kcpp_gradient_ai_rope_base, used by load_model when the user gives no --ropeconfig and the model sets no
RoPE of its own), against the reference function itself: oracle/_ref/ref_sampler compiles gpttype_adapter.cpp as its
one translation unit and evaluates the static function in its "rope" mode.  Float results must be equal (the same
float log10f / powf sequence); cases cover contexts at / below the trained one and the 2048 floor (unchanged base),
Llama-3 (base 500000), Llama-2 (10000) and the SOLAR rule (context x 8 plus the positive offset)."""
import os
import subprocess

import numpy as np
import pytest

import refharness as R

SAMPLER = os.path.join(R.ROOT, "oracle", "_ref", "ref_sampler")
CASES = [(500000.0, 8192, 4096, 0), (500000.0, 8192, 8192, 0), (500000.0, 8192, 8200, 0), (500000.0, 8192, 16384, 0),
         (500000.0, 8192, 131072, 0), (10000.0, 4096, 16384, 0), (10000.0, 2048, 2048, 0), (10000.0, 1024, 2000, 0),
         (10000.0, 2048, 4096, 0), (10000.0, 4096, 8192, 1), (10000.0, 4096, 32768, 1), (1000000.0, 32768, 65536, 0),
         (500000.0, 1024, 3000, 0)]


def test_gradient_ai_rope_base_matches_reference():
    if not os.path.exists(SAMPLER):
        pytest.skip("reference harness not built (make -C oracle ref)")
    import koboldcpp_amd.lib as K
    inp = "\n".join("%r %d %d %d" % c for c in CASES) + "\n"
    r = subprocess.run([SAMPLER, "rope"], input=inp, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    want = [np.float32(float(v)) for v in r.stdout.split()]
    assert len(want) == len(CASES)
    for c, w in zip(CASES, want):
        got = np.float32(K._L.kcpp_gradient_ai_rope_base(*c))
        assert got == w, (c, got, w)
    # the auto scaling does change the base beyond the trained context, and leaves it alone within it
    assert want[3] > 500000.0 * 1.5 and want[0] == np.float32(500000.0) and want[6] == np.float32(10000.0)
