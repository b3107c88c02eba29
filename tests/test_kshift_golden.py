"""CPU check of the context shift's rotation against the reference (no GPU): the runtime's (cos, sin) row for
position -diff (kcpp_rope_row, host code of the library; ggml_rope_cache_init's values) applied as rope_f16 does
(f32 products, f16 result) reproduces the reference build_k_shift output of tests/golden/kshift.npz bit for bit."""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("base", [10000, 500000])
@pytest.mark.parametrize("diff", [1, 37, 1000])
def test_rope_row_reproduces_reference_k_shift(base, diff):
    import koboldcpp_amd.lib as K
    fx = np.load(os.path.join(HERE, "golden", "kshift.npz"))
    k = fx["k_in"].view(np.float16)
    D = k.shape[-1]
    row = np.zeros(D, np.float32)
    K.call("kcpp_rope_row", row.ctypes.data, -diff, D, float(base), 1.0, 0.0, 1.0, 32.0, 1.0, 4096)
    c, s = row[0::2], row[1::2]
    x0, x1 = k[..., 0::2].astype(np.float32), k[..., 1::2].astype(np.float32)
    want = np.empty_like(k)
    want[..., 0::2] = (x0 * c - x1 * s).astype(np.float16)
    want[..., 1::2] = (x0 * s + x1 * c).astype(np.float16)
    assert np.array_equal(want.view(np.uint16), fx["k_shift_%d_%d" % (base, diff)])
