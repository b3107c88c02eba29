"""Row split (koboldcpp --rowsplit, LLAMA_SPLIT_MODE_ROW): the per-device row ranges of kcpp_row_split_range vs a
restatement of the reference's rule -- tensor_split normalized to cumulative starts
(ggml_backend_cuda_split_buffer_type, ggml/src/ggml-cuda.cu:918-938; all zero: equal shares, the default split of
identical GPUs), bounds from float32 nrows * start truncated and rounded down to the MMQ tile height (128 rows on
AMD, get_mmq_y_host mmq.cuh:123, get_row_rounding ggml-cuda.cu:625-636) unless they reach nrows
(ggml_cuda_op_mul_mat, ggml-cuda.cu:1445-1463).  Host only."""
import numpy as np
import pytest


def ref_ranges(nrows, ts):
    n = len(ts)
    f = np.float32
    zero = all(v == 0 for v in ts)
    start, acc = [], f(0)
    for v in ts:
        start.append(acc)
        acc = f(acc + f(1.0 if zero else v))
    start = [f(s / acc) for s in start]
    out = []
    for i in range(n):
        lo, hi = 0, nrows
        if i != 0:
            lo = int(f(nrows) * start[i])
            if lo < nrows:
                lo -= lo % 128
        if i != n - 1:
            hi = int(f(nrows) * start[i + 1])
            if hi < nrows:
                hi -= hi % 128
        out.append((lo, hi))
    return out


@pytest.fixture(scope="module")
def K():
    import koboldcpp_amd.lib as K
    return K


SPLITS = [(1.0,), (1.0, 1.0), (0.5, 0.3, 0.2), (3.0, 1.0), (0.0, 0.0, 0.0, 0.0), (1.0, 0.0, 1.0), (0.0, 1.0),
          (1.0,) * 8, (7.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0)]
NROWS = [128, 512, 1000, 1024, 4096, 14336, 28672, 32000, 128256, 100]


@pytest.mark.parametrize("ts", SPLITS)
def test_row_ranges_match_reference_rule(K, ts):
    for nrows in NROWS:
        want = ref_ranges(nrows, ts)
        got = [K.row_split_range(nrows, ts, i) for i in range(len(ts))]
        assert got == want, (nrows, ts, got, want)
        # the ranges tile [0, nrows) in device order; every inner bound is a multiple of 128
        assert got[0][0] == 0 and got[-1][1] == nrows
        for (a, b), (c, d) in zip(got, got[1:]):
            assert b == c and a <= b
        for lo, hi in got:
            assert lo % 128 == 0 or lo == nrows


def test_row_ranges_bad_args(K):
    from koboldcpp_amd.lib import KcppError
    with pytest.raises(KcppError):
        K.row_split_range(128, (1.0, 1.0), 2)
