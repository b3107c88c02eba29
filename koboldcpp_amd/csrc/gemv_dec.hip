// gemv_dec.hip -- C entry of the fused single-token mat-vec (gemv_dec_impl.h, one TU per type).
#include "kcpp_internal.h"
#include "kcpp_common.h"

#include <cstdlib>

template <int TYPE> int dispatch_mode(const DecArgs &a, int mode, int pro, int rows_per_wave, hipStream_t s);

extern "C" int kcpp_gemv_dec(int type, const void *args, int mode, int pro, int rows_per_wave, void *stream) {
    const DecArgs &a = *(const DecArgs *)args;
    hipStream_t s = (hipStream_t)stream;
    // row-major decode layouts: only the RS kernels read them (gemv_rs.hip)
    if (type == KT_Q4_K_RS || type == KT_Q5_K_RS || type == KT_Q6_K_RS) return kcpp_gemv_rs(type, args, mode, pro, stream);
    // coalesced-streaming kernel where it covers the type/shape (gemv_stream.hip), else unit-per-lane
    if (type == KT_Q4_K) {
        const int rc = kcpp_gemv_q4k(args, mode, pro, stream);
        if (rc != -3) return rc;
    }
    {
        const int rc = kcpp_gemv_stream(type, args, mode, pro, stream);
        if (rc != -3) return rc;
    }
    switch (type) {
    case KT_Q4_K: return dispatch_mode<KT_Q4_K>(a, mode, pro, rows_per_wave, s);
    case KT_Q5_K: return dispatch_mode<KT_Q5_K>(a, mode, pro, rows_per_wave, s);
    case KT_Q6_K: return dispatch_mode<KT_Q6_K>(a, mode, pro, rows_per_wave, s);
    case KT_Q3_K: return dispatch_mode<KT_Q3_K>(a, mode, pro, rows_per_wave, s);
    case KT_Q2_K: return dispatch_mode<KT_Q2_K>(a, mode, pro, rows_per_wave, s);
    case KT_Q4_0: return dispatch_mode<KT_Q4_0>(a, mode, pro, rows_per_wave, s);
    case KT_Q5_0: return dispatch_mode<KT_Q5_0>(a, mode, pro, rows_per_wave, s);
    case KT_Q8_0: return dispatch_mode<KT_Q8_0>(a, mode, pro, rows_per_wave, s);
    case KT_IQ4_NL: return dispatch_mode<KT_IQ4_NL>(a, mode, pro, rows_per_wave, s);
    case KT_IQ4_XS: return dispatch_mode<KT_IQ4_XS>(a, mode, pro, rows_per_wave, s);
    case KT_IQ2_XXS: return dispatch_mode<KT_IQ2_XXS>(a, mode, pro, rows_per_wave, s);
    case KT_IQ2_XS: return dispatch_mode<KT_IQ2_XS>(a, mode, pro, rows_per_wave, s);
    case KT_IQ2_S: return dispatch_mode<KT_IQ2_S>(a, mode, pro, rows_per_wave, s);
    case KT_IQ3_XXS: return dispatch_mode<KT_IQ3_XXS>(a, mode, pro, rows_per_wave, s);
    case KT_IQ3_S: return dispatch_mode<KT_IQ3_S>(a, mode, pro, rows_per_wave, s);
    case KT_IQ1_S: return dispatch_mode<KT_IQ1_S>(a, mode, pro, rows_per_wave, s);
    case KT_IQ1_M: return dispatch_mode<KT_IQ1_M>(a, mode, pro, rows_per_wave, s);
    default: return -3;
    }
}

extern "C" int64_t kcpp_gemv_dec_args_size(void) { return (int64_t)sizeof(DecArgs); }
